"""Diagnostic: does mm_hold_cus keep chunk-kernel blocks off the CUs it holds? Event timeline of a holder on a side
stream and a 3-step chunk launch on the main stream (tests/test_gpu_chunk.py co-residency test)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402

from minimarl._lib import check, lib  # noqa: E402
from minimarl.engine import RolloutEngine  # noqa: E402
from minimarl.qnet import ptr  # noqa: E402

cus = torch.cuda.get_device_properties(0).multi_processor_count
print("cus", cus)
e = RolloutEngine(4096, 8, f1=64, g=64, h=64, chunk=10, capacity=4 * 4096, seed=3, persistent=True, device="cuda")
e.step(0.3)
torch.cuda.synchronize()
side = torch.cuda.Stream()
seen = torch.zeros(1, dtype=torch.int32, device="cuda")
check(lib().mm_hold_cus(1, 0, ptr(e.hx), 0, 0, ptr(seen), side.cuda_stream), "hold")
torch.cuda.synchronize()
for nblk in (192, 224, 240, 252, 255, 160):
    seen.zero_()
    e.err.zero_()
    seq = int(e.ctl[0].item())
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record(side)
    check(lib().mm_hold_cus(nblk, 10_000_000, ptr(e.hx), e.hx.numel(), (seq + 1) & 0xFFFFFFFF, ptr(seen),
                            side.cuda_stream), "hold")
    ev[1].record(side)
    time.sleep(0.02)
    ev[2].record()
    e.chunk_only(3)
    ev[3].record()
    torch.cuda.synchronize()
    print(f"holder blocks {nblk}: holder {ev[0].elapsed_time(ev[1]):.2f} ms, chunk start {ev[0].elapsed_time(ev[2]):.2f}"
          f" end {ev[0].elapsed_time(ev[3]):.2f} ms (chunk {ev[2].elapsed_time(ev[3]):.2f} ms), seen {int(seen.item())},"
          f" err {int(e.err.item())}", flush=True)

# two chunk-persistent launches on two streams at once (two engines): each needs every CU
print(torch.cuda.get_device_properties(0))
f = RolloutEngine(4096, 8, f1=64, g=64, h=64, chunk=10, capacity=4 * 4096, seed=4, persistent=True, device="cuda")
f.step(0.3)
torch.cuda.synchronize()
for rep in range(3):
    e.err.zero_()
    f.err.zero_()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record(side)
    with torch.cuda.stream(side):
        f.chunk_only(3)
    ev[1].record(side)
    ev[2].record()
    e.chunk_only(3)
    ev[3].record()
    torch.cuda.synchronize()
    print(f"two chunk launches: side {ev[0].elapsed_time(ev[1]):.2f} ms, main start {ev[0].elapsed_time(ev[2]):.3f} "
          f"end {ev[0].elapsed_time(ev[3]):.2f} ms, err main {int(e.err.item())} side {int(f.err.item())}", flush=True)
