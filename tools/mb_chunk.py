"""A/B microbenchmark of the rollout step modes at the headline shape (4096 envs x 8 agents, GRU-64, PER 65536
chunks pre-filled so every insert evicts): ms per step of 20-step region graphs (the bench's timed region) from a
chunk boundary and from mid-chunk, per mode; plus the chunk kernel alone (C steps per launch) and the fused step
alone, event-timed. GPU only. usage: python tools/mb_chunk.py [modes...]  (modes: chunk fused)"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402
import minimarl._lib as _L  # noqa: E402
from minimarl.engine import RolloutEngine  # noqa: E402

# A/B: MB_LIB = another build of libminimarl.so; MB_HOLD=neh = hidden states stored [N][E][H] (feature-contiguous)
if os.environ.get("MB_LIB"):
    _L.LIB_PATH = os.path.abspath(os.environ["MB_LIB"])

E, N, C, CAP = 4096, 8, 10, 65536
modes = sys.argv[1:] or ["chunk", "fused"]


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


out = {}
for mode in modes:
    kw = dict(persistent=True) if mode == "chunk" else dict(fused=True)
    eng = RolloutEngine(E, N, f1=64, g=64, h=64, chunk=C, capacity=CAP, seed=1, device="cuda", **kw)
    if os.environ.get("MB_HOLD") == "neh":   # feature-contiguous hidden-state storage
        eng.h = torch.zeros(N, E, 64, device="cuda").permute(0, 2, 1)
        eng.ht = torch.zeros(N, E, 64, device="cuda").permute(0, 2, 1)
        eng._build_io()
    while len(eng.per) < CAP:
        eng.run_steps(eng.graph_steps(), 0.5)
    res = {}
    for start in (0, 5):
        while eng.t % eng.graph_steps() != start:
            eng.step(0.1)
        eng.capture_region(20)
        for _ in range(3):
            eng.run_region(20, 0.1)
        ms = []
        for _ in range(10):
            ms.append(timed(lambda: eng.run_region(20, 0.1), 1) / 20)
        ms.sort()
        res[f"region20_phase{start}_ms_per_step"] = {"median": ms[5], "min": ms[0], "max": ms[-1]}
    if mode == "chunk":
        res["chunk_kernel_10steps_us"] = 1000 * timed(lambda: eng.chunk_only(C), 20)
        res["chunk_kernel_1step_us"] = 1000 * timed(lambda: eng.chunk_only(1), 20)
        eng.check_errors()
    else:
        res["fused_step_kernel_us"] = 1000 * timed(lambda: eng.fused_step_only(1), 20)
    # digest of the final state (A/B builds that claim identical arithmetic must agree on it)
    import hashlib
    hs = hashlib.sha1()
    for tsr in (eng.h, eng.ht, eng.store.obs, eng.store.act, eng.chunk_td, eng.per.tree()):
        hs.update(tsr.contiguous().cpu().numpy().tobytes())
    res["state_sha1"] = hs.hexdigest()[:16]
    out[mode] = res
    del eng
    torch.cuda.empty_cache()
out["lib"] = _L.LIB_PATH
out["hold"] = os.environ.get("MB_HOLD", "0")
print(json.dumps(out))
