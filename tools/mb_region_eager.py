"""The bench's rollout region (4096 envs x 8 agents, GRU-64, chunk 10, PER full) launched eagerly, 20 steps at a
time, for a kernel timeline under `rocprofv3 --kernel-trace` (graph-replayed kernels carry no usable per-kernel
timestamps): where a driver-timed step goes outside the chunk-persistent kernel. Prints the region's event time.

usage: rocprofv3 --kernel-trace --output-format csv -d <dir> -- python3 tools/mb_region_eager.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mini-marl_amd"))
import torch  # noqa: E402

from minimarl.engine import RolloutEngine  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    E, N = 4096, 8
    eng = RolloutEngine(E, N, f1=64, g=64, h=64, chunk=10, capacity=16 * E, seed=1234, device=dev)
    eng.set_epsilon(0.1)
    eng._advance(16 * 10 + 20)
    torch.cuda.synchronize()
    ts = []
    for _ in range(8):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng._advance(20)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    eng.check_errors()
    # the same region as one captured graph (bench.py's timed form), both graph phases
    G = eng.graph_steps()
    for i in range(G // 20):
        eng.capture_region(20, start=eng.t + 20 * i)
    tg = []
    for _ in range(8):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.run_steps(20)
        torch.cuda.synchronize()
        tg.append(time.perf_counter() - t0)
    eng.check_errors()
    # the chunk launch alone (20 steps from a ring cycle start, no fold / insert), event-timed like bench.py's roofline
    ev0, ev1 = torch.cuda.Event(True), torch.cuda.Event(True)
    tc = []
    for _ in range(8):
        ev0.record()
        eng.chunk_only(20)
        ev1.record()
        torch.cuda.synchronize()
        tc.append(ev0.elapsed_time(ev1))
    # an empty graph region: launch + synchronize cost alone
    g = torch.cuda.CUDAGraph()
    s_ = torch.cuda.Stream()
    x = torch.zeros(1, device=dev)
    with torch.cuda.stream(s_):
        g.capture_begin()
        x.add_(1)
        g.capture_end()
    te = []
    for _ in range(8):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        te.append(time.perf_counter() - t0)
    print({"chunk_only20_ms_min": round(min(tc), 4), "tiny_graph_ms_min": round(min(te) * 1e3, 4)})
    print({"eager_region_ms_min": round(min(ts) * 1e3, 4), "graph_region_ms_min": round(min(tg) * 1e3, 4),
           "eager_ms": [round(x * 1e3, 3) for x in ts], "graph_ms": [round(x * 1e3, 3) for x in tg], "steps": 20})


if __name__ == "__main__":
    main()
