"""Fixed cost of a timed bench region: the driver runs ``bench.py --steps 20 --warmup 5``,
so every timed region is 20 lockstep steps bracketed by synchronize. This probe builds the bench's rollout
engine (4096 x 8, PER pre-filled), then times R regions of K steps the way bench.py does and prints, per
region, the host wall time and CLOCK_MONOTONIC / CLOCK_BOOTTIME stamps of t0 / t1, so a rocprofv3
--kernel-trace of the same run can place the region's first and last kernel inside it (t0 -> first kernel,
last kernel -> synchronize return). Variant ``MB_MODE=region`` replays one captured K-step graph instead.
Prints one JSON line per mode to stdout."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-marl_amd"))
if os.environ.get("MB_SPIN") == "1":
    # hipDeviceScheduleSpin before the runtime creates its context: synchronize spin-waits for completion
    import ctypes
    _hip = ctypes.CDLL("libamdhip64.so")
    assert _hip.hipSetDeviceFlags(ctypes.c_uint(1)) == 0
import torch  # noqa: E402
from minimarl.engine import RolloutEngine  # noqa: E402

E, N, K, R, W = 4096, 8, int(os.environ.get("MB_K", 20)), int(os.environ.get("MB_R", 10)), 5
modes = os.environ.get("MB_MODES", "steps").split(",")


def stamp():
    return {"mono": time.clock_gettime_ns(time.CLOCK_MONOTONIC), "boot": time.clock_gettime_ns(time.CLOCK_BOOTTIME)}


eng = RolloutEngine(E, N, f1=64, g=64, h=64, chunk=10, capacity=16 * E, seed=1234)
for _ in range(16):
    eng.run_graph(0.1)
eng.capture_steps()
eng.run_steps(W, 0.1)
for mode in modes:
    regs = []
    if mode == "region":
        eng.capture_region(K)
    for _ in range(R):
        torch.cuda.synchronize()
        torch.cuda.synchronize()
        a = stamp()
        t0 = time.perf_counter()
        if mode == "region":
            eng.run_region(K)
        else:
            eng.run_steps(K, 0.1)
        t_sub = time.perf_counter()
        torch.cuda.synchronize()
        t_s1 = time.perf_counter()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        b = stamp()
        regs.append({"ms": el * 1e3, "submit_ms": (t_sub - t0) * 1e3, "sync1_ms": (t_s1 - t_sub) * 1e3,
                     "t0": a, "t1": b})
    ms = sorted(r["ms"] for r in regs)
    print(json.dumps({"mode": mode, "K": K, "median_ms_per_step": ms[len(ms) // 2] / K, "regions": regs}), flush=True)
