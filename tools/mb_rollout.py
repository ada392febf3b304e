"""Microbenchmark of the fused rollout step launch (mm_rollout_step) at the bench shape (4096 envs x 8
agents, D=47, 64/64/64, A=5) beside the unfused dual forward; MM_LIB picks an A/B library build.
Prints one JSON line (microseconds per launch)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402
from minimarl.engine import RolloutEngine  # noqa: E402

E = int(os.environ.get("MB_E", 4096))


def timeit(fn, it=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


out = {"lib": os.path.basename(os.environ.get("MM_LIB", "libminimarl.so")), "E": E}
a = RolloutEngine(E, 8, f1=64, g=64, h=64, chunk=10, capacity=4 * E, seed=1, fused=True)
for _ in range(12):
    a.step(0.1)
out["fused_step_us"] = timeit(a.fused_forward)
if os.environ.get("MB_UNFUSED", "1") == "1":
    b = RolloutEngine(E, 8, f1=64, g=64, h=64, chunk=10, capacity=4 * E, seed=1, fused=False)
    for _ in range(12):
        b.step(0.1)
    out["dual_fwd_us"] = timeit(b.fused_forward)
print(json.dumps(out))
