"""clock64 phase trace of one learner kernel inside a B=32 QMIX update (block 0).

usage: python tools/trace_lrn.py ENV_VAR   (MM_MIX_TRACE_FWD | MM_MIX_TRACE_BWD | MM_ABWD_TRACE | MM_REC_TRACE)
Prints the prologue slots [0..3] relative to slot 0 and, per step, the deltas between that step's 4 slots
(slot 4 + 4t + k; MM_REC_TRACE uses 8 per step: see tools/trace_rec.py).
"""
import json
import os
import sys

var = sys.argv[1]
os.environ[var] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import ctypes  # noqa: E402

import torch  # noqa: E402
from minimarl import _lib  # noqa: E402
from minimarl.engine import RolloutEngine  # noqa: E402
from minimarl.learner import Mixer, QLearner  # noqa: E402

E, N, C = 512, 8, 10
assert _lib.lib().mm_debug_trace(None, 0) == 0
eng = RolloutEngine(E, N, f1=64, g=64, h=64, chunk=C, capacity=4 * E, seed=1, device="cuda")
for _ in range(4):
    eng.run_graph(0.1)
mix, tmix = Mixer(N, N * eng.D, 64, 32, "cuda", seed=7), Mixer(N, N * eng.D, 64, 32, "cuda", seed=7)
L = QLearner(eng.behavior, eng.target, mix, tmix, batch=32, chunk=C, mode="qmix", device="cuda")
L.capture_update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=3)
for _ in range(3):
    L.replay_update()
torch.cuda.synchronize()
buf = (ctypes.c_uint64 * 4096)()
assert _lib.lib().mm_debug_trace(ctypes.addressof(buf), 4096) == 0
t = list(buf)
k = 4
out = {"var": var, "prologue": [int(t[i] - t[0]) if t[i] else None for i in range(8)],
       "sub": [int(t[i] - t[0]) if t[i] else None for i in range(100, 106)], "steps": []}
for s in range(C):
    r = t[4 + k * s: 4 + k * s + k]
    out["steps"].append([int(r[i + 1] - r[i]) if r[i + 1] and r[i] else None for i in range(k - 1)])
print(json.dumps(out))
