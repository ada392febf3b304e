"""Per-phase clock64 trace of the gate-parallel REC sequence kernel inside one B=32 QMIX update.

Run with MM_REC_TRACE=1 (the kernel then stamps block 0: wave 0 = gate wave g0/hb0, and the Q wave).
Per step: [0] top, [1] after MFMA chain, [2] after barrier A, [3] gates done, [4] after barrier B,
Q wave: [5] after barrier B, [6] after Q MFMA, [7] after epilogue.
"""
import ctypes
import json
import os
import sys

os.environ.setdefault("MM_REC_TRACE", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
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
lib = _lib.lib()
torch.cuda.synchronize()

assert lib.mm_debug_trace(ctypes.addressof(buf), 4096) == 0
t = list(buf)
base = t[3]
out = {"prologue": t[0] - base, "gate_wave_total": t[1] - base, "q_wave_total": t[2] - base, "steps": []}
for s in range(C):
    r = t[4 + 8 * s: 12 + 8 * s]
    out["steps"].append({"mfma": r[1] - r[0], "barA": r[2] - r[1], "gates": r[3] - r[2], "barB": r[4] - r[3],
                         "q_wait": r[5] - (t[4 + 8 * (s - 1) + 7] if s else t[0]), "q_mfma": r[6] - r[5],
                         "q_epi": r[7] - r[6], "gate_step": (t[4 + 8 * (s + 1)] if s + 1 < C else t[1]) - r[0]})
print(json.dumps(out))
