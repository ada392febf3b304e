"""Per-block timeline of ONE fused rollout-step launch (MM_ROLL_TRACE stamps, csrc/agent_fwd.hip MM_RSTAMP):
0 start (after the first kernarg-dependent load), 1 env inputs staged (wave 0), 2 kernel entry (first instruction), 3 env step done (wave 0), 4 after the second
barrier, 5 obs k-step 0 built, 6 / 7 body end of waves 0 / 15. Prints, per stamp, min / median / max over blocks in us from the earliest start. GPU only."""
import ctypes
import os
import sys

import numpy as np
import torch

os.environ["MM_ROLL_TRACE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mini-marl_amd")]
from minimarl._lib import lib  # noqa: E402
from minimarl.engine import RolloutEngine  # noqa: E402

E = int(os.environ.get("MB_E", "4096"))
assert lib().mm_debug_trace(None, 0) == 0
eng = RolloutEngine(E, 8, f1=64, g=64, h=64, chunk=10, capacity=4 * E, seed=1, device="cuda")
for _ in range(41):
    eng.step(0.1)
for rep in range(3):
    torch.cuda.synchronize()
    eng.fused_step_only()
    torch.cuda.synchronize()
    buf = np.zeros(4096, np.uint64)
    assert lib().mm_debug_trace(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 4096) == 0
    nb = 2 * (E // 256) * 8
    tr = buf[: 8 * nb].reshape(nb, 8).astype(np.int64)
    t0 = tr[:, 0].min()
    rel = (tr - t0) * 0.01
    print(f"rep {rep}: blocks {nb}")
    for i, name in enumerate(["start", "env staged", "entry", "env done", "barrier B", "obs ks0", "end w0", "end w15"]):
        col = rel[:, i]
        print(f"  {i} {name:11s} min {col.min():6.2f} med {np.median(col):6.2f} max {col.max():6.2f}  "
              f"(target med {np.median(col[: nb // 2]):6.2f}, behavior med {np.median(col[nb // 2:]):6.2f})")
