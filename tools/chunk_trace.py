"""Per-step timeline of ONE chunk-persistent launch (10 steps, 4096 envs x 8 agents), from the MM_ROLL_DEBUG build's
s_memrealtime stamps (csrc/agent_fwd.hip MM_CSTAMP, 100 MHz) of waves 0 and 15 of every block: per step 0 loop top,
1 hand-off flags seen, 2 dynamics done, 3 forward done. Prints the medians over behavior blocks of each phase per
step and the per-step period, in us, and the in-kernel shader clock (s_memtime / s_memrealtime around each block's
step loop, after ~0.5 s of back-to-back launches: MI355X_MICROARCH.md DVFS check). GPU only; needs
`make -C mini-marl_amd debug`."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

os.environ["MM_ROLL_TRACE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mini-marl_amd")]
import minimarl._lib as L  # noqa: E402

L.LIB_PATH = os.path.join(ROOT, "mini-marl_amd", "lib_dbg", "libminimarl.so")
from minimarl.engine import RolloutEngine  # noqa: E402

E, N, C = 4096, 8, 10
assert L.lib().mm_debug_trace(None, 0) == 0
eng = RolloutEngine(E, N, f1=64, g=64, h=64, chunk=C, capacity=4 * E, seed=1, device="cuda", persistent=True)
for _ in range(3):
    eng.run_steps(20, 0.1)
out = {}
for _ in range(2000):                               # ~0.5 s of back-to-back launches before the stamped ones (DVFS)
    eng.chunk_only(C)
for rep in range(2):
    torch.cuda.synchronize()
    eng.chunk_only(C)
    torch.cuda.synchronize()
    buf = np.zeros(65536, np.uint64)
    assert L.lib().mm_debug_trace(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 65536) == 0
    nb = 2 * (E // 256) * N
    tr = buf[: nb * 2 * 16 * 4].reshape(nb, 2, 16, 4).astype(np.int64)[:, :, :C, :]
    t0 = tr[tr > 0].min()
    rel = np.where(tr > 0, (tr - t0) * 0.01, np.nan)
    beh = (np.arange(nb) % (2 * N)) >= N
    for wi, wname in ((0, "wave 0"), (1, "wave 15")):
        b = rel[beh, wi]                                    # [blocks, C, 4]
        per = np.nanmedian(np.diff(b[:, :, 0], axis=1), axis=0)
        wait = np.nanmedian(b[:, 1:, 1] - b[:, 1:, 0], axis=0)
        dyn = np.nanmedian(b[:, :, 2] - np.where(np.isnan(b[:, :, 1]), b[:, :, 0], b[:, :, 1]), axis=0)
        fwd = np.nanmedian(b[:, :, 3] - b[:, :, 2], axis=0)
        end = np.nanmax(rel[:, wi, C - 1, 3])
        print(f"rep {rep} behavior {wname}: period {np.round(per, 2).tolist()}\n  wait {np.round(wait, 2).tolist()}\n"
              f"  dyn {np.round(dyn, 2).tolist()}\n  fwd {np.round(fwd, 2).tolist()}  last end {end:.2f}")
        out[f"rep{rep}_{wname}"] = {"period": per.tolist(), "wait": wait.tolist(), "dyn": dyn.tolist(),
                                     "fwd": fwd.tolist()}
    # in-kernel clock: delta s_memtime / delta s_memrealtime x 100 MHz around every block's step loop
    ck = buf[60000:60000 + 4 * nb].reshape(nb, 4).astype(np.float64)
    ghz = (ck[:, 2] - ck[:, 0]) / np.maximum(ck[:, 3] - ck[:, 1], 1) * 0.1
    print(f"rep {rep} in-kernel clock GHz: median {np.median(ghz):.3f} min {ghz.min():.3f} max {ghz.max():.3f}")
    out[f"rep{rep}_clock_ghz_median"] = float(np.median(ghz))
print(json.dumps(out))
eng.check_errors()
