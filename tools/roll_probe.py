"""Time the fused rollout-step launch (and the two-launch step's kernels) at the headline shape; run with
MM_LIB=<probe build> to decompose the fused kernel (csrc/agent_fwd.hip MM_ROLL_PROBE). GPU only."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mini-marl_amd")]
from bench import time_kernel  # noqa: E402
from minimarl.engine import RolloutEngine  # noqa: E402

E = int(os.environ.get("MB_E", "4096"))
eng = RolloutEngine(E, 8, f1=64, g=64, h=64, chunk=10, capacity=4 * E, seed=1, device="cuda")
assert eng.fused
for _ in range(40):
    eng.step(0.1)
torch.cuda.synchronize()
out = {"lib": os.path.basename(os.environ.get("MM_LIB", "default")),
       "fused_us": round(time_kernel(eng.fused_step_only) * 1e6, 2),
       "dual_fwd_us": round(time_kernel(eng.fused_forward) * 1e6, 2),
       "env_us": round(time_kernel(eng.env_only) * 1e6, 2)}
print(json.dumps(out), flush=True)
