"""Microbenchmark driver for counter passes: 40 eager fused rollout steps (mm_rollout_step, 4096 envs x 8
agents, GRU-64, PER 65536 chunks) after 20 warm-up steps. Prints the fused flag and the step count."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402
from minimarl.engine import RolloutEngine  # noqa: E402

eng = RolloutEngine(4096, 8, f1=64, g=64, h=64, chunk=10, capacity=65536, seed=1, device="cuda")
for _ in range(60):
    eng.step(0.1)
torch.cuda.synchronize()
print(json.dumps({"fused": eng.fused, "steps": eng.t}))
