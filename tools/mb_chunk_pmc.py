"""Eager chunk-kernel launches for counter runs (tools/pmc_chunk.sh): the headline shape (4096 envs x 8 agents,
GRU-64, chunk 10), 3 warm-up launches, then 10 launches of 20 steps (the bench region's launch). GPU only."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402
from minimarl.engine import RolloutEngine  # noqa: E402

E, N, C = 4096, 8, 10
eng = RolloutEngine(E, N, f1=64, g=64, h=64, chunk=C, capacity=4 * E, seed=1, device="cuda", persistent=True)
for _ in range(13):
    eng.chunk_only(2 * C)
torch.cuda.synchronize()
eng.check_errors()
print("ok")
