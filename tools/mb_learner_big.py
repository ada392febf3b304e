"""Microbenchmark: QMIX learner update at the throughput batch of SURVEY 8(d) (B = 4096 chunks,
C = 10, GRU-64 agents, Hm = 64 mixer) from a device PER filled by the rollout engine.
Usage: python tools/mb_learner_big.py [B]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402
from minimarl.engine import RolloutEngine  # noqa: E402
from minimarl.learner import Mixer, QLearner  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
E, N = 4096, 8
eng = RolloutEngine(E, N, f1=64, g=64, h=64, chunk=10, capacity=4 * E, seed=1, device="cuda")
for _ in range(4):
    eng.run_graph(0.1)
mix, tmix = Mixer(N, N * eng.D, 64, 32, "cuda", seed=7), Mixer(N, N * eng.D, 64, 32, "cuda", seed=7)
L = QLearner(eng.behavior, eng.target, mix, tmix, batch=B, chunk=10, mode="qmix", device="cuda")
L.capture_update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=3)
for _ in range(3):
    L.replay_update()
torch.cuda.synchronize()
a, b = torch.cuda.Event(True), torch.cuda.Event(True)
it = 10
a.record()
for _ in range(it):
    L.replay_update()
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / it
flop = B * 10 * (4 * N * 2 * (47 * 64 + 64 * 64 + 6 * 64 * 64 + 64 * 5) + 4 * 2 * (N * 47 * 3 * 64 + 3 * 64 * 64))
print(json.dumps({"B": B, "C": 10, "ms_per_update": round(ms, 3), "updates_per_s": round(1e3 / ms, 1),
                  "chunk_samples_per_s": round(B * 1e3 / ms, 1), "approx_tflops": round(flop / ms / 1e9, 2),
                  "loss": float(L.loss.item())}))
