"""Microbenchmark: one QMIX learner update (B=32, C=10, GRU-64, Hm=64) from a filled device PER."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402
from minimarl.engine import RolloutEngine  # noqa: E402
from minimarl.learner import Mixer, QLearner  # noqa: E402

E, N = int(os.environ.get("MB_E", 512)), 8
CAP = int(os.environ.get("MB_CAP", 4 * E))     # bench: E = 4096, capacity 65536 chunks
eng = RolloutEngine(E, N, f1=64, g=64, h=64, chunk=10, capacity=CAP, seed=1, device="cuda")
for _ in range(max(4, CAP // E + 1)):
    eng.run_graph(0.1)
mix, tmix = Mixer(N, N * eng.D, 64, 32, "cuda", seed=7), Mixer(N, N * eng.D, 64, 32, "cuda", seed=7)
kw = {k: os.environ[v] == "1" for k, v in (("fwd_side", "MB_FWD_SIDE"),) if v in os.environ}
L = QLearner(eng.behavior, eng.target, mix, tmix, batch=32, chunk=10, mode="qmix", device="cuda", **kw)
K = int(os.environ.get("MB_K", 10))              # updates per graph launch (the trainer's update_iter)
L.capture_update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=3, per_replay=K)
if os.environ.get("MB_FUSED", "1") == "0":     # A/B: the two-graph replay path
    L.graph_fused = None
L.replay_updates(10)
torch.cuda.synchronize()
a, b = torch.cuda.Event(True), torch.cuda.Event(True)
a.record()
L.replay_updates(50)
b.record()
torch.cuda.synchronize()
print(json.dumps({"kw": kw, "per_replay": K, "fused": L.graph_fused is not None,
                  "ms_per_update": a.elapsed_time(b) / 50}))
