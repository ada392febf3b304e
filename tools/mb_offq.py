"""Microbenchmark: one offpolicy QMix / VDN train_policy_on_batch (episode BPTT, T = 100,
B = 32 episodes) on device tensors, plus the optional HIP-graph replay of the same update.

Usage: python tools/mb_offq.py [N] [mixer]   (defaults: N = 2 (Checkers), qmix)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-marl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import minimarl._lib as _L  # noqa: E402

if os.environ.get("MB_LIB"):   # A/B: another build of libminimarl.so
    _L.LIB_PATH = os.path.abspath(os.environ["MB_LIB"])
import numpy as np  # noqa: E402
import torch  # noqa: E402
from minimarl.synth import offq_episode_batch as make_batch  # noqa: E402
from minimarl.offq import OffQMix  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2
mixer = sys.argv[2] if len(sys.argv) > 2 else "qmix"
T, B, D, A = 100, 32, 47, 5
tr = OffQMix(N, D, A, T, B, mixer=mixer, seed=1)
rng = np.random.default_rng(0)
obs, share, acts, rew, dones, dones_env = make_batch(rng, N, T, B, D, A)
dev = lambda x: torch.as_tensor(x).cuda().contiguous()  # noqa: E731
pid = "policy_0"
batch = ({pid: dev(obs)}, {pid: dev(share)}, {pid: dev(acts)}, {pid: dev(rew)}, {pid: dev(dones)},
         {pid: dev(dones_env)}, {pid: None}, dev((0.5 + rng.random(B)).astype(np.float32)), None)
for _ in range(3):
    tr.train_policy_on_batch(batch)
    tr.soft_target_updates()
torch.cuda.synchronize()
a, b = torch.cuda.Event(True), torch.cuda.Event(True)
it = 30
a.record()
for _ in range(it):
    tr.train_policy_on_batch(batch)
    tr.soft_target_updates()
b.record()
torch.cuda.synchronize()
eager = a.elapsed_time(b) / it
# graph replay of the same update (device batch tensors fixed)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    tr.train_policy_on_batch(batch)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        tr.train_policy_on_batch(batch)
        tr.soft_target_updates()
torch.cuda.synchronize()
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
a.record()
for _ in range(it):
    g.replay()
b.record()
torch.cuda.synchronize()
graph = a.elapsed_time(b) / it
print(json.dumps({"algo": f"offpolicy {mixer} train_policy_on_batch + soft update", "N": N, "T": T, "B": B, "D": D,
                  "ms_per_update_eager": round(eager, 4), "ms_per_update_graph": round(graph, 4),
                  "loss": float(tr.stats[0])}))
