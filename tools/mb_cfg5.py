"""Microbenchmark: the cfg5 QMIX update exactly as bench.py times it (N = 27, D = 300, A = 36, GRU-32 agents,
Hm = 32 mixer over the 8100-wide state on fp16 MFMA, B = 4096 chunks x C = 10, synthetic batch resident in HBM).
Prints one JSON line (ms per update, event-timed graph replays). Usage: python tools/mb_cfg5.py [B] [iters]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402
from minimarl.learner import Mixer, QLearner  # noqa: E402
from minimarl.qnet import AgentQNet  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
it = int(sys.argv[2]) if len(sys.argv) > 2 else 5
N, D, A, C, dev = 27, 300, 36, 10, "cuda"
nets = [AgentQNet(N, D, A, 64, 32, 32, dev, seed=s) for s in (1, 2)]
m5 = [Mixer(N, N * D, 32, 32, dev, seed=7 + k) for k in range(2)]
L = QLearner(nets[1], nets[0], m5[0], m5[1], batch=B, chunk=C, mode="qmix", device=dev, mixer_fp16=True)
g = torch.Generator(device=dev).manual_seed(5)
st = (torch.rand(B, C, N, D, device=dev, generator=g) < 0.2).float()
ns = (torch.rand(B, C, N, D, device=dev, generator=g) < 0.2).float()
act = torch.randint(0, A, (B, C, N), device=dev, generator=g).float()
rew = torch.randn(B, C, N, device=dev, generator=g) * 0.5
dn = (torch.rand(B, C, 1, device=dev, generator=g) < 0.1).float()
w = torch.rand(B, 1, device=dev, generator=g) * 0.5 + 0.5
L.load_batch(st, act, rew, ns, dn, w)
del st, ns
L.capture_update(None, None, None)
L.replay_update()
torch.cuda.synchronize()
a, b = torch.cuda.Event(True), torch.cuda.Event(True)
a.record()
for _ in range(it):
    L.replay_update()
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / it
print(json.dumps({"B": B, "C": C, "ms_per_update": round(ms, 3), "loss": float(L.loss.item())}))
