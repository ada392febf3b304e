"""Microbenchmark: agent forward kernel variants (hidden layout) at 4096 envs x 8 agents, GRU-64."""
import os, sys, time, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch
from minimarl.qnet import AgentQNet
from minimarl._lib import MM_Q_MAX, MM_Q_ACT

E, N, D, H = 4096, 8, 47, 64
dev = "cuda"
net = AgentQNet(N, D, 5, 64, 64, 64, dev, seed=1)
net2 = AgentQNet(N, D, 5, 64, 64, 64, dev, seed=2)
obs = torch.rand(E, N, D, device=dev)
res = {}
def timeit(fn, it=200):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3
for name, mk in [("ENH", lambda: torch.zeros(E, N, H, device=dev)),
                 ("NHE", lambda: torch.zeros(N, H, E, device=dev).permute(2, 0, 1))]:
    h = mk()
    qmax = torch.empty(E, N, device=dev)
    io = net.make_io(obs, h, h, None, MM_Q_MAX)
    io.qsel_out = qmax.data_ptr()
    net.pack()
    res[name + "_single"] = timeit(lambda: net.forward_io(E, io))
print(json.dumps(res))
