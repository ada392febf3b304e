"""Microbenchmark of the agent forward (GPU): single-net and dual-net launches at the bench
shape (4096 envs x 8 agents, D=47, GRU-64, A=5), hidden in the engine's [N, H, E] layout.
Prints one JSON line of microseconds per launch and achieved fp32 TFLOP/s.
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402
from minimarl._lib import MM_Q_ACT, MM_Q_MAX, lib  # noqa: E402
from minimarl.qnet import AgentQNet, ptr, stream_handle  # noqa: E402

E = int(os.environ.get("MB_E", 4096))
N, D, H, A = 8, 47, 64, 5
dev = "cuda"
nets = [AgentQNet(N, D, A, 64, 64, H, dev, seed=s) for s in (1, 2)]
for n in nets:
    n.pack()
obs = [torch.rand(E, N, D, device=dev) for _ in range(2)]
hid = [torch.rand(N, H, E, device=dev).permute(2, 0, 1) for _ in range(2)]
hout = [torch.empty(N, H, E, device=dev).permute(2, 0, 1) for _ in range(2)]
qsel = [torch.empty(E, N, device=dev) for _ in range(2)]
act = torch.empty(E, N, dtype=torch.int32, device=dev)
ios = []
for k, mode in enumerate((MM_Q_MAX, MM_Q_ACT)):
    io = nets[k].make_io(obs[k], hid[k], hout[k], None, mode)
    io.qsel_out = qsel[k].data_ptr()
    if mode == MM_Q_ACT:
        io.act_out = act.data_ptr()
        io.epsilon = 0.05
    ios.append(io)


def timeit(fn, it=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


L = lib()
st = stream_handle()


def dual():
    L.mm_agent_q_fwd2(ctypes.byref(nets[0].dims), ptr(nets[0].packed), ctypes.byref(ios[0]), E,
                      ptr(nets[1].packed), ctypes.byref(ios[1]), E, st)


flop = 2 * (D * 64 + 64 * 64 + 3 * 64 * 64 * 2 + 64 * A) * E * N
res = {"E": E, "single_us": timeit(lambda: nets[0].forward_io(E, ios[0])), "dual_us": timeit(dual)}
res["single_tflops"] = flop / res["single_us"] * 1e-6
res["dual_tflops"] = 2 * flop / res["dual_us"] * 1e-6
print(json.dumps(res))
