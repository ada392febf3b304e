"""Microbenchmark of the env step kernel (4096 envs x 8 agents, auto-reset, two obs outputs)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import ctypes  # noqa: E402

import torch  # noqa: E402
from minimarl._lib import lib  # noqa: E402
from minimarl.env import VecEnv  # noqa: E402
from minimarl.qnet import ptr, stream_handle  # noqa: E402

E, N = int(os.environ.get("MB_E", 4096)), 8
CUR = int(os.environ.get("MB_CUR", 1))
env = VecEnv(E, N, max_steps=100, device="cuda")
obs = env.reset()
act = torch.randint(0, 5, (E, N), dtype=torch.int32, device="cuda")
nxt, cur = torch.empty_like(obs), torch.empty_like(obs)
rew = torch.empty(E, N, device="cuda")
done = torch.empty(E, dtype=torch.uint8, device="cuda")
s = stream_handle()


def step():
    lib().mm_env_step(env.handle(), ptr(act), ptr(nxt), ptr(cur) if CUR else None, ptr(rew), ptr(done), s)


for _ in range(20):
    step()
torch.cuda.synchronize()
a, b = torch.cuda.Event(True), torch.cuda.Event(True)
a.record()
for _ in range(200):
    step()
b.record()
torch.cuda.synchronize()
print(json.dumps({"eb": os.environ.get("MM_ENV_EB", "default"), "env_step_us": a.elapsed_time(b) / 200 * 1e3}))
