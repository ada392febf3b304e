"""MAPPO phase timing at BASELINE config 3 (4096 envs x 8 agents, T=100, L=5, 15 PPO epochs).

usage: python tools/mb_mappo.py [--envs E] [--epochs K] [--episodes n]
Prints one JSON line: ms per rollout step, per compute (values + GAE), per train() and per epoch.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
import torch  # noqa: E402
import minimarl._lib as _L  # noqa: E402

if os.environ.get("MB_LIB"):   # A/B: another build of libminimarl.so
    _L.LIB_PATH = os.path.abspath(os.environ["MB_LIB"])
from minimarl.env import VecEnv  # noqa: E402
from minimarl.mappo import MappoPolicy, MappoRunner  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--T", type=int, default=100)
    ap.add_argument("--epochs", type=int, default=15)
    ap.add_argument("--episodes", type=int, default=2)
    a = ap.parse_args()
    env = VecEnv(a.envs, a.agents, max_steps=100, device="cuda")
    p = MappoPolicy(env.obs_dim, 5, 32, "cuda", seed=0)
    r = MappoRunner(env, p, T=a.T, L=5, ppo_epoch=a.epochs, seed=1)
    r.warmup()
    ev = lambda: torch.cuda.Event(enable_timing=True)
    res = []
    for ep in range(a.episodes + 1):
        e0, e1, e2, e3 = ev(), ev(), ev(), ev()
        e0.record()
        r.rollout()
        e1.record()
        r.compute()
        e2.record()
        info = r.train()
        e3.record()
        torch.cuda.synchronize()
        if ep > 0:
            res.append((e0.elapsed_time(e1), e1.elapsed_time(e2), e2.elapsed_time(e3)))
    ro = sum(x[0] for x in res) / len(res)
    co = sum(x[1] for x in res) / len(res)
    tr = sum(x[2] for x in res) / len(res)
    rows = a.envs * a.agents * a.T
    out = {"envs": a.envs, "agents": a.agents, "T": a.T, "epochs": a.epochs,
           "rollout_ms_per_step": ro / a.T, "compute_ms": co, "train_ms": tr, "train_ms_per_epoch": tr / a.epochs,
           "episode_ms": ro + co + tr, "agent_env_steps_per_s_incl_train": rows / ((ro + co + tr) / 1e3),
           "rollout_agent_env_steps_per_s": rows / (ro / 1e3), "train_info": {k: float(v) for k, v in info.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
