"""Times the reference's offpolicy QMix.train_policy_on_batch on this container's CPU (build
container only: imports /root/reference read-only). Usage: python tools/ref_time_offq.py [N] [threads]"""
import os
import sys
import time

import numpy as np
import torch

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import make_golden_offq as mg  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2
th = int(sys.argv[2]) if len(sys.argv) > 2 else 8
torch.set_num_threads(th)
m = mg.load()
T, B, D, A = 100, 32, 47, 5
args = m.config.get_config().parse_known_args([])[0]
args.episode_length, args.batch_size = T, B
cfg = {"args": args, "device": torch.device("cpu"), "num_agents": N}
pcfg = {"obs_space": mg.Box(shape=(D,)), "act_space": mg.Discrete(A), "cent_obs_dim": N * D}
pol = m.policy.QMixPolicy(args, cfg, pcfg)
tr = m.qmix.QMix(args, N, B, {"policy_0": pol}, lambda a: "policy_0", device=torch.device("cpu"), episode_length=T)
rng = np.random.default_rng(0)
obs, share, acts, rew, dones, dones_env = mg.make_batch(rng, N, T, B, D, A)
pid = "policy_0"
batch = ({pid: obs}, {pid: share}, {pid: acts}, {pid: rew}, {pid: dones}, {pid: dones_env}, {pid: None},
         (0.5 + rng.random(B)).astype(np.float32), np.arange(B))
tr.train_policy_on_batch(batch)
t0 = time.time()
n = 5
for _ in range(n):
    tr.train_policy_on_batch(batch)
    tr.soft_target_updates()
dt = (time.time() - t0) / n
print({"reference_cpu_ms_per_update": round(dt * 1e3, 1), "N": N, "T": T, "B": B, "threads": th})
