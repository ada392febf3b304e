"""Learning diagnostics of QMIX on the Switch2 env (QTrainer, env="switch"): greedy test score and loss
curves for a few trainer settings; prints one line per test."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mini-marl_amd")]

import torch  # noqa: E402

from minimarl.config import QTrainConfig  # noqa: E402
from minimarl.train import QTrainer  # noqa: E402

runs = [
    dict(algo="qmix", reference_compat=False, n_envs=64, batch_size=64, epsilon_anneal_episode=300, lr=1e-3),
    dict(algo="qmix", reference_compat=False, n_envs=16, batch_size=32, epsilon_anneal_episode=1000, lr=5e-4),
    dict(algo="vdn", reference_compat=False, n_envs=64, batch_size=64, epsilon_anneal_episode=300, lr=1e-3),
    dict(algo="qmix", reference_compat=True, n_envs=64, batch_size=64, epsilon_anneal_episode=300, lr=1e-3),
]
if os.environ.get("SWEEP"):    # seed / setting sweep around the learning test's configuration
    runs = [dict(algo="qmix", reference_compat=False, n_envs=ne, batch_size=32, epsilon_anneal_episode=an, lr=lr, seed=sd)
            for (ne, an, lr) in ((16, 1000, 5e-4), (16, 600, 5e-4), (8, 600, 5e-4), (16, 1000, 1e-3))
            for sd in (5, 6, 7)]
episodes = int(os.environ.get("EPISODES", "2000"))
for kw in runs:
    a = dict(env="switch", n_agents=2, full_observable=False, buffer_limit=4096, alpha=0.8, beta=0.2,
             use_step_weight=False, max_epsilon=1.0, min_epsilon=0.05, max_episodes=episodes,
             update_target_interval=10, update_iter=10, test_interval=100, test_envs=16, seed=5)
    a.update(kw)
    if a["algo"] == "vdn":
        a.update(alpha=0.4, beta=0.4)
    cfg = QTrainConfig(**a)
    tr = QTrainer(cfg, device="cuda")
    t0 = time.time()
    out = []
    for rec in tr.train(episodes):
        q = tr.eng.behavior.flat.abs().max().item()
        out.append((rec["episode"], round(rec["test_score"], 2), round(rec["train_score"] or 0, 2), round(rec["loss"], 3),
                    round(q, 2)))
    print(kw, "secs", round(time.time() - t0, 1), flush=True)
    for o in out:
        print("   ", o, flush=True)
