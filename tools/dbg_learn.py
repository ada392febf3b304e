"""Learning-curve probe of the integrated trainer (greedy test score every 50 episodes)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-marl_amd"))
import torch  # noqa: E402

from minimarl.config import QTrainConfig  # noqa: E402
from minimarl.train import QTrainer  # noqa: E402

variants = {
    "vdn_compat": dict(algo="vdn"),
    "vdn_textbook": dict(algo="vdn", reference_compat=False),
    "qmix_min": dict(algo="qmix_min", f1=128, g=32, h=32, mixer_hidden=64, use_step_weight=False),
    "vdn_textbook_lr5e-4": dict(algo="vdn", reference_compat=False, lr=5e-4),
}
for name, kw in variants.items():
    base = dict(n_envs=64, n_agents=2, full_observable=True, buffer_limit=2048, max_epsilon=1.0, min_epsilon=0.05,
                epsilon_anneal_episode=int(os.environ.get("ANNEAL", 150)), max_episodes=400,
                update_target_interval=10, test_interval=50, test_envs=128, seed=3)
    base.update(kw)
    cfg = QTrainConfig(**base)
    tr = QTrainer(cfg, device="cuda")
    t0 = time.time()
    hist = tr.train(int(os.environ.get("EPISODES", 400)))
    q = tr.learner.qa.abs().mean().item()
    print(name, f"{time.time() - t0:.1f}s", "|Q|", round(q, 3),
          [(h["episode"], round(h["test_score"], 2), None if h["train_score"] is None else round(h["train_score"], 2),
            round(h["loss"], 3)) for h in hist], flush=True)
