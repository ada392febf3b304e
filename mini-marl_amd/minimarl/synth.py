"""Synthetic episode batches for benchmarks and tests (no environment, no reference code).

``offq_episode_batch`` produces the sample layout of the offpolicy recurrent replay
(``PrioritizedRecReplayBuffer.sample``, offpolicy/utils/rec_buffer.py:192-240,278-304) for
``OffQMix.train_policy_on_batch``: gridworld-like observations (2 coordinates in [0, 1] plus
Bernoulli(0.2) feature bits), one-hot actions, the gridworld's reward values and episodes
that end at random steps.
"""
import numpy as np


def gen_obs(rng, shape):
    o = (rng.random(shape) < 0.2).astype(np.float32)
    o[..., :2] = rng.random(shape[:-1] + (2,)).astype(np.float32)
    return o


def offq_episode_batch(rng, N, T, B, D, A):
    """obs [N, T+1, B, D], share_obs [T+1, B, N*D] (obs_sharing = concat of the agents' obs,
    offpolicy/runner/shared/base_runner.py:337-340), acts one-hot [N, T, B, A], rewards [N, T, B, 1],
    dones [N, T, B, 1], dones_env [T, B, 1]; episodes end at random steps (then all later steps stay
    done, like the runner's all-ones initialisation)."""
    obs = gen_obs(rng, (N, T + 1, B, D))
    share = np.transpose(obs, (1, 2, 0, 3)).reshape(T + 1, B, N * D).copy()
    a = rng.integers(0, A, (N, T, B))
    acts = np.eye(A, dtype=np.float32)[a]
    rew = rng.choice(np.array([-0.01, 0.99, -1.01, 9.99, -10.01], np.float32), (N, T, B, 1))
    end = rng.integers(T // 2, T + 2, B)          # >= T: no done inside the episode
    t = np.arange(T)[:, None]
    dones_env = (t >= end[None, :]).astype(np.float32)[..., None]
    dones = np.broadcast_to(dones_env[None], (N, T, B, 1)).copy()
    return obs, share, acts, rew, dones, dones_env
