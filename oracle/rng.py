"""Oracle (test infrastructure only): numpy restatement of the build's device counter RNG.

The reference draws its exploration randomness from the torch CPU / Python ``random`` streams
(vdn/_network.py:52-58, qmix/_network.py:66-74); those cannot be reproduced on the device, so
the engine uses a stateless splitmix64 counter RNG (csrc/common.h ``mix64`` / ``rng_draw`` /
``rng_uniform``). Restating it here lets the headline-path tests predict every exploratory
action the engine takes (``eps_greedy_draws``) instead of checking rates only.
All arithmetic is uint64 with wrap-around, vectorised over arrays.
"""
import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _u64(x):
    return np.asarray(x, dtype=np.uint64)


def mix64(z):
    with np.errstate(over="ignore"):
        z = _u64(z) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def rng_draw(seed, counter, a, b):
    """mix64(seed ^ mix64(counter * K1 ^ mix64(a * K2 + b))) (common.h rng_draw)."""
    with np.errstate(over="ignore"):
        inner = mix64(_u64(a) * np.uint64(0x8CB92BA72F3D8DD7) + _u64(b))
        mid = mix64((_u64(counter) * np.uint64(0xD1B54A32D192ED03)) ^ inner)
        return mix64(_u64(seed) ^ mid)


def rng_uniform(r):
    """f32 uniform in [0, 1) from the top 24 bits (exact in f32)."""
    return ((_u64(r) >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)).astype(np.float32)


def eps_greedy_draws(seed, counter, n_envs, n_agents, n_actions):
    """The fused forward's epsilon-greedy draws for one step (agent_fwd.hip, MM_Q_ACT epilogue):
    one uniform per env row (all agents of a row explore together, vdn/_network.py:53) and a
    random action per (env, agent). Returns (u [E] f32, rand_act [E, N] int64)."""
    e = np.arange(n_envs, dtype=np.uint64)
    u = rng_uniform(rng_draw(seed, counter, e, 0xFFFFFFFF))
    ee = np.repeat(e[:, None], n_agents, 1)
    aa = np.tile(np.arange(n_agents, dtype=np.uint64)[None], (n_envs, 1))
    ra = rng_draw(np.uint64(seed) ^ np.uint64(0x5bd1e995), counter, ee, aa) % np.uint64(n_actions)
    return u, ra.astype(np.int64)
