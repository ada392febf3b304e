"""World-size-2 gloo tests of the data-parallel semantics (CPU; no GPU needed).

The learner all-reduces the flat gradient once per update and scales by 1/world before
clip + Adam (minimarl.dist / QLearner.update). These tests check, with the CPU oracle as
the per-rank gradient producer, that the averaged gradient of two half batches equals the
single-process gradient of the full batch, that replicas stay bit-identical after the
update, and that env shards need no collective.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import nets


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(seed, B, C, N, D, A):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(B, C, N, D, generator=g), torch.randint(0, A, (B, C, N), generator=g).float(),
            torch.randn(B, C, N, generator=g), torch.rand(B, C, N, D, generator=g),
            (torch.rand(B, C, 1, generator=g) < 0.2).float(), torch.rand(B, 1, generator=g) + 0.5)


def _params(N, D, A, H=32, F1=64, G=32, seed=0):
    g = torch.Generator().manual_seed(seed)
    sh = {"W1": (N, F1, D), "b1": (N, F1), "W2": (N, G, F1), "b2": (N, G), "Wih": (N, 3 * H, G),
          "Whh": (N, 3 * H, H), "bih": (N, 3 * H), "bhh": (N, 3 * H), "Wq": (N, A, H), "bq": (N, A)}
    return {k: (torch.rand(v, generator=g) - 0.5) * 0.3 for k, v in sh.items()}


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
    from minimarl import dist as mdist
    torch.set_num_threads(1)
    r, w = mdist.init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    N, D, A, B, C = 2, 12, 5, 8, 4
    P = _params(N, D, A, seed=1 + rank)          # deliberately different per rank ...
    flat = torch.cat([P[k].reshape(-1) for k in nets.AGENT_KEYS])
    mdist.broadcast_params(flat, 0)              # ... until the broadcast makes replicas identical
    o = 0
    for k in nets.AGENT_KEYS:
        n = P[k].numel()
        P[k] = flat[o:o + n].view_as(P[k]).clone()
        o += n
    T = _params(N, D, A, seed=99)
    full = _batch(5, 2 * B, C, N, D, A)
    shard = tuple(x[rank * B:(rank + 1) * B] for x in full)
    Pg = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    loss, _, _ = nets.vdn_loss(Pg, T, shard, 0.99)
    grads = torch.autograd.grad(loss, [Pg[k] for k in nets.AGENT_KEYS])
    gflat = torch.cat([g.reshape(-1) for g in grads])
    allreduce = mdist.make_allreduce()
    scale = 1.0 / allreduce(gflat)
    out[rank] = (flat.numpy().copy(), (gflat * scale).numpy().copy())
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_two_rank_gradient_average_equals_full_batch():
    ctx = mp.get_context("spawn")
    port = _free_port()
    with ctx.Manager() as m:
        out = m.dict()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, out)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
            assert p.exitcode == 0
        res = dict(out)
    (p0, g0), (p1, g1) = res[0], res[1]
    np.testing.assert_array_equal(p0, p1)          # replicas identical after the broadcast
    np.testing.assert_array_equal(g0, g1)          # identical averaged gradients on both ranks
    # single-process gradient of the full (2B) batch from rank 0's parameters
    N, D, A, B, C = 2, 12, 5, 8, 4
    P = _params(N, D, A, seed=1)
    T = _params(N, D, A, seed=99)
    full = _batch(5, 2 * B, C, N, D, A)
    Pg = {k: v.clone().requires_grad_(True) for k, v in P.items()}
    loss, _, _ = nets.vdn_loss(Pg, T, full, 0.99)
    grads = torch.autograd.grad(loss, [Pg[k] for k in nets.AGENT_KEYS])
    gfull = torch.cat([g.reshape(-1) for g in grads]).numpy()
    np.testing.assert_allclose(g0, gfull, rtol=1e-4, atol=1e-6)


def test_env_shards_are_independent():
    """Weak scaling: rank r owns envs [r*E, (r+1)*E); the oracle env evolves each env alone."""
    from oracle.env import EnvSpec, VecEnvOracle
    spec = EnvSpec(8, 100)
    E = 64
    whole = VecEnvOracle(spec, 2 * E)
    parts = [VecEnvOracle(spec, E) for _ in range(2)]
    rng = np.random.default_rng(0)
    for _ in range(30):
        a = rng.integers(0, 5, (2 * E, 8))
        o, r, d = whole.step(a)
        for k in range(2):
            ok, rk, dk = parts[k].step(a[k * E:(k + 1) * E])
            np.testing.assert_array_equal(ok, o[k * E:(k + 1) * E])
            np.testing.assert_array_equal(rk, r[k * E:(k + 1) * E])
        whole.reset_envs(d)
        for k in range(2):
            parts[k].reset_envs(d[k * E:(k + 1) * E])


def _mappo_worker(rank, world, port, out):
    """MAPPO data-parallel statistics protocol (MappoTrainer.prepare): each rank reduces its own
    buffer to the 5 raw sums (adv, count, ret, ret^2, adv^2 over active rows), one all-reduce,
    then every rank derives the same global statistics (mm_mappo_stats_from_sums formula)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mini-marl_amd"))
    from minimarl import dist as mdist
    torch.set_num_threads(1)
    mdist.init_from_env(backend="gloo")
    rng = np.random.default_rng(10 + rank)
    adv = rng.standard_normal(3000) * (1 + rank)
    ret = rng.standard_normal(3000) + rank
    act = (rng.random(3000) > 0.15).astype(np.float64)
    sums = torch.tensor([(adv * act).sum(), act.sum(), ret.sum(), (ret ** 2).sum(), (adv ** 2 * act).sum()],
                        dtype=torch.float64)
    world_n = mdist.make_allreduce()(sums)
    s, n, sr, sr2, s2 = sums.tolist()
    R = 3000 * world_n
    mu = s / n
    out[rank] = (mu, float(np.sqrt(max(s2 / n - mu * mu, 0.0))), n, sr / R, sr2 / R)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_two_rank_mappo_statistics_are_global():
    ctx = mp.get_context("spawn")
    port = _free_port()
    with ctx.Manager() as m:
        out = m.dict()
        procs = [ctx.Process(target=_mappo_worker, args=(r, 2, port, out)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
            assert p.exitcode == 0
        res = dict(out)
    assert res[0] == res[1]                         # replicas normalise identically
    adv, ret, act = [], [], []
    for r in range(2):
        rng = np.random.default_rng(10 + r)
        adv.append(rng.standard_normal(3000) * (1 + r))
        ret.append(rng.standard_normal(3000) + r)
        act.append(rng.random(3000) > 0.15)
    adv, ret, act = np.concatenate(adv), np.concatenate(ret), np.concatenate(act)
    a = adv.copy()
    a[~act] = np.nan                                # ramppo_network.py:227-231 (nan-masked)
    mu, sd, n, rm, rsq = res[0]
    np.testing.assert_allclose(mu, np.nanmean(a), rtol=1e-10)
    np.testing.assert_allclose(sd, np.nanstd(a), rtol=1e-9)
    assert n == act.sum()
    np.testing.assert_allclose(rm, ret.mean(), rtol=1e-12)
    np.testing.assert_allclose(rsq, (ret ** 2).mean(), rtol=1e-12)
