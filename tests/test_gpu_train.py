"""GPU: the integrated QMIX / VDN trainer (minimarl/train.py; vdn/main.py:80-198, qmix/main.py:100-277)
and the data-parallel learner path."""
import numpy as np
import pytest
import torch

from oracle.env import EnvSpec, VecEnvOracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _random_policy_score(n_agents, full_obs, E=256, seed=0):
    """Mean episode return of uniformly random actions on the oracle env (every env runs 100 steps)."""
    ora = VecEnvOracle(EnvSpec(n_agents, 100, full_observable=full_obs), E)
    rng = np.random.default_rng(seed)
    score, active = np.zeros(E), np.ones(E, bool)
    for _ in range(100):
        _, rew, done = ora.step(rng.integers(0, 5, (E, n_agents)))
        score += active * rew.sum(1)
        active &= ~done
    return float(score.mean())


@pytest.mark.parametrize("algo,kw", [("vdn", dict(reference_compat=False)),
                                     ("qmix_min", dict(f1=128, g=32, h=32, mixer_hidden=64, use_step_weight=False))])
def test_trainer_learns_gridworld(algo, kw):
    """VDN (Target_Dqn with the textbook target, reference_compat=False) and the minimal QMIX
    (qmix/qmix.py) on the 2-agent gridworld: the greedy test score after a fixed budget of 400
    training episodes (64 envs, 10 updates of 32 chunks per episode) is far above the random policy's.
    (With the reference's x N bootstrap and IS-scaled target, reference_compat=True, VDN's Q-values
    diverge at this replay size and epsilon schedule: |Q| ~ 70 and a growing loss, DESIGN.md.)"""
    from minimarl.config import QTrainConfig
    from minimarl.train import QTrainer
    cfg = QTrainConfig(algo=algo, n_envs=64, n_agents=2, full_observable=True, buffer_limit=2048,
                       max_epsilon=1.0, min_epsilon=0.05, epsilon_anneal_episode=150, max_episodes=400,
                       update_target_interval=10, test_interval=100, test_envs=128, seed=3, **kw)
    tr = QTrainer(cfg, device=DEV)
    before = tr.test()["test_score"]
    hist = tr.train(400)
    rand = _random_policy_score(2, True)
    after = hist[-1]["test_score"]
    print("random", rand, "greedy before", before, "history", [(h["episode"], round(h["test_score"], 2),
                                                                  h["train_score"]) for h in hist])
    assert after > rand + 5.0 and after > before + 5.0, (rand, before, after)
    assert np.isfinite(hist[-1]["loss"])


def test_trainer_schedule_and_target_sync():
    """epsilon anneal per episode (vdn/main.py:133-134), hard target sync every update_target_interval
    episodes incl. episode 0 (:184-186), QMIX keeps its target mixer (qmix/main.py:255-256),
    update_iter learner updates per episode, replay filled to buffer_limit by the warm-up."""
    from minimarl.config import QTrainConfig
    from minimarl.train import QTrainer
    cfg = QTrainConfig(algo="qmix", n_envs=32, n_agents=4, full_observable=False, buffer_limit=256,
                       max_epsilon=0.9, min_epsilon=0.05, epsilon_anneal_episode=4, update_target_interval=3,
                       update_iter=2, max_step=20, test_interval=0, test_envs=0, seed=1)
    tr = QTrainer(cfg, device=DEV)
    tm0 = tr.tmix.flat.clone()
    eps = []
    for ep in range(7):
        eps.append(tr.train_episode())
        torch.cuda.synchronize()
        synced = torch.equal(tr.eng.target.flat, tr.eng.behavior.flat)
        assert synced == (ep % 3 == 0), ep
        assert len(tr.eng.per) == 256
        assert tr.learner.updates == 2 * (ep + 1)
    np.testing.assert_allclose(eps, [cfg.epsilon(e) for e in range(7)])
    assert eps[0] == 0.9 and abs(eps[-1] - 0.05) < 1e-12
    assert torch.equal(tr.tmix.flat, tm0)           # the target mixer is never re-synced
    assert not torch.equal(tr.mix.flat, tm0)
    assert tr.eng.t == 7 * 20 + 256 // 32 * 10


def test_dp_learner_half_batches_equal_full_batch():
    """Two QLearner replicas on half batches + a stand-in sum all-reduce (averaged by 1/world inside
    clip/Adam) equal the full-batch update: the post-reduce global norm over the AGENT params only
    (qmix/_train.py:111-115), the clipped agent / unclipped mixer gradients and the parameters. The
    replicas run the captured graphs with the 1/world scale baked in, as bench.py and QTrainer do."""
    from minimarl.learner import MIX_KEYS, Mixer, QLearner
    from minimarl.qnet import AgentQNet
    N, D, A, B, C = 4, 47, 5, 64, 10
    g = torch.Generator().manual_seed(4)
    st, ns = torch.rand(B, C, N, D, generator=g), torch.rand(B, C, N, D, generator=g)
    act = torch.randint(0, A, (B, C, N), generator=g).float()
    rew = torch.randn(B, C, N, generator=g) * 3.0            # large enough that clipping is active
    dn = (torch.rand(B, C, 1, generator=g) < 0.2).float()
    w = torch.rand(B, 1, generator=g) * 0.5 + 0.5

    def make(bs):
        beh, tgt = AgentQNet(N, D, A, 64, 64, 64, DEV, seed=1), AgentQNet(N, D, A, 64, 64, 64, DEV, seed=2)
        mix, tmix = Mixer(N, N * D, 64, 32, DEV, seed=3), Mixer(N, N * D, 64, 32, DEV, seed=4)
        return QLearner(beh, tgt, mix, tmix, batch=bs, chunk=C, mode="qmix", device=DEV)

    full = make(B)
    full.load_batch(st, act, rew, ns, dn, w)
    full.train_step(full._obs_buf, full._obs_buf)
    reps = [make(B // 2) for _ in range(2)]
    for k, r in enumerate(reps):
        sl = slice(k * B // 2, (k + 1) * B // 2)
        r.load_batch(st[sl], act[sl], rew[sl], ns[sl], dn[sl], w[sl])
        r._graph_scale = 0.5
        r.capture_update(None, None, None)
    for r in reps:
        r.graphs[0].replay()
    gsum = reps[0].Gr + reps[1].Gr                     # the stand-in all-reduce (sum)
    for r in reps:
        r.Gr.copy_(gsum)
        r.graphs[1].replay()
    torch.cuda.synchronize()
    assert torch.equal(reps[0].P, reps[1].P)           # replicas stay bit-identical
    nf, nr = float(full.norm[0]), float(reps[0].norm[0])
    assert nf > 5.0                                    # clipping active
    np.testing.assert_allclose(nr, nf, rtol=1e-5)
    coef = min(1.0, 5.0 / (nf + 1e-6))
    ga_f = full.Gr[:full.n_agent] * coef
    ga_r = gsum[:full.n_agent] * 0.5 * coef
    scale = float(ga_f.abs().max())
    assert float((ga_f - ga_r).abs().max()) <= 1e-5 * scale
    gm_f, gm_r = full.Gr[full.n_agent:], gsum[full.n_agent:] * 0.5
    assert float((gm_f - gm_r).abs().max()) <= 1e-5 * float(gm_f.abs().max())
    # post-Adam parameters where the gradient is not negligible (Adam's first step ~ lr * sign(g))
    sel = (full.Gr.abs() > 1e-3 * full.Gr.abs().max())
    np.testing.assert_allclose(reps[0].P[sel].cpu().numpy(), full.P[sel].cpu().numpy(), atol=2e-6)
    assert MIX_KEYS


def test_vdn_double_graph_replay_matches_eager():
    """vdn_double with a device-RNG double net (epsilon > 0): the captured update advances the RNG
    counter and reads epsilon on the device, so graph replays equal eager updates."""
    from minimarl.learner import QLearner
    from minimarl.qnet import AgentQNet
    N, D, A, B, C = 2, 94, 5, 32, 10
    g = torch.Generator().manual_seed(6)
    st, ns = torch.rand(B, C, N, D, generator=g), torch.rand(B, C, N, D, generator=g)
    act = torch.randint(0, A, (B, C, N), generator=g).float()
    rew = torch.randn(B, C, N, generator=g)
    dn = (torch.rand(B, C, 1, generator=g) < 0.2).float()
    w = torch.ones(B, 1)
    outs = []
    for graph in (False, True):
        beh, tgt = AgentQNet(N, D, A, 64, 32, 32, DEV, seed=1), AgentQNet(N, D, A, 64, 32, 32, DEV, seed=2)
        L = QLearner(beh, tgt, None, None, batch=B, chunk=C, mode="vdn_double", device=DEV)
        L.double_eps = 0.5
        L.load_batch(st, act, rew, ns, dn, w)
        acts = []
        if graph:
            L.capture_update(None, None, None)
        for k in range(3):
            if k == 2:
                L.double_eps = 0.25                      # a changed epsilon reaches the captured graph
            if graph:
                L.replay_update()
            else:
                L.train_step(L._obs_buf, L._obs_buf)
            acts.append(L.act_d.clone())
        torch.cuda.synchronize()
        outs.append((L.P.clone(), acts))
    assert torch.equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1], outs[1][1]):
        assert torch.equal(a, b)
    assert not torch.equal(outs[0][1][0], outs[0][1][1])   # fresh draws per update
