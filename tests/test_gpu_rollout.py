"""GPU parity of the rollout hot path (HIP via the C ABI) against the golden vectors and the oracle.

Tolerances (fp32, stated per SURVEY 8c): single-step Q / hidden rtol 1e-5 atol 1e-5
(exact-f32 MFMA vs MKL summation order); actions exact; env integer state, rewards and
obs bit-exact; sum-tree f64 rtol 1e-12 (tree rebuild vs incremental propagation),
IS weights rtol 1e-6.
"""
import numpy as np
import pytest
import torch

from oracle import nets
from oracle.env import EnvSpec, VecEnvOracle
from oracle.sumtree import SumTreeOracle

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _net_from_fixture(fx, style, f1=64, g=32, h=32):
    from minimarl.qnet import AgentQNet
    P = nets.agent_from_state(fx, "p.", style)
    N, F1, D = P["W1"].shape
    A = P["Wq"].shape[1]
    net = AgentQNet(N, D, A, f1, g, h, DEV)
    net.load_reference_state(fx, "p.", style)
    return net, P


@pytest.mark.parametrize("tag,style", [("qmix_n2", "qmix"), ("qmix_n8", "qmix"), ("vdn_n2", "vdn")])
def test_qnet_forward_golden(golden, tag, style):
    fx = golden("qnet_" + tag)
    net, _ = _net_from_fixture(fx, style)
    q, h = net.forward(torch.tensor(fx["obs"]).to(DEV), torch.tensor(fx["hidden"]).to(DEV))
    np.testing.assert_allclose(q.cpu().numpy(), fx["q"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(h.cpu().numpy(), fx["next_hidden"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("tag", ["qmix", "vdn"])
def test_sample_action_golden_same_seed(golden, tag):
    """The reference-shaped adapter consumes the torch CPU RNG like the reference: equal actions."""
    from minimarl.qnet import Q_Net, _Space
    fx = golden("sample_action_" + tag)
    N, D = fx["obs"].shape[1:]
    qn = Q_Net([_Space((D,))] * N, [_Space(n=5)] * N)
    qn.net.load_reference_state(fx, "p.", tag)
    torch.manual_seed(1234)
    act, h2, q = qn.sample_action(torch.tensor(fx["obs"]), torch.tensor(fx["hidden"]), float(fx["epsilon"]))
    np.testing.assert_array_equal(act.cpu().numpy(), fx["action"])
    np.testing.assert_allclose(q.cpu().numpy(), fx["q"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(h2.cpu().numpy(), fx["next_hidden"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("f1,g,h,n,d,a,e", [(64, 64, 64, 8, 47, 5, 1000), (64, 32, 32, 8, 47, 5, 257),
                                            (64, 64, 64, 8, 47, 5, 2304), (64, 32, 32, 2, 94, 5, 4096),
                                            (128, 32, 32, 2, 94, 5, 130), (64, 32, 32, 4, 300, 36, 96),
                                            # cfg5 SMAC-scale agent net (N=27, D=300, A=36) on the LDS path
                                            (64, 32, 32, 27, 300, 36, 2048)])
def test_qnet_forward_vs_oracle_shapes(f1, g, h, n, d, a, e):
    from minimarl.qnet import AgentQNet
    net = AgentQNet(n, d, a, f1, g, h, DEV, seed=3)
    P = {k: v.detach().cpu().clone() for k, v in net.params().items()}
    gen = torch.Generator().manual_seed(9)
    obs = torch.rand(e, n, d, generator=gen)
    hid = torch.randn(e, n, h, generator=gen) * 0.5
    q, h2 = net.forward(obs.to(DEV), hid.to(DEV))
    qo, ho = nets.agent_forward(P, obs, hid)
    np.testing.assert_allclose(q.cpu().numpy(), qo.numpy(), rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(h2.cpu().numpy(), ho.numpy(), rtol=1e-5, atol=2e-5)
    # epilogues: max and act(eps=0) == argmax, q_taken == gathered q
    qmax, _ = net.max_q(obs.to(DEV), hid.to(DEV))
    np.testing.assert_allclose(qmax.cpu().numpy(), qo.max(2)[0].numpy(), rtol=1e-5, atol=2e-5)
    act, qsel, _, qd = net.act(obs.to(DEV), hid.to(DEV), 0.0)
    greedy = qd.cpu().argmax(2)
    np.testing.assert_array_equal(act.cpu().numpy(), greedy.numpy())
    np.testing.assert_allclose(qsel.cpu().numpy(), qd.cpu().gather(2, greedy.unsqueeze(-1)).squeeze(-1).numpy())


@pytest.mark.parametrize("case", ["activation", "weight"])
def test_fp16x3_range_guard_falls_back_to_f32(case):
    """The fp16x3-split forward (E >= 2048 uses the LDS image path) must not overflow silently: an agent
    whose layer-1 output bound (|obs| <= 1) or largest weight reaches the f16 range is flagged at pack
    time and runs on the exact-f32 image; results still match the f32 oracle for every agent."""
    from minimarl.qnet import AgentQNet
    n, d, a, e = 4, 47, 5, 2304
    net = AgentQNet(n, d, a, 64, 64, 64, DEV, seed=3)
    with torch.no_grad():
        if case == "activation":
            net.view("W1")[1, 0, :] = 3.0e3          # x1 ~ 3e3 * sum(obs) ~ 7e4 > 65504 for agent 1
        elif case == "weight":
            net.view("Whh")[2, 5, 7] = 1.0e5          # not representable in f16: inf in the hi image
    net.mark_dirty()
    P = {k: v.detach().cpu().clone() for k, v in net.params().items()}
    gen = torch.Generator().manual_seed(9)
    obs = torch.rand(e, n, d, generator=gen)
    hid = torch.randn(e, n, 64, generator=gen) * 0.5
    q, h2 = net.forward(obs.to(DEV), hid.to(DEV))
    qo, ho = nets.agent_forward(P, obs, hid)
    assert torch.isfinite(q).all() and torch.isfinite(h2).all()
    scale = max(1.0, float(qo.abs().max()))
    np.testing.assert_allclose(q.cpu().numpy(), qo.numpy(), rtol=1e-5, atol=2e-5 * scale)
    np.testing.assert_allclose(h2.cpu().numpy(), ho.numpy(), rtol=1e-5, atol=2e-5)


def test_eps_greedy_device_rng_rate():
    from minimarl.qnet import AgentQNet
    net = AgentQNet(8, 47, 5, 64, 32, 32, DEV, seed=1)
    E = 4096
    obs = torch.rand(E, 8, 47, device=DEV)
    hid = torch.zeros(E, 8, 32, device=DEV)
    act, _, _, q = net.act(obs, hid, 0.3, seed=5, counter=11)
    greedy = q.argmax(2)
    rand_rows = (act != greedy).any(1).float().mean().item()
    # a random row differs from greedy with prob 1 - (1/5)^8 ~ 1
    assert 0.25 < rand_rows < 0.35
    assert act.min().item() >= 0 and act.max().item() <= 4


@pytest.mark.parametrize("n_agents,full_obs", [(2, False), (2, True), (8, False), (3, False), (17, False), (5, True)])
def test_env_bit_exact_vs_oracle(n_agents, full_obs):
    """The restated ma_gym Checkers dynamics (oracle/env.py) bit for bit: obs, rewards, done, auto-reset obs and
    the integer state (agent_pos, the stale agent_prev_pos, _full_obs codes, counters) over 230 steps of a
    left-biased walk (fruit eaten, apples run out, agents block and erase each other)."""
    from minimarl.env import VecEnv
    E, steps = 300, 230
    spec = EnvSpec(n_agents, max_steps=100, full_observable=full_obs)
    ora = VecEnvOracle(spec, E)
    env = VecEnv(E, n_agents, 100, -0.01, full_obs, device=DEV)
    obs0 = env.reset()
    np.testing.assert_array_equal(obs0.cpu().numpy(), ora.observe())
    rng = np.random.default_rng(4)
    for t in range(steps):
        # biased walk towards the fruit so that apples run out in some envs
        a = np.where(rng.random((E, n_agents)) < 0.6, 1, rng.integers(0, 5, (E, n_agents))).astype(np.int32)
        nxt, rew, done, cur = env.step(torch.tensor(a), autoreset=True)
        onxt, orew, odone = ora.step(a)
        np.testing.assert_array_equal(nxt.cpu().numpy(), onxt)
        np.testing.assert_array_equal(rew.cpu().numpy(), orew)
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), odone)
        ora.reset_envs(odone)
        np.testing.assert_array_equal(cur.cpu().numpy(), ora.observe())
    pos, prev, grid, st, ap = env.get_state()
    np.testing.assert_array_equal(pos, ora.pos)
    np.testing.assert_array_equal(prev, ora.prev)
    np.testing.assert_array_equal(grid, ora.grid)
    np.testing.assert_array_equal(st, ora.steps)
    np.testing.assert_array_equal(ap, ora.apples)


def _per_pair(flavor, cap):
    from minimarl.replay import DevicePER
    if flavor == "vdn":
        kw = dict(alpha=0.4, beta=0.4, eps=1e-6, step_weight=0.99, use_step_weight=True, update_alpha_beta=True,
                  max_episodes=30000, update_iter=10)
        o = SumTreeOracle(cap, "vdn", 0.4, 0.4, alpha_inc=0.6 / 300000, beta_inc=0.6 / 300000)
    else:
        kw = dict(alpha=0.8, beta=0.2, eps=1e-6, use_step_weight=False, update_alpha_beta=True,
                  max_episodes=100000, update_iter=10)
        o = SumTreeOracle(cap, "qmix", 0.8, 0.2, alpha_inc=0.2 / 1e6, beta_inc=0.8 / 1e6)
    return DevicePER(cap, flavor, device=DEV, **kw), o


@pytest.mark.parametrize("flavor", ["vdn", "qmix"])
def test_per_golden_sequence_single_inserts(golden, flavor):
    """Replays the reference's own PER op sequence (K=1 inserts) on the device tree."""
    fx = golden("per_" + flavor)
    cap, b = int(fx["capacity"]), int(fx["batch"])
    dev, _ = _per_pair(flavor, cap)
    for k in range(int(fx["n_ops"])):
        kind = int(fx[f"op{k}.kind"])
        if kind == 0:
            dev.add(torch.tensor([float(fx[f"op{k}.td"])], dtype=torch.float32))
        elif kind == 1:
            nodes, slots, w = dev.sample(b, fracs=fx[f"op{k}.fracs"])
            np.testing.assert_array_equal(nodes.cpu().numpy(), fx[f"op{k}.idx"])
            np.testing.assert_allclose(w.cpu().numpy(), fx[f"op{k}.is_weight"].ravel(), rtol=1e-5)
            last_nodes = nodes
        else:
            dev.update(last_nodes, torch.tensor(fx[f"op{k}.td"]))
        np.testing.assert_allclose(dev.tree().cpu().numpy(), fx[f"op{k}.tree"], rtol=2e-6, atol=1e-9)


@pytest.mark.parametrize("flavor,cap,kb,rounds", [("vdn", 1000, 700, 7), ("qmix", 4099, 700, 7),
                                                  # power-of-two capacities: register-resident fast insert
                                                  ("vdn", 2048, 700, 7), ("qmix", 8192, 3000, 6),
                                                  # >= 16384: the multi-block insert
                                                  ("qmix", 65536, 8192, 10), ("vdn", 16384, 5000, 8),
                                                  ("qmix", 32768, 4096, 12),
                                                  # clustered priorities: threshold bins of ~all leaves
                                                  ("qmix", 65536, 16384, 8)])
def test_per_batched_vs_oracle(flavor, cap, kb, rounds):
    dev, ora = _per_pair(flavor, cap)
    rng = np.random.default_rng(1)
    for rnd in range(rounds):
        td = (rng.random(kb) * 3).astype(np.float32)
        if rnd == rounds - 2:
            td[:50] = td[50]                       # ties
        if cap == 32768 and rnd in (3, 4, 5, 6, 7, 8, 9):
            td[:] = 0.5                            # whole rounds of equal priorities (huge tie sets)
        if kb == 16384 and rnd >= 3:               # one 24-bit key prefix, ties mixed with distinct keys
            td = (0.5 + np.floor(rng.random(kb) * 300) * 1e-7).astype(np.float32)
        slots = dev.add(torch.tensor(td))
        oslots = ora.add_batch([float(x) for x in td])
        np.testing.assert_array_equal(slots.cpu().numpy(), oslots)
        np.testing.assert_allclose(dev.tree().cpu().numpy(), ora.tree, rtol=1e-6, atol=1e-9)
        fr = rng.random(256)
        nodes, s2, w = dev.sample(256, fracs=fr)
        on, os_, _, ow = ora.sample(256, fr)
        np.testing.assert_array_equal(nodes.cpu().numpy(), on)
        np.testing.assert_allclose(w.cpu().numpy(), ow, rtol=1e-5)
        np.testing.assert_allclose(dev.tree().cpu().numpy(), ora.tree, rtol=1e-6, atol=1e-9)
        newtd = (rng.random(256)).astype(np.float32)
        dev.update(nodes, torch.tensor(newtd))
        # oracle: last duplicate wins; priority computed in f32 like the reference
        for k in range(256):
            p32 = np.float32((np.float32(newtd[k]) + np.float32(1e-6)) ** np.float32(ora.alpha))
            ora.tree[on[k]] = float(p32)
        ora.rebuild()
        np.testing.assert_allclose(dev.tree().cpu().numpy(), ora.tree, rtol=1e-6, atol=1e-9)


def test_per_batched_edge_bins_vs_oracle():
    """Multi-block insert with priorities outside the first selection level's binades (2^-16 .. 2^15): tiny (eps
    1e-12, td = 0: (1e-12)^0.8 ~ 2^-32) and huge (td up to 1e9) keys, so the threshold falls in either edge bin of the
    first level in some rounds (every listed key a candidate), and in an interior bin in others."""
    from minimarl.replay import DevicePER
    cap, kb = 65536, 8192
    kw = dict(alpha=0.8, beta=0.2, eps=1e-12, use_step_weight=False, update_alpha_beta=True, max_episodes=100000,
              update_iter=10)
    dev = DevicePER(cap, "qmix", device=DEV, **kw)
    ora = SumTreeOracle(cap, "qmix", 0.8, 0.2, eps=1e-12, alpha_inc=0.2 / 1e6, beta_inc=0.8 / 1e6)
    rng = np.random.default_rng(5)
    for rnd in range(14):
        if rnd % 3 == 0:
            td = np.zeros(kb, np.float32)                                    # all in the low edge bin
            td[: kb // 4] = (rng.random(kb // 4) * 1e-9).astype(np.float32)
        elif rnd % 3 == 1:
            td = (10.0 ** (rng.random(kb) * 9)).astype(np.float32)          # up to 1e9: the high edge bin
        else:
            td = (10.0 ** (rng.random(kb) * 20 - 12)).astype(np.float32)    # every bin kind at once
        slots = dev.add(torch.tensor(td))
        oslots = ora.add_batch([float(x) for x in td])
        np.testing.assert_array_equal(slots.cpu().numpy(), oslots)
        tree = dev.tree().cpu().numpy()
        # leaves exact; the root within f64 summation-order noise (the oracle propagates deltas: huge - huge + tiny)
        np.testing.assert_allclose(tree[cap - 1:], ora.tree[cap - 1:], rtol=1e-12, atol=0)
        np.testing.assert_allclose(tree[0], ora.tree[cap - 1:].sum(), rtol=1e-9)


@pytest.mark.parametrize("cap,B", [(65536, 32), (65536, 64), (1024, 1), (1024, 64), (4, 8)])
def test_per_small_batch_update_vs_oracle(cap, B):
    """Small-batch priority update (LDS path re-sum, B <= 64 on power-of-two trees) vs the oracle's full
    rebuild: sampled nodes with duplicates and shared ancestors, several rounds."""
    dev, ora = _per_pair("qmix", cap)
    rng = np.random.default_rng(7)
    td = (rng.random(cap) * 2).astype(np.float32)
    dev.add(torch.tensor(td))
    ora.add_batch([float(x) for x in td])
    for rnd in range(4):
        fr = rng.random(B)
        nodes, _, _ = dev.sample(B, fracs=fr)
        on, _, _, _ = ora.sample(B, fr)               # keeps the oracle's alpha / beta schedule in step
        nd = nodes.cpu().numpy().copy()
        np.testing.assert_array_equal(nd, on)
        if B > 2:
            nd[1] = nd[0]                              # a duplicate: the later sample wins
            nd[2] = ((nd[0] + 1) ^ 1) - 1              # the sibling leaf of a changed leaf
        newtd = rng.random(B).astype(np.float32)
        dev.update(torch.tensor(nd, device=DEV), torch.tensor(newtd))
        for k in range(B):
            ora.tree[nd[k]] = float(np.float32((np.float32(newtd[k]) + np.float32(1e-6)) ** np.float32(ora.alpha)))
        ora.rebuild()
        np.testing.assert_allclose(dev.tree().cpu().numpy(), ora.tree, rtol=1e-6, atol=1e-9)
    assert dev.error_word() == 0


@pytest.mark.parametrize("cap", [64, 100])
def test_per_update_flags_out_of_range_nodes(cap):
    """Nodes outside the leaf range are skipped (tree unchanged there) and set the sticky error bit;
    in-range nodes of the same update are applied as usual."""
    dev, ora = _per_pair("vdn", cap)
    td = np.linspace(0.1, 2.0, 40).astype(np.float32)
    dev.add(torch.tensor(td))
    ora.add_batch([float(x) for x in td])
    assert dev.error_word() == 0
    good = cap - 1 + 3
    nodes = torch.tensor([good, 0, cap - 2, 2 * cap - 1, -5], dtype=torch.int64, device=DEV)
    dev.update(nodes, torch.tensor([0.7, 9.0, 9.0, 9.0, 9.0]))
    ora.tree[good] = float(np.float32((np.float32(0.7) + np.float32(1e-6)) ** np.float32(ora.alpha)))
    ora.rebuild()
    np.testing.assert_allclose(dev.tree().cpu().numpy(), ora.tree, rtol=1e-6, atol=1e-9)
    assert dev.error_word() == 1
    with pytest.raises(IndexError):
        dev.check_errors()                       # raises and clears
    assert dev.error_word() == 0
    dev.update(nodes[:1], torch.tensor([0.3]))
    dev.check_errors()                           # in-range only: no error


def test_env_stale_prev_erase_scenario():
    """ma_gym's stale agent_prev_pos (oracle/env.py): agent 1 leaves (1,6) for (1,7), agent 0 moves into (1,6);
    in the same step agent 1's view update (its stale prev is (1,6)) writes empty there, so agent 0 vanishes
    from _full_obs and from every observation (its own centre cell included) while both stay put. Scripted in
    env 0 on the device env and the oracle, random actions in the other envs."""
    from minimarl.env import VecEnv
    E = 64
    spec = EnvSpec(2, max_steps=100, full_observable=True)
    ora = VecEnvOracle(spec, E)
    env = VecEnv(E, 2, 100, -0.01, True, device=DEV)
    env.reset()
    rng = np.random.default_rng(8)
    script = [(4, 2), (4, 3), (0, 4), (4, 4), (4, 4)]
    for a_env0 in script:
        a = rng.integers(0, 5, (E, 2)).astype(np.int32)
        a[0] = a_env0
        nxt, rew, done, cur = env.step(torch.tensor(a), autoreset=True)
        onxt, orew, odone = ora.step(a)
        np.testing.assert_array_equal(nxt.cpu().numpy(), onxt)
        np.testing.assert_array_equal(rew.cpu().numpy(), orew)
        ora.reset_envs(odone)
    assert tuple(ora.pos[0, 0]) == (1, 6) and tuple(ora.pos[0, 1]) == (1, 7) and ora.grid[0, 1, 6] == 0
    centre = 2 + 4 * 5                                    # agent 0's own cell, channel "A1"
    assert onxt[0, 0, centre + 2] == 0.0
    pos, prev, grid, _, _ = env.get_state()
    np.testing.assert_array_equal(pos, ora.pos)
    np.testing.assert_array_equal(prev, ora.prev)
    np.testing.assert_array_equal(grid, ora.grid)


def test_rollout_engine_end_to_end_vs_oracle():
    """Engine transitions (store contents), TD chunk priorities and actions vs an oracle replay.
    In-chunk steps run the env kernel fused with the previous step's TD/store, so the store rows
    and chunk priorities are checked once each chunk is complete (and mid-chunk after flush_td)."""
    from minimarl.engine import RolloutEngine
    E, N, C = 96, 8, 10
    eng = RolloutEngine(E, N, f1=64, g=64, h=64, chunk=C, capacity=512, seed=7, device=DEV)
    P = {k: v.detach().cpu().clone() for k, v in eng.behavior.params().items()}
    spec = EnvSpec(N, 100)
    ora = VecEnvOracle(spec, E)
    obs = torch.tensor(ora.observe())
    h = torch.zeros(E, N, 64)
    ht = torch.zeros(E, N, 64)
    td_chunk = np.zeros(E, np.float64)
    hist = []
    steps = 2 * C + 3
    for t in range(steps):
        rows = eng.staging.cpu().numpy()          # staging rows of this step (swapped at chunk end)
        eng.step(epsilon=0.2)
        c = t % C
        if t == C + 4:
            eng.flush_td()                        # exercise the unfused path mid-chunk once
        torch.cuda.synchronize()
        act = eng.act.cpu().numpy().astype(np.int64)
        q, h = nets.agent_forward(P, obs, h)
        greedy = q.argmax(2).numpy()
        qs = q.gather(2, torch.tensor(act).unsqueeze(-1)).squeeze(-1)
        # rows where the engine acted greedily must equal the oracle argmax
        same = (act == greedy).all(1)
        assert same.mean() > 0.6
        nxt, rew, done = ora.step(act)
        np.testing.assert_array_equal(eng.store.obs[rows, c + 1].cpu().numpy(), nxt)
        np.testing.assert_array_equal(eng.rew.cpu().numpy(), rew)
        np.testing.assert_array_equal(eng.done_buf[t % 2].cpu().numpy().astype(bool), done)
        tq, ht = nets.agent_forward(P, torch.tensor(nxt), ht)
        td = (torch.tensor(rew).sum(1) + (1 - torch.tensor(done, dtype=torch.float32)) * 0.99 * tq.max(2)[0].sum(1)
              - qs.sum(1)).abs().numpy()
        td_chunk = td if c == 0 else td_chunk + td
        hist.append((act, rew, done))
        if c == C - 1 or t == C + 4:
            # complete chunk (or flushed step): store rows and the chunk priority so far
            for cc in range(c + 1):
                a_, r_, d_ = hist[t - c + cc]
                np.testing.assert_array_equal(eng.store.act[rows, cc].cpu().numpy(), a_)
                np.testing.assert_array_equal(eng.store.rew[rows, cc].cpu().numpy(), r_)
                np.testing.assert_array_equal(eng.store.done[rows, cc].cpu().numpy().astype(bool), d_)
            np.testing.assert_allclose(eng.chunk_td.cpu().numpy(), td_chunk, rtol=2e-4, atol=2e-4)
        keep = torch.tensor(~done, dtype=torch.float32).view(E, 1, 1)
        h, ht = h * keep, ht * keep
        ora.reset_envs(done)
        obs = torch.tensor(ora.observe())
        np.testing.assert_array_equal(eng.current_obs().cpu().numpy(), obs.numpy())
    assert len(eng.per) == 2 * E
    tree = eng.per.tree().cpu().numpy()
    assert tree[0] > 0


def test_fused_td_matches_unfused():
    """env+TD fused launches give bit-identical stores, priorities and PER to the unfused path."""
    from minimarl.engine import RolloutEngine
    kw = dict(f1=64, g=64, h=64, chunk=10, capacity=512, seed=5, device=DEV)
    a = RolloutEngine(64, 8, **kw)
    b = RolloutEngine(64, 8, **kw)
    for _ in range(25):
        a.step(0.3)
        b.step(0.3)
        b.flush_td()
    a.flush_td()
    torch.cuda.synchronize()
    for x, y in [(a.store.obs, b.store.obs), (a.store.act, b.store.act), (a.store.rew, b.store.rew),
                 (a.store.done, b.store.done), (a.h, b.h), (a.ht, b.ht), (a.chunk_td, b.chunk_td),
                 (a.counter_dev, b.counter_dev), (a.per.tree(), b.per.tree()), (a.per.slot_rows(), b.per.slot_rows())]:
        assert torch.equal(x, y)


def test_graph_replay_matches_eager():
    """A captured chunk replays bit-identically to eager launches (same seed -> same RNG stream)."""
    from minimarl.engine import RolloutEngine
    kw = dict(f1=64, g=64, h=64, chunk=10, capacity=256, seed=11, device=DEV)
    a = RolloutEngine(64, 8, **kw)
    b = RolloutEngine(64, 8, **kw)
    for _ in range(30):
        a.step(0.3)
    for _ in range(3):
        b.run_graph(0.3)
    torch.cuda.synchronize()
    assert a.t == b.t == 30 and len(a.per) == len(b.per) == 192
    for x, y in [(a.store.obs, b.store.obs), (a.store.act, b.store.act), (a.store.rew, b.store.rew),
                 (a.store.done, b.store.done), (a.h, b.h), (a.ht, b.ht), (a.cur_row, b.cur_row),
                 (a.staging, b.staging), (a.per.tree(), b.per.tree()), (a.per.slot_rows(), b.per.slot_rows())]:
        assert torch.equal(x, y)


def test_run_steps_exact_counts_match_eager():
    """run_steps (chunk graphs + single-step graphs, bench.py's exact W / K steps) is bit-identical
    to eager steps, starting and stopping mid-chunk."""
    from minimarl.engine import RolloutEngine
    kw = dict(f1=64, g=64, h=64, chunk=10, capacity=256, seed=13, device=DEV)
    a = RolloutEngine(64, 8, **kw)
    b = RolloutEngine(64, 8, **kw)
    for _ in range(37):
        a.step(0.3)
    a.flush_td()
    b.run_steps(3, 0.3)
    b.run_steps(14, 0.3)
    b.run_steps(20, 0.3)
    b.flush_td()
    torch.cuda.synchronize()
    assert a.t == b.t == 37 and len(a.per) == len(b.per) == 192
    for x, y in [(a.store.obs, b.store.obs), (a.store.act, b.store.act), (a.store.rew, b.store.rew),
                 (a.store.done, b.store.done), (a.h, b.h), (a.ht, b.ht), (a.cur_row, b.cur_row),
                 (a.staging, b.staging), (a.chunk_td, b.chunk_td), (a.per.tree(), b.per.tree()),
                 (a.per.slot_rows(), b.per.slot_rows())]:
        assert torch.equal(x, y)


def _engine_state(e):
    torch.cuda.synchronize()
    st = [e.store.obs, e.store.act, e.store.rew, e.store.done, e.h, e.ht, e.chunk_td, e.cur_row, e.staging,
          e.per.tree(), e.per.slot_rows(), e.act, e.last_rew, e.last_done, e.counter_dev]
    return [x.clone() for x in st] + [torch.as_tensor(v) for v in e.env.get_state()]


def test_region_graphs_match_eager():
    """bench.py's timed regions: ONE captured graph of exactly K steps from any graph phase (capture_region /
    run_steps) is bit-identical to eager steps, through chunk ends, PER eviction and the env's auto-resets."""
    from minimarl.engine import RolloutEngine
    kw = dict(f1=64, g=64, h=64, chunk=10, capacity=256, seed=17, device=DEV)
    a = RolloutEngine(64, 8, **kw)
    b = RolloutEngine(64, 8, **kw)
    for _ in range(57):
        a.step(0.3)
    a.flush_td()
    b.run_steps(3, 0.3)
    b.capture_region(20)
    b.run_steps(20, 0.3)                      # the region graph (phase 3)
    b.capture_region(14, start=b.t + 20)      # captured ahead for the phase two regions later
    b.run_steps(20, 0.3)
    b.run_steps(14, 0.3)
    b.flush_td()
    assert a.t == b.t == 57 and len(a.per) == len(b.per) == 256
    for i, (x, y) in enumerate(zip(_engine_state(a), _engine_state(b))):
        assert torch.equal(x.cpu(), y.cpu()), i
