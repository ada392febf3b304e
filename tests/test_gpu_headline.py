"""GPU parity of the EXACT launch configuration the headline bench times, against the oracle.

bench.py times ``RolloutEngine(E=4096, N=8, f1=g=h=64, chunk=10, capacity=16*E)`` through HIP-graph
replays: the dual fp16x3 forward (``agent_q_fwd_h3_kernel``: target net on s'_t + behavior net on
s_{t+1} in one launch, second net's params off the kernarg segment), ``obs_row`` indirection into
the chunk store with -1 rows (= the env's reset obs), reset flags, the device-RNG epsilon-greedy
epilogue, the fused env + TD kernel and the multi-block PER insert with eviction. This test runs
that configuration past the point where the PER is full and evicting, and checks at every chunk

* the env transitions in the store rows (s_0, s'_t, actions, rewards, dones) bit-exact vs
  ``oracle/env.py`` driven with the stored actions;
* every exploratory action bit-exact vs the restated device RNG (``oracle/rng.py``);
* the PER: the device's own chunk priorities fed to ``SumTreeOracle.add_batch`` give the same
  slots, the same tree (rtol 1e-6) and the same slot -> row map and staging rows; and the slots' CONTENTS:
  the store row each slot points at holds the chunk the oracle put in that slot (a digest of its obs /
  actions / rewards / dones), for every slot filled by the chunk and a sample of 256 older slots (rows
  swapped in by the insert are never written again while their slot lives);

and on two two-chunk windows (one before, one after eviction starts), from the device's hidden
states at the window start, with the torch-CPU oracle nets (``oracle/nets.py``, fp32):

* every greedy action = the oracle argmax (a different index only on a near-tie, |dQ| <= 2e-5);
* the chunk TD priority (rollout ``cal_td_error`` summed over the chunk, vdn/_utils.py:44-52)
  within rtol 1e-4 / atol 5e-4 (fp16x3-split products vs fp32, summed over 10 steps x 8 agents).

Reference call sites restated: qmix/main.py:180-233 (rollout step + chunking), qmix/_network.py:44-74
(Q_Net.forward / sample_action), vdn/_utils.py:44-52 (cal_td_error), qmix/replay_buffer/per.py:28-34 +
sumtree.py:37-55 (collect_sample / add with min eviction).
"""
import ctypes
import hashlib

import numpy as np
import pytest
import torch

from oracle import nets
from oracle.env import EnvSpec, VecEnvOracle
from oracle.rng import eps_greedy_draws
from oracle.sumtree import SumTreeOracle

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _counter_of_step(t):
    """RNG counter of the behavior forward that picks act_t: the prologue uses 2^63-1, then the
    TD kernel of step t-1 has advanced the device counter to t-1 (engine.py _build_io)."""
    return 0x7FFFFFFFFFFFFFFF if t == 0 else t - 1


def _check_actions_rng(act, t, seed, eps, N):
    u, ra = eps_greedy_draws(seed, _counter_of_step(t), act.shape[0], N, 5)
    expl = u <= np.float32(eps)
    np.testing.assert_array_equal(act[expl], ra[expl])
    return expl


@pytest.mark.parametrize("mode", ["chunk", "fused"])
def test_headline_engine_vs_oracle_through_eviction(mode):
    """mode "chunk": the benched chunk-persistent launches (graph cycle 2C); "fused": one launch per step (lcm(C, 6))."""
    from minimarl.engine import RolloutEngine
    E, N, H, C = 4096, 8, 64, 10
    cap = 16 * E
    eps = 0.1
    seed = 1234
    kw = dict(persistent=True) if mode == "chunk" else dict(fused=True)
    eng = RolloutEngine(E, N, f1=64, g=H, h=H, chunk=C, capacity=cap, seed=seed, device=DEV, **kw)
    if mode == "chunk":
        assert eng.chunked and eng.graph_steps() == eng.S * C
        assert RolloutEngine(E, N, f1=64, g=H, h=H, chunk=C, capacity=E, device=DEV).chunked   # the default mode
    else:
        assert eng.fused and eng.graph_steps() == 3 * C
    P = {k: v.detach().cpu().clone() for k, v in eng.behavior.params().items()}
    Pt = {k: v.detach().cpu().clone() for k, v in eng.target.params().items()}
    spec = EnvSpec(N, 100)
    ora = VecEnvOracle(spec, E)
    tree = SumTreeOracle(cap, "qmix", 0.4, 0.4)
    slot_row = eng.per.slot_rows().cpu().numpy().copy()
    n_chunks = cap // E + 3                 # 16 fills + 3 evicting chunks
    windows = {2, 17}                       # check chunks (k-1, k) with the oracle nets
    snap = None
    last_done = np.zeros(E, bool)
    n_near_tie = 0
    slot_digest = {}                        # slot -> digest of the chunk the oracle put there
    pick = np.random.default_rng(0)

    def digests(o, a, r, d):
        return [hashlib.blake2b(o[i].tobytes() + a[i].tobytes() + r[i].tobytes() + d[i].tobytes(),
                                digest_size=16).digest() for i in range(o.shape[0])]

    for k in range(n_chunks):
        rows = eng.staging.cpu().numpy().copy()
        if k + 1 in windows:                # window start: hidden states before chunk k
            snap = dict(h=eng.h.permute(2, 0, 1).cpu().clone(), ht=eng.ht.permute(2, 0, 1).cpu().clone(),
                        done_prev=last_done.copy(), steps=[])
        eng.run_region(C, eps)              # one chunk: a captured C-step region graph per graph phase
        torch.cuda.synchronize()
        O = eng.store.obs[rows].cpu().numpy()
        A = eng.store.act[rows].cpu().numpy().astype(np.int64)
        R = eng.store.rew[rows].cpu().numpy()
        Dn = eng.store.done[rows].cpu().numpy().astype(bool)
        td_dev = eng.chunk_td.cpu().numpy().copy()
        # ---- env transitions, bit-exact
        np.testing.assert_array_equal(O[:, 0], ora.observe())
        for c in range(C):
            t = k * C + c
            s_t = ora.observe()
            _check_actions_rng(A[:, c], t, seed, eps, N)
            nxt, rew, done = ora.step(A[:, c])
            np.testing.assert_array_equal(O[:, c + 1], nxt)
            np.testing.assert_array_equal(R[:, c], rew)
            np.testing.assert_array_equal(Dn[:, c], done)
            if snap is not None:
                snap["steps"].append((t, s_t, A[:, c].copy(), rew, done, nxt))
            ora.reset_envs(done)
        last_done = Dn[:, C - 1].copy()
        # ---- PER: the device's chunk priorities through the oracle's batched insert
        slots = np.asarray(tree.add_batch([float(x) for x in td_dev]), np.int64)
        np.testing.assert_allclose(eng.per.tree().cpu().numpy(), tree.tree, rtol=1e-6, atol=1e-9)
        new_staging = slot_row[slots].copy()
        slot_row[slots] = rows
        np.testing.assert_array_equal(eng.per.slot_rows().cpu().numpy(), slot_row)
        # (the evicted rows go back into this chunk's staging set: chunk mode rotates S sets, the fused mode has one)
        np.testing.assert_array_equal(eng.staging_all[eng.staging_set(k * C)].cpu().numpy(), new_staging)
        assert len(eng.per) == min(cap, (k + 1) * E)
        # ---- PER slot contents: the rows the device's slot map names hold the oracle's chunks
        for sl, dg in zip(slots, digests(O, eng.store.act[rows].cpu().numpy(), R, eng.store.done[rows].cpu().numpy())):
            slot_digest[int(sl)] = dg
        older = np.setdiff1d(np.fromiter(slot_digest.keys(), np.int64), slots)
        check = np.concatenate([slots, pick.choice(older, min(256, older.size), replace=False) if older.size else
                                np.zeros(0, np.int64)])
        dev_rows = torch.as_tensor(eng.per.slot_rows().cpu().numpy()[check], device=DEV)
        got = digests(eng.store.obs[dev_rows].cpu().numpy(), eng.store.act[dev_rows].cpu().numpy(),
                      eng.store.rew[dev_rows].cpu().numpy(), eng.store.done[dev_rows].cpu().numpy())
        assert got == [slot_digest[int(sl)] for sl in check]
        # ---- oracle nets over the window (chunks k-1, k), from the device hidden states
        if k in windows:
            n_near_tie += _check_window(snap, P, Pt, td_dev, eng, E, N, C, seed, eps)
            snap = None
    assert tree.n_data == cap
    assert n_near_tie <= 64, n_near_tie


def _check_window(snap, P, Pt, td_dev, eng, E, N, C, seed, eps):
    """Steps T0..T0+2C-1 (T0 = the window's first step). Device state at the window start:
    h = behavior hidden after forward(s_T0) (act_T0 was chosen in the previous replay),
    ht = target hidden after forward(s'_{T0-1})."""
    steps = snap["steps"]
    h, ht = snap["h"], snap["ht"]
    done_prev = snap["done_prev"]
    qtaken, maxq = {}, {}
    near = 0
    with torch.no_grad():
        for i, (t, s_t, a_t, rew, done, nxt) in enumerate(steps):
            # target net on s'_t with reset = done_{t-1}
            keep = torch.tensor(~done_prev, dtype=torch.float32).view(E, 1, 1)
            tq, ht = nets.agent_forward(Pt, torch.tensor(nxt), ht * keep)
            maxq[t] = tq.max(2)[0]
            if i > 0:    # behavior net on s_t (its hidden after s_{t-1} with reset = done_{t-1})
                q, h = nets.agent_forward(P, torch.tensor(s_t), h * keep)
                u, _ = eps_greedy_draws(seed, _counter_of_step(t), E, N, 5)
                greedy_rows = u > np.float32(eps)
                qn = q.numpy()
                am = qn.argmax(2)
                diff = (a_t != am) & greedy_rows[:, None]
                if diff.any():
                    qa = np.take_along_axis(qn, a_t[..., None], 2)[..., 0]
                    gap = qn.max(2) - qa
                    assert (gap[diff] <= 2e-5).all(), f"step {t}: greedy action off by {gap[diff].max()}"
                    near += int(diff.sum())
                qtaken[t] = q.gather(2, torch.tensor(a_t).unsqueeze(-1)).squeeze(-1)
            done_prev = done
        # TD priority of the window's second chunk (rollout cal_td_error, no xN, summed over C steps)
        td = torch.zeros(E, dtype=torch.float64)
        for t, s_t, a_t, rew, done, nxt in steps[C:]:
            d = torch.tensor(done, dtype=torch.float32)
            e = (torch.tensor(rew).sum(1) + (1 - d) * 0.99 * maxq[t].sum(1) - qtaken[t].sum(1)).abs()
            td += e.double()
    np.testing.assert_allclose(td_dev, td.numpy(), rtol=1e-4, atol=5e-4)
    return near


def _pack_q(net):
    net.pack()
    return net.packed


@pytest.mark.parametrize("E", [2048, 4096])
def test_dual_forward_two_nets_obs_row_resets(E):
    """``mm_agent_q_fwd2`` at the h3 sizes with two DIFFERENT nets: net 0 in MAX mode on store rows
    (obs_row with -1 = reset obs) with reset flags, net 1 in ACT mode (device RNG) on other rows,
    engine hidden layout [N, H, E]; q, h', max / act / Q(a) vs the oracle."""
    from minimarl._lib import MM_Q_ACT, MM_Q_MAX, QFwdIO, check, lib
    from minimarl.qnet import AgentQNet, ptr, stream_handle
    N, D, H, C = 8, 47, 64, 10
    nets_ = [AgentQNet(N, D, 5, 64, 64, H, DEV, seed=s) for s in (21, 22)]
    Ps = [{k: v.detach().cpu().clone() for k, v in n.params().items()} for n in nets_]
    g = torch.Generator().manual_seed(5)
    rows = 2 * E
    store = (torch.rand(rows, C + 1, N, D, generator=g) < 0.25).float()
    store[..., :2] = torch.rand(rows, C + 1, N, 2, generator=g)
    reset_obs = torch.rand(N, D, generator=g)
    slot = 3
    orow = [torch.randint(0, rows, (E,), generator=g) for _ in range(2)]
    for r in orow:
        r[torch.rand(E, generator=g) < 0.1] = -1
    reset = [(torch.rand(E, generator=g) < 0.15).to(torch.uint8) for _ in range(2)]
    h_in = [torch.randn(N, H, E, generator=g) * 0.5 for _ in range(2)]
    eps, seed, ctr = 0.3, 77, 1234
    d_store, d_reset_obs = store.to(DEV), reset_obs.to(DEV)
    d_orow = [r.to(DEV) for r in orow]
    d_reset = [r.to(DEV) for r in reset]
    d_h = [h.to(DEV) for h in h_in]
    qsel = [torch.empty(E, N, device=DEV) for _ in range(2)]
    act = torch.empty(E, N, dtype=torch.int32, device=DEV)
    eps_dev = torch.full((1,), eps, device=DEV)
    ctr_dev = torch.full((1,), ctr, dtype=torch.int64, device=DEV)
    ios = []
    for k in range(2):
        io = QFwdIO()
        io.obs, io.obs_se, io.obs_sa, io.obs_off = d_store.data_ptr(), (C + 1) * N * D, D, slot * N * D
        io.obs_row, io.reset_obs = d_orow[k].data_ptr(), d_reset_obs.data_ptr()
        io.h_in = io.h_out = d_h[k].data_ptr()
        io.hin_se = io.hout_se = 1
        io.hin_sa = io.hout_sa = H * E
        io.hin_sf = io.hout_sf = E
        io.reset = d_reset[k].data_ptr()
        io.qsel_out = qsel[k].data_ptr()
        ios.append(io)
    ios[0].mode = MM_Q_MAX
    ios[1].mode = MM_Q_ACT
    ios[1].act_out = act.data_ptr()
    ios[1].seed = seed
    ios[1].eps_ptr, ios[1].counter_ptr = eps_dev.data_ptr(), ctr_dev.data_ptr()
    check(lib().mm_agent_q_fwd2(ctypes.byref(nets_[0].dims), ptr(_pack_q(nets_[0])), ctypes.byref(ios[0]), E,
                                ptr(_pack_q(nets_[1])), ctypes.byref(ios[1]), E, stream_handle(DEV)), "fwd2")
    torch.cuda.synchronize()
    for k in range(2):
        ob = torch.where((orow[k] >= 0).view(E, 1, 1), store[orow[k].clamp(min=0), slot],
                         reset_obs.view(1, N, D).expand(E, N, D))
        hin = h_in[k].permute(2, 0, 1) * (1 - reset[k].float()).view(E, 1, 1)
        qo, ho = nets.agent_forward(Ps[k], ob, hin)
        np.testing.assert_allclose(d_h[k].permute(2, 0, 1).cpu().numpy(), ho.numpy(), rtol=1e-5, atol=2e-5)
        if k == 0:
            np.testing.assert_allclose(qsel[0].cpu().numpy(), qo.max(2)[0].numpy(), rtol=1e-5, atol=2e-5)
        else:
            a = act.cpu().numpy().astype(np.int64)
            u, ra = eps_greedy_draws(seed, ctr, E, N, 5)
            expl = u <= np.float32(eps)
            np.testing.assert_array_equal(a[expl], ra[expl])
            qn = qo.numpy()
            gap = qn.max(2) - np.take_along_axis(qn, a[..., None], 2)[..., 0]
            assert (gap[~expl] <= 2e-5).all()
            np.testing.assert_allclose(qsel[1].cpu().numpy(), np.take_along_axis(qn, a[..., None], 2)[..., 0],
                                       rtol=1e-5, atol=2e-5)
            assert 0.25 < expl.mean() < 0.35


def test_cfg5_dual_forward_vs_oracle():
    """bench.py's cfg5 dual forward exactly as timed (E = 8192, N = 27, D = 300, A = 36, F1 = 64,
    GRU-32; net 0 MAX mode, net 1 ACT mode with epsilon 0.05, [E, N, D] obs, zero hidden states in the
    [N, H, E] engine layout) vs the torch-CPU oracle: hiddens, max_a Q and Q(a) rtol 1e-5 (fp16x3
    products), greedy actions = the oracle argmax except within 2e-5 of a tie, exploring rows = the
    restated device RNG."""
    from minimarl._lib import MM_Q_ACT, MM_Q_MAX, check, lib
    from minimarl.qnet import AgentQNet, ptr, stream_handle
    E, N, D, A, H = 8192, 27, 300, 36, 32
    n5 = [AgentQNet(N, D, A, 64, 32, H, DEV, seed=s) for s in (1, 2)]
    Ps = [{k: v.detach().cpu().clone() for k, v in n.params().items()} for n in n5]
    for n in n5:
        n.pack()
    g = torch.Generator().manual_seed(5)
    obs = [(torch.rand(E, N, D, generator=g) < 0.2).float() for _ in range(2)]
    o_dev = [o.to(DEV) for o in obs]
    h5 = [torch.zeros(N, H, E, device=DEV).permute(2, 0, 1) for _ in range(2)]
    hq = [torch.empty(N, H, E, device=DEV).permute(2, 0, 1) for _ in range(2)]
    qs = [torch.empty(E, N, device=DEV) for _ in range(2)]
    act = torch.empty(E, N, dtype=torch.int32, device=DEV)
    ios = []
    for k, mode in enumerate((MM_Q_MAX, MM_Q_ACT)):
        io = n5[k].make_io(o_dev[k], h5[k], hq[k], None, mode)
        io.qsel_out = qs[k].data_ptr()
        if mode == MM_Q_ACT:
            io.act_out, io.epsilon = act.data_ptr(), 0.05
            io.seed, io.counter = 77, 5
        ios.append(io)
    check(lib().mm_agent_q_fwd2(ctypes.byref(n5[0].dims), ptr(n5[0].packed), ctypes.byref(ios[0]), E,
                                ptr(n5[1].packed), ctypes.byref(ios[1]), E, stream_handle(DEV)), "fwd2 cfg5")
    torch.cuda.synchronize()
    with torch.no_grad():
        for k in range(2):
            qo, ho = nets.agent_forward(Ps[k], obs[k], torch.zeros(E, N, H))
            np.testing.assert_allclose(hq[k].cpu().numpy(), ho.numpy(), rtol=1e-5, atol=2e-5)
            qn = qo.numpy()
            if k == 0:
                np.testing.assert_allclose(qs[0].cpu().numpy(), qn.max(2), rtol=1e-5, atol=2e-5)
                continue
            a = act.cpu().numpy().astype(np.int64)
            qa = np.take_along_axis(qn, a[..., None], 2)[..., 0]
            np.testing.assert_allclose(qs[1].cpu().numpy(), qa, rtol=1e-5, atol=2e-5)
            u, ra = eps_greedy_draws(77, 5, E, N, A)
            expl = u <= np.float32(0.05)
            np.testing.assert_array_equal(a[expl], ra[expl])
            gap = qn.max(2) - qa
            assert (gap[~expl] <= 2e-5).all(), gap[~expl].max()
            assert 0.03 < expl.mean() < 0.07


def _batch_from_store(eng, slots):
    """The reference-shaped batch (qmix/replay_buffer/per.py:36-77 sample outputs) of the sampled
    PER slots, read straight from the chunk store on the host: s_t = slot t of the row unless the
    env finished at t-1 (then the env's reset obs), s'_t = slot t+1."""
    rows = eng.per.slot_rows().cpu().numpy()[slots]
    O = eng.store.obs[torch.as_tensor(rows, device=DEV)].cpu()
    Dn = eng.store.done[torch.as_tensor(rows, device=DEV)].cpu().float()
    act = eng.store.act[torch.as_tensor(rows, device=DEV)].cpu().float()
    rew = eng.store.rew[torch.as_tensor(rows, device=DEV)].cpu()
    C = eng.C
    reset_obs = torch.tensor(VecEnvOracle(EnvSpec(eng.N, 100), 1).observe()[0])
    st = O[:, :C].clone()
    for t in range(1, C):
        m = Dn[:, t - 1] > 0.5
        st[m, t] = reset_obs
    return st, act, rew, O[:, 1:].clone(), Dn.unsqueeze(-1)


def test_headline_learner_b4096_vs_oracle():
    """bench.py's throughput-batch learner exactly as timed (RolloutEngine 4096 x 8 store, PER
    capacity 65536, QLearner B = 4096, C = 10, GRU-64 agents, Hm = 64 mixer, captured HIP graphs
    g1 = PER sample + gather + fwd/BPTT, g2 = clip/Adam + repack + reprioritize) against the oracle's
    Train_dqn update (qmix/_train.py:19-121) on the same sampled batch: loss, new priorities, every
    gradient (agent clipped by the agent-only norm, mixer unclipped), post-Adam parameters."""
    from minimarl.learner import MIX_KEYS, Mixer, QLearner
    E, N = 4096, 8
    eng = RolloutEngine_(E, N)
    for _ in range(2):
        eng.run_graph(0.5)
    D = eng.D
    mix, tmix = Mixer(N, N * D, 64, 32, DEV, seed=7), Mixer(N, N * D, 64, 32, DEV, seed=8)
    P0 = {k: v.detach().cpu().clone() for k, v in eng.behavior.params().items()}
    T0 = {k: v.detach().cpu().clone() for k, v in eng.target.params().items()}
    M0 = {k: mix.view(k).detach().cpu().clone() for k in MIX_KEYS}
    TM0 = {k: tmix.view(k).detach().cpu().clone() for k in MIX_KEYS}
    L = QLearner(eng.behavior, eng.target, mix, tmix, batch=4096, chunk=10, mode="qmix", device=DEV)
    L.capture_update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=5)
    L.replay_update()
    torch.cuda.synchronize()
    slots = L.slots.cpu().numpy()
    assert slots.min() >= 0 and slots.max() < len(eng.per)
    st, act, rew, ns, dn = _batch_from_store(eng, slots)
    w = L.isw.cpu().view(-1, 1)
    newP, newM, grads, loss, td = nets.qmix_train_step(P0, M0, T0, TM0, (st, act, rew, ns, dn, w), 0.99, 1e-3, 5.0,
                                                       hidden_dim=32)
    np.testing.assert_allclose(float(L.loss.item()), float(loss), rtol=1e-4)
    np.testing.assert_allclose(L.td_last.cpu().numpy(), td.numpy(), rtol=1e-4, atol=1e-4)
    coef = min(1.0, 5.0 / (float(L.norm[0].item()) + 1e-6))

    def close(g_dev, g_ref):
        scale = np.abs(g_ref).max()
        np.testing.assert_array_less(np.abs(g_dev - g_ref), 2e-4 * scale + 1e-3 * np.abs(g_ref) + 1e-12)

    for key in nets.AGENT_KEYS:
        g_ref = grads[key].numpy()
        close(L.beh.view(key, L.Gr[:L.n_agent]).cpu().numpy() * coef, g_ref)
        sel = np.abs(g_ref) > 1e-3 * np.abs(g_ref).max()
        np.testing.assert_allclose(L.beh.view(key).cpu().numpy()[sel], newP[key].numpy()[sel], atol=2e-6)
    for key in MIX_KEYS:
        g_ref = grads["m." + key].numpy()
        close(L.mix.view(key, L.Gr[L.n_agent:]).cpu().numpy(), g_ref)
        sel = np.abs(g_ref) > 1e-3 * np.abs(g_ref).max()
        np.testing.assert_allclose(L.mix.view(key).cpu().numpy()[sel], newM[key].numpy()[sel], atol=2e-6)


def RolloutEngine_(E, N):
    from minimarl.engine import RolloutEngine
    return RolloutEngine(E, N, f1=64, g=64, h=64, chunk=10, capacity=16 * E, seed=1234, device=DEV)


@pytest.mark.parametrize("dims,flag", [((27, 300, 36, 64, 32, 32), None), ((8, 47, 5, 64, 64, 64), None),
                                       ((27, 300, 36, 64, 32, 32), 5)])
def test_pre_h3_matches_exact_pre(dims, flag):
    """``mm_agent_q_pre2_h3`` (the cfg5 fast-mode learner PRE on the fp16x3 image) vs the exact-f32
    ``mm_agent_q_pre2`` on the same rows of two nets: gi and the x1 | x2 training saves within the fp16x3
    forward's rtol 1e-5; with ``flag`` an agent pushed out of the f16 range takes the exact-f32 image
    (then bit-identical to the exact PRE for that agent)."""
    from minimarl._lib import QFwdIO, check, lib
    from minimarl.qnet import AgentQNet, ptr, stream_handle
    N, D, A, F1, G, H = dims
    nets_ = [AgentQNet(N, D, A, F1, G, H, DEV, seed=s) for s in (31, 32)]
    if flag is not None:
        with torch.no_grad():
            nets_[0].view("W1")[flag, 0, :] = 3.0e3
        nets_[0].mark_dirty()
    E, rows = 5000, 3000
    g = torch.Generator().manual_seed(8)
    store = torch.rand(rows, N, D, generator=g).to(DEV)
    reset_obs = torch.rand(N, D, generator=g).to(DEV)
    offs = [torch.randint(0, rows, (E,), generator=g) * (N * D) for _ in range(2)]
    for o in offs:
        o[torch.rand(E, generator=g) < 0.1] = -1
    offs = [o.to(DEV) for o in offs]
    SD = F1 + G + 6 * H
    out = {}
    for fn in ("mm_agent_q_pre2", "mm_agent_q_pre2_h3"):
        gis = [torch.zeros(E, N, 3 * H, device=DEV) for _ in range(2)]
        save = torch.zeros(E, N, SD, device=DEV)
        ios = []
        for k in range(2):
            io = QFwdIO()
            io.obs, io.obs_se, io.obs_sa, io.obs_off = store.data_ptr(), 1, D, 0
            io.obs_row, io.reset_obs = offs[k].data_ptr(), reset_obs.data_ptr()
            io.h_in = store.data_ptr()      # unused by PRE
            io.gi = gis[k].data_ptr()
            ios.append(io)
        ios[0].save = save.data_ptr()
        check(getattr(lib(), fn)(ctypes.byref(nets_[0].dims), ptr(_pack_q(nets_[0])), ctypes.byref(ios[0]), E,
                                 ptr(_pack_q(nets_[1])), ctypes.byref(ios[1]), E, stream_handle(DEV)), fn)
        torch.cuda.synchronize()
        out[fn] = (gis[0].cpu().numpy(), gis[1].cpu().numpy(), save[..., :F1 + G].cpu().numpy())
    ex, h3 = out["mm_agent_q_pre2"], out["mm_agent_q_pre2_h3"]
    for a, b in zip(h3, ex):
        scale = max(1.0, float(np.abs(b).max()))
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=2e-5 * scale)
    if flag is not None:   # net 0's flagged agent: gi and saves from the exact-f32 image
        for i in (0, 2):
            np.testing.assert_array_equal(h3[i][:, flag], ex[i][:, flag])
