"""GPU parity of the HIP learner (QMIX Train_dqn / VDN Target_Dqn) against the reference's own update.

Golden fixtures tests/golden/{qmix,vdn}_train.npz hold the reference's weights, its sampled
batch and its outputs after ONE update. Tolerances (fp32, 10-step BPTT): loss rtol 1e-4;
gradients |g - g_ref| <= 2e-4 * max|g_ref| + 1e-3 * |g_ref|; new priorities rtol 1e-4;
post-Adam params atol 2e-6 where |g_ref| > 1e-4 * max|g_ref| (Adam's first step is
lr * sign(g), so near-zero gradients are compared through the gradient check instead).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from oracle import nets

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _grad_view(learner, key):
    return learner.beh.view(key, learner.Gr[:learner.n_agent])


def _check_grads(g_dev, g_ref, what=""):
    scale = np.abs(g_ref).max()
    np.testing.assert_array_less(np.abs(g_dev - g_ref), 2e-4 * scale + 1e-3 * np.abs(g_ref) + 1e-12, err_msg=what)


def _make(fx, style, mode):
    from minimarl.learner import Mixer, QLearner
    from minimarl.qnet import AgentQNet
    pre = {"qmix": ("before_q.", "target_q."), "vdn": ("before.", "target.")}[mode]
    P = nets.agent_from_state(fx, pre[0], style)
    N, F1, D = P["W1"].shape
    A = P["Wq"].shape[1]
    beh = AgentQNet(N, D, A, 64, 32, 32, DEV)
    beh.load_reference_state(fx, pre[0], style)
    tgt = AgentQNet(N, D, A, 64, 32, 32, DEV)
    tgt.load_reference_state(fx, pre[1], style)
    mix = tmix = None
    if mode == "qmix":
        mix = Mixer(N, N * D, 32, 32, DEV)
        mix.load_reference_state(fx, "before_m.")
        tmix = Mixer(N, N * D, 32, 32, DEV)
        tmix.load_reference_state(fx, "target_m.")
    L = QLearner(beh, tgt, mix, tmix, batch=32, chunk=10, gamma=float(fx["gamma"]), lr=float(fx["lr"]),
                 grad_clip=float(fx["grad_clip"]), mode=mode, device=DEV)
    L.load_batch(fx["states"], fx["actions"], fx["rewards"], fx["next_states"], fx["dones"], fx["is_weight"])
    return L, P


@pytest.mark.parametrize("mode", ["qmix", "vdn"])
def test_learner_matches_reference_update(golden, mode):
    fx = golden(mode + "_train")
    style = "qmix" if mode == "qmix" else "vdn"
    L, P = _make(fx, style, mode)
    L.train_step(L._obs_buf, L._obs_buf)
    torch.cuda.synchronize()
    np.testing.assert_allclose(float(L.loss.item()), float(fx["loss"]), rtol=1e-4)
    np.testing.assert_allclose(L.td_last.cpu().numpy(), fx["new_td"], rtol=1e-4, atol=1e-4)
    # gradients (the reference captured them after clip_grad_norm_; apply our clip coefficient)
    norm = float(L.norm[0].item())
    coef = min(1.0, float(fx["grad_clip"]) / (norm + 1e-6))
    N = P["W1"].shape[0]

    def gidx(i, k):
        # parameters() order: qmix registers per agent (feature, gru, action); vdn registers the
        # ParameterLists feature_net[*], gru_net[*], action_net[*] (vdn/_network.py:21-25)
        if mode == "qmix":
            return 10 * i + k
        return 4 * i + k if k < 4 else (4 * N + 4 * i + k - 4 if k < 8 else 8 * N + 2 * i + k - 8)

    for i in range(N):
        for k, key in enumerate(nets.AGENT_KEYS):
            g_ref = fx[f"g0.{gidx(i, k)}"]
            g_dev = _grad_view(L, key)[i].cpu().numpy() * coef
            _check_grads(g_dev, g_ref)
    after = nets.agent_from_state(fx, "after_q." if mode == "qmix" else "after.", style)
    for key in nets.AGENT_KEYS:
        g_all = np.stack([fx[f"g0.{gidx(i, nets.AGENT_KEYS.index(key))}"] for i in range(N)])
        sel = np.abs(g_all) > 1e-4 * np.abs(g_all).max()
        got = L.beh.view(key).cpu().numpy()
        np.testing.assert_allclose(got[sel], after[key].numpy()[sel], rtol=0, atol=2e-6)
    if mode == "qmix":
        from minimarl.learner import MIX_KEYS
        afterM = nets.mixer_from_state(fx, "after_m.")
        for j, key in enumerate(MIX_KEYS):
            g_ref = fx[f"g1.{j}"]
            g_dev = L.mix.view(key, L.Gr[L.n_agent:]).cpu().numpy()   # mixer grads are not clipped
            _check_grads(g_dev, g_ref)
            sel = np.abs(g_ref) > 1e-4 * np.abs(g_ref).max()
            np.testing.assert_allclose(L.mix.view(key).cpu().numpy()[sel], afterM[key].numpy()[sel], atol=2e-6)


@pytest.mark.parametrize("B", [48, 1024])
def test_learner_gru64_vs_oracle(B):
    """GRU-64 agents + Hm=64 mixer (the cfg2 shapes; no reference sizes exist) vs the torch-CPU oracle;
    B = 1024 exercises the multi-chunk slices of the batched weight-gradient reduction."""
    from minimarl.learner import MIX_KEYS, Mixer, QLearner
    from minimarl.qnet import AgentQNet
    N, D, A, C = 4, 47, 5, 6
    beh = AgentQNet(N, D, A, 64, 64, 64, DEV, seed=1)
    tgt = AgentQNet(N, D, A, 64, 64, 64, DEV, seed=2)
    mix = Mixer(N, N * D, 64, 32, DEV, seed=3)
    tmix = Mixer(N, N * D, 64, 32, DEV, seed=4)
    P0 = {k: v.detach().cpu().clone() for k, v in beh.params().items()}
    T0 = {k: v.detach().cpu().clone() for k, v in tgt.params().items()}
    M0 = {k: mix.view(k).detach().cpu().clone() for k in MIX_KEYS}
    TM0 = {k: tmix.view(k).detach().cpu().clone() for k in MIX_KEYS}
    L = QLearner(beh, tgt, mix, tmix, batch=B, chunk=C, mode="qmix", device=DEV)
    g = torch.Generator().manual_seed(0)
    st = torch.rand(B, C, N, D, generator=g)
    ns = torch.rand(B, C, N, D, generator=g)
    act = torch.randint(0, A, (B, C, N), generator=g).float()
    rew = torch.randn(B, C, N, generator=g) * 0.5
    dn = (torch.rand(B, C, 1, generator=g) < 0.2).float()
    w = torch.rand(B, 1, generator=g) * 0.5 + 0.5
    L.load_batch(st, act, rew, ns, dn, w)
    L.train_step(L._obs_buf, L._obs_buf)
    torch.cuda.synchronize()
    newP, newM, grads, loss, td = nets.qmix_train_step(P0, M0, T0, TM0, (st, act, rew, ns, dn, w), 0.99, 1e-3, 5.0)
    np.testing.assert_allclose(float(L.loss.item()), float(loss), rtol=1e-4)
    np.testing.assert_allclose(L.td_last.cpu().numpy(), td.numpy(), rtol=1e-4, atol=1e-4)
    coef = min(1.0, 5.0 / (float(L.norm[0].item()) + 1e-6))
    for key in nets.AGENT_KEYS:
        _check_grads(_grad_view(L, key).cpu().numpy() * coef, grads[key].numpy())
    for key in MIX_KEYS:
        _check_grads(L.mix.view(key, L.Gr[L.n_agent:]).cpu().numpy(), grads["m." + key].numpy())


@pytest.mark.parametrize("mixer_fp16", [False, True])
def test_learner_cfg5_shapes_vs_oracle(mixer_fp16):
    """cfg5 SMAC-scale shapes (27 agents, obs 300, 36 actions, GRU-32 agents, Hm=32 mixer over an
    8100-wide state) through the whole QMIX update vs the torch-CPU oracle. mixer_fp16: the cfg5 mode
    with the mixer state projection on fp16 MFMA, held to SURVEY 8c's separate tolerance (rtol 2e-3 on
    Q_tot: here on the loss, the TD errors and the batch Q_tot)."""
    from minimarl.learner import MIX_KEYS, Mixer, QLearner
    from minimarl.qnet import AgentQNet
    N, D, A, B, C = 27, 300, 36, 32, 3
    beh = AgentQNet(N, D, A, 64, 32, 32, DEV, seed=5)
    tgt = AgentQNet(N, D, A, 64, 32, 32, DEV, seed=6)
    mix = Mixer(N, N * D, 32, 32, DEV, seed=7)
    tmix = Mixer(N, N * D, 32, 32, DEV, seed=8)
    P0 = {k: v.detach().cpu().clone() for k, v in beh.params().items()}
    T0 = {k: v.detach().cpu().clone() for k, v in tgt.params().items()}
    M0 = {k: mix.view(k).detach().cpu().clone() for k in MIX_KEYS}
    TM0 = {k: tmix.view(k).detach().cpu().clone() for k in MIX_KEYS}
    L = QLearner(beh, tgt, mix, tmix, batch=B, chunk=C, mode="qmix", device=DEV, mixer_fp16=mixer_fp16)
    g = torch.Generator().manual_seed(1)
    st = (torch.rand(B, C, N, D, generator=g) < 0.2).float()
    ns = (torch.rand(B, C, N, D, generator=g) < 0.2).float()
    act = torch.randint(0, A, (B, C, N), generator=g).float()
    rew = torch.randn(B, C, N, generator=g) * 0.5
    dn = (torch.rand(B, C, 1, generator=g) < 0.2).float()
    w = torch.rand(B, 1, generator=g) * 0.5 + 0.5
    L.load_batch(st, act, rew, ns, dn, w)
    L.train_step(L._obs_buf, L._obs_buf)
    torch.cuda.synchronize()
    newP, newM, grads, loss, td = nets.qmix_train_step(P0, M0, T0, TM0, (st, act, rew, ns, dn, w), 0.99, 1e-3, 5.0)
    if mixer_fp16:
        qtot_ref = nets.qmix_qtot(P0, M0, (st, act, rew, ns, dn, w))   # [C, B] behavior Q_tot (fp32 oracle)
        np.testing.assert_allclose(L.qtot.cpu().numpy(), qtot_ref.numpy(), rtol=2e-3,
                                   atol=2e-3 * float(qtot_ref.abs().max()))
        np.testing.assert_allclose(float(L.loss.item()), float(loss), rtol=2e-3)
        np.testing.assert_allclose(L.td_last.cpu().numpy(), td.numpy(), rtol=2e-3,
                                   atol=2e-3 * float(td.abs().max()))
        return
    np.testing.assert_allclose(float(L.loss.item()), float(loss), rtol=1e-4)
    np.testing.assert_allclose(L.td_last.cpu().numpy(), td.numpy(), rtol=1e-4, atol=1e-4)
    coef = min(1.0, 5.0 / (float(L.norm[0].item()) + 1e-6))
    for key in nets.AGENT_KEYS:
        _check_grads(_grad_view(L, key).cpu().numpy() * coef, grads[key].numpy())
    for key in MIX_KEYS:
        _check_grads(L.mix.view(key, L.Gr[L.n_agent:]).cpu().numpy(), grads["m." + key].numpy())


@pytest.mark.parametrize("mixer_fp16", [False, True])
def test_learner_cfg5_benched_path_vs_oracle(mixer_fp16):
    """The cfg5 update exactly as bench.py times it (resident batch via load_batch, captured HIP graphs
    replayed): 27 agents, obs 300, 36 actions, GRU-32 agents, Hm = 32 mixer over the 8100-wide state,
    C = 10 and B = 512 chunk samples, so the large-batch kernels run: agent_split (row tiles of 32
    samples), the chunk-sequence REC, the 8-samples-per-block mixer forward / backward (B >= 512) and,
    with mixer_fp16, mixer_gi_f16 over 5120 rows per net and the mixer's bf16x3 weight-gradient products (the
    agent path stays exact f32: the opt-in fp16x3 PRE, QLearner.fast_pre, flips ~0.3 % of dW1 / dW2 elements past
    this bar through ReLU masks of near-zero pre-activations).

    Tolerances. fp32 mode: the file's fp32 bar (loss rtol 1e-4; gradients 2e-4 * max + 1e-3 * |g|;
    post-Adam params atol 2e-6 where |g| > 1e-3 max).

    fp16 mode. (1) SURVEY 8c's separate bar for the fp16 state projection: Q_tot, loss and TD within rtol 2e-3
    of the exact fp32 oracle. (2) Everything else is held against the oracle run on the SAME f16-rounded mixer
    W_ih (behavior and target mixer): mixer_gi_f16 rounds W_ih and the state to f16 (RTNE) and accumulates in
    fp32, and this batch's states are {0,1} bits (exact in f16), so that oracle computes the same function up
    to summation order. Against it: Q_tot / loss / TD at rtol 1e-4 and EVERY AGENT gradient and post-Adam agent
    param at the fp32 bar with no outlier allowance (the agent path is exact f32 / fp16x3 at rtol 1e-5). The
    mixer's weight gradients are bf16x3 products (~2^-16 relative per product): |g - g_ref| <= 1e-3 * max|g_ref|
    + 1e-2 * |g_ref|, post-Adam mixer params (as the update delta, since the device keeps the unrounded fp32
    W_ih) atol 2e-6 where |g_ref| > 2e-2 * max|g_ref| and the gradient is within its bound."""
    from minimarl.learner import MIX_KEYS, Mixer, QLearner
    from minimarl.qnet import AgentQNet
    N, D, A, B, C = 27, 300, 36, 512, 10
    beh = AgentQNet(N, D, A, 64, 32, 32, DEV, seed=11)
    tgt = AgentQNet(N, D, A, 64, 32, 32, DEV, seed=12)
    mix = Mixer(N, N * D, 32, 32, DEV, seed=13)
    tmix = Mixer(N, N * D, 32, 32, DEV, seed=14)
    P0 = {k: v.detach().cpu().clone() for k, v in beh.params().items()}
    T0 = {k: v.detach().cpu().clone() for k, v in tgt.params().items()}
    M0 = {k: mix.view(k).detach().cpu().clone() for k in MIX_KEYS}
    TM0 = {k: tmix.view(k).detach().cpu().clone() for k in MIX_KEYS}
    L = QLearner(beh, tgt, mix, tmix, batch=B, chunk=C, mode="qmix", device=DEV, mixer_fp16=mixer_fp16)
    assert L.mixer_bf3 == mixer_fp16
    g = torch.Generator().manual_seed(3)
    st = (torch.rand(B, C, N, D, generator=g) < 0.2).float()
    ns = (torch.rand(B, C, N, D, generator=g) < 0.2).float()
    act = torch.randint(0, A, (B, C, N), generator=g).float()
    rew = torch.randn(B, C, N, generator=g) * 0.5
    dn = (torch.rand(B, C, 1, generator=g) < 0.1).float()
    w = torch.rand(B, 1, generator=g) * 0.5 + 0.5
    L.load_batch(st, act, rew, ns, dn, w)
    L.capture_update(None, None, None)          # bench.py's cfg5 line: resident batch, graph replay
    L.replay_update()
    torch.cuda.synchronize()
    batch = (st, act, rew, ns, dn, w)
    qtot_dev = L.qtot.cpu().numpy()
    if mixer_fp16:
        # (1) the SURVEY 8c bar against the exact fp32 oracle
        _, _, _, loss32, td32 = nets.qmix_train_step(P0, M0, T0, TM0, batch, 0.99, 1e-3, 5.0)
        q32 = nets.qmix_qtot(P0, M0, batch)
        rt = 2e-3
        np.testing.assert_allclose(qtot_dev, q32.numpy(), rtol=rt, atol=rt * float(q32.abs().max()))
        np.testing.assert_allclose(float(L.loss.item()), float(loss32), rtol=rt)
        np.testing.assert_allclose(L.td_last.cpu().numpy(), td32.numpy(), rtol=rt, atol=rt * float(td32.abs().max()))
        # (2) the reference for everything else: the oracle on the f16-rounded mixer W_ih
        M0r, TM0r = dict(M0), dict(TM0)
        M0r["gWih"] = M0["gWih"].half().float()
        TM0r["gWih"] = TM0["gWih"].half().float()
        Mref, TMref = M0r, TM0r
        mga, mgr, mpsel = 1e-3, 1e-2, 2e-2
    else:
        Mref, TMref = M0, TM0
        mga, mgr, mpsel = 2e-4, 1e-3, 1e-3
    newP, newM, grads, loss, td = nets.qmix_train_step(P0, Mref, T0, TMref, batch, 0.99, 1e-3, 5.0)
    qtot_ref = nets.qmix_qtot(P0, Mref, batch)
    np.testing.assert_allclose(qtot_dev, qtot_ref.numpy(), rtol=1e-4, atol=1e-4 * float(qtot_ref.abs().max()))
    np.testing.assert_allclose(float(L.loss.item()), float(loss), rtol=1e-4)
    np.testing.assert_allclose(L.td_last.cpu().numpy(), td.numpy(), rtol=1e-4, atol=1e-4)
    coef = min(1.0, 5.0 / (float(L.norm[0].item()) + 1e-6))

    for key in nets.AGENT_KEYS:      # the fp32 bar in both modes, no outliers
        g_ref = grads[key].numpy()
        g_dev = _grad_view(L, key).cpu().numpy() * coef
        _check_grads(g_dev, g_ref, key)
        sel = np.abs(g_ref) > 1e-3 * np.abs(g_ref).max()
        np.testing.assert_allclose(L.beh.view(key).cpu().numpy()[sel], newP[key].numpy()[sel], atol=2e-6,
                                   err_msg=key)
    for key in MIX_KEYS:
        g_ref = grads["m." + key].numpy()
        g_dev = L.mix.view(key, L.Gr[L.n_agent:]).cpu().numpy()
        bound = mga * np.abs(g_ref).max() + mgr * np.abs(g_ref) + 1e-12
        np.testing.assert_array_less(np.abs(g_dev - g_ref), bound, err_msg="m." + key)
        sel = np.abs(g_ref) > mpsel * np.abs(g_ref).max()
        step_dev = L.mix.view(key).cpu().numpy() - M0[key].numpy()
        step_ref = newM[key].numpy() - Mref[key].numpy()
        np.testing.assert_allclose(step_dev[sel], step_ref[sel], atol=2e-6, err_msg="m." + key)


@pytest.mark.parametrize("mode", ["qmix", "vdn"])
def test_learner_switch_shapes_vs_oracle(mode):
    """The Switch2 shapes QMIX trains on by default (qmix/_config.py:14-19): 2 agents, obs D = 3 (one partial
    32-deep k-step), GRU-32 agents, Hm = 32 mixer over the 6-wide state; B = 32, C = 10, dones inside the
    chunks. Loss rtol 1e-4, gradients 2e-4 * max + 1e-3 * |g| vs the torch-CPU oracle."""
    from minimarl.learner import MIX_KEYS, Mixer, QLearner
    from minimarl.qnet import AgentQNet
    N, D, A, B, C = 2, 3, 5, 32, 10
    beh = AgentQNet(N, D, A, 64, 32, 32, DEV, seed=21)
    tgt = AgentQNet(N, D, A, 64, 32, 32, DEV, seed=22)
    mix = tmix = None
    if mode == "qmix":
        mix, tmix = Mixer(N, N * D, 32, 32, DEV, seed=23), Mixer(N, N * D, 32, 32, DEV, seed=24)
    P0 = {k: v.detach().cpu().clone() for k, v in beh.params().items()}
    T0 = {k: v.detach().cpu().clone() for k, v in tgt.params().items()}
    L = QLearner(beh, tgt, mix, tmix, batch=B, chunk=C, mode=mode, device=DEV)
    g = torch.Generator().manual_seed(4)
    st = torch.rand(B, C, N, D, generator=g)
    ns = torch.rand(B, C, N, D, generator=g)
    act = torch.randint(0, A, (B, C, N), generator=g).float()
    rew = torch.randn(B, C, N, generator=g)
    dn = (torch.rand(B, C, 1, generator=g) < 0.15).float()
    w = torch.rand(B, 1, generator=g) * 0.5 + 0.5
    batch = (st, act, rew, ns, dn, w)
    L.load_batch(*batch)
    if mode == "qmix":
        M0 = {k: mix.view(k).detach().cpu().clone() for k in MIX_KEYS}
        TM0 = {k: tmix.view(k).detach().cpu().clone() for k in MIX_KEYS}
        newP, newM, grads, loss, td = nets.qmix_train_step(P0, M0, T0, TM0, batch, 0.99, 1e-3, 5.0)
    else:
        newP, grads, loss, td = nets.vdn_train_step(P0, T0, batch, 0.99, 1e-3, 5.0)
    L.train_step(L._obs_buf, L._obs_buf)
    torch.cuda.synchronize()
    np.testing.assert_allclose(float(L.loss.item()), float(loss), rtol=1e-4)
    np.testing.assert_allclose(L.td_last.cpu().numpy(), td.numpy(), rtol=1e-4, atol=1e-4)
    coef = min(1.0, 5.0 / (float(L.norm[0].item()) + 1e-6))
    for key in nets.AGENT_KEYS:
        _check_grads(_grad_view(L, key).cpu().numpy() * coef, grads[key].numpy())
    if mode == "qmix":
        for key in MIX_KEYS:
            _check_grads(L.mix.view(key, L.Gr[L.n_agent:]).cpu().numpy(), grads["m." + key].numpy())


def test_learner_update_from_device_per():
    """sample -> gather -> train -> priority update through the engine's PER and chunk store."""
    from minimarl.engine import RolloutEngine
    from minimarl.learner import Mixer, QLearner
    E, N = 128, 4
    eng = RolloutEngine(E, N, f1=64, g=64, h=64, chunk=10, capacity=512, seed=5, device=DEV)
    for _ in range(3):
        eng.run_graph(0.5)
    mix = Mixer(N, N * eng.D, 64, 32, DEV, seed=1)
    tmix = Mixer(N, N * eng.D, 64, 32, DEV, seed=1)
    L = QLearner(eng.behavior, eng.target, mix, tmix, batch=32, chunk=10, mode="qmix", device=DEV)
    tree0 = eng.per.tree().cpu().numpy()
    p0 = L.P.clone()
    for k in range(3):
        L.update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=9, counter=k)
    torch.cuda.synchronize()
    assert np.isfinite(L.loss.item())
    assert not torch.equal(p0, L.P)
    tree1 = eng.per.tree().cpu().numpy()
    assert not np.array_equal(tree0, tree1)
    # the tree stays a consistent sum tree
    cap = eng.per.capacity
    for node in range(cap - 1):
        assert abs(tree1[node] - tree1[2 * node + 1] - tree1[2 * node + 2]) <= 1e-9 * max(1.0, tree1[node])
    # rollout keeps running with the updated weights (packed fragments refreshed)
    eng.run_graph(0.5)
    torch.cuda.synchronize()


@pytest.mark.parametrize("mode", ["qmix", "vdn_double"])
def test_learner_graph_replay_matches_eager(mode):
    """Replays of the captured update (one fused graph per update) equal eager updates, including the
    double net's device-RNG epsilon-greedy draws (vdn_double, epsilon 0.3: fresh draws per update)."""
    from minimarl.engine import RolloutEngine
    from minimarl.learner import Mixer, QLearner

    def build():
        eng = RolloutEngine(64, 4, f1=64, g=64, h=64, chunk=10, capacity=256, seed=3, device=DEV)
        for _ in range(2):
            eng.run_graph(0.5)
        if mode == "vdn_double":
            L = QLearner(eng.behavior, eng.target, None, None, batch=16, chunk=10, mode=mode, device=DEV)
            L.double_eps = 0.3
            return eng, L
        mix = Mixer(4, 4 * eng.D, 64, 32, DEV, seed=1)
        tmix = Mixer(4, 4 * eng.D, 64, 32, DEV, seed=2)
        return eng, QLearner(eng.behavior, eng.target, mix, tmix, batch=16, chunk=10, mode="qmix", device=DEV)

    e1, l1 = build()
    e2, l2 = build()
    for _ in range(3):
        l1.update(e1.per, e1.store, e1.env.reset_obs_ptr(), seed=5, counter=0)
    l2.capture_update(e2.per, e2.store, e2.env.reset_obs_ptr(), seed=5)
    for _ in range(3):
        l2.replay_update()
    torch.cuda.synchronize()
    assert torch.equal(l1.P, l2.P)
    assert torch.equal(e1.per.tree(), e2.per.tree())
    assert torch.equal(l1.loss, l2.loss)


def test_qmix_min_matches_reference_update(golden):
    """Minimal QMIX (qmix/qmix.py train, row a15): QNet D->128->32 + GRU-32, MixNet hx 64, Huber loss,
    unweighted sum target, separate agent / mixer clipping; one update vs the reference's."""
    from minimarl.learner import MIX_KEYS, Mixer, QLearner
    from minimarl.qnet import AgentQNet
    fx = golden("qmix_min_train")
    N, D, A, B, C = (int(x) for x in fx["meta"])
    gamma, lr = (float(x) for x in fx["gamma_lr"])
    beh = AgentQNet(N, D, A, 128, 32, 32, DEV)
    beh.load_reference_state(fx, "q.", "min")
    tgt = AgentQNet(N, D, A, 128, 32, 32, DEV)
    tgt.load_reference_state(fx, "qt.", "min")
    mix, tmix = Mixer(N, N * D, 64, 32, DEV), Mixer(N, N * D, 64, 32, DEV)
    mix.load_reference_state(fx, "m.")
    tmix.load_reference_state(fx, "mt.")
    L = QLearner(beh, tgt, mix, tmix, batch=B, chunk=C, gamma=gamma, lr=lr, grad_clip=5.0, mode="qmix_min",
                 device=DEV)
    L.load_batch(fx["s"], fx["a"], fx["r"], fx["s2"], fx["done"], np.ones((B, 1), np.float32))
    L.train_step(L._obs_buf, L._obs_buf)
    torch.cuda.synchronize()
    na, nm = (float(x) for x in L.norm.cpu())
    ca, cm = min(1.0, 5.0 / (na + 1e-6)), min(1.0, 5.0 / (nm + 1e-6))
    gref = nets.agent_from_state(fx, "grad.q.", "min")
    post = nets.agent_from_state(fx, "post.q.", "min")
    for key in nets.AGENT_KEYS:
        g_ref = gref[key].numpy()
        _check_grads(_grad_view(L, key).cpu().numpy() * ca, g_ref)
        sel = np.abs(g_ref) > 1e-4 * np.abs(g_ref).max()
        np.testing.assert_allclose(L.beh.view(key).cpu().numpy()[sel], post[key].numpy()[sel], atol=2e-6)
    gmref = nets.mixer_from_state(fx, "grad.m.")
    postM = nets.mixer_from_state(fx, "post.m.")
    for key in MIX_KEYS:
        g_ref = gmref[key].numpy()
        _check_grads(L.mix.view(key, L.Gr[L.n_agent:]).cpu().numpy() * cm, g_ref)
        sel = np.abs(g_ref) > 1e-4 * np.abs(g_ref).max()
        np.testing.assert_allclose(L.mix.view(key).cpu().numpy()[sel], postM[key].numpy()[sel], atol=2e-6)


def test_qmix_min_uniform_replay_from_engine():
    """qmix_min updates from the device chunk store with uniform chunk sampling (no priorities)."""
    from minimarl.engine import RolloutEngine
    from minimarl.learner import Mixer, QLearner
    E, N = 128, 4
    eng = RolloutEngine(E, N, f1=128, g=32, h=32, chunk=10, capacity=512, seed=5, device=DEV)
    for _ in range(3):
        eng.run_graph(0.5)
    mix, tmix = Mixer(N, N * eng.D, 64, 32, DEV, seed=1), Mixer(N, N * eng.D, 64, 32, DEV, seed=1)
    L = QLearner(eng.behavior, eng.target, mix, tmix, batch=32, chunk=10, mode="qmix_min", device=DEV)
    tree0 = eng.per.tree().clone()
    p0 = L.P.clone()
    for k in range(3):
        L.update_uniform(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=3, counter=k)
    torch.cuda.synchronize()
    assert np.isfinite(L.loss.item()) and not torch.equal(p0, L.P)
    assert torch.equal(tree0, eng.per.tree())          # uniform replay leaves priorities alone
    slots = L.slots.cpu().numpy()
    assert slots.min() >= 0 and slots.max() < len(eng.per)


def test_vdn_double_matches_reference_update(golden):
    """VDN Double-DQN (Target_Double_Dqn, vdn/_train.py:104-158): the double net's eps-greedy draws
    injected from the reference run; loss, priorities, clipped gradients and post-Adam params."""
    from minimarl.learner import QLearner
    from minimarl.qnet import AgentQNet
    fx = golden("vdn_double_train")
    P = nets.agent_from_state(fx, "before.", "vdn")
    N, F1, D = P["W1"].shape
    A = P["Wq"].shape[1]
    beh = AgentQNet(N, D, A, 64, 32, 32, DEV)
    beh.load_reference_state(fx, "before.", "vdn")
    tgt = AgentQNet(N, D, A, 64, 32, 32, DEV)
    tgt.load_reference_state(fx, "target.", "vdn")
    L = QLearner(beh, tgt, None, None, batch=32, chunk=10, gamma=float(fx["gamma"]), lr=float(fx["lr"]),
                 grad_clip=float(fx["grad_clip"]), mode="vdn_double", device=DEV)
    L.double_eps = float(fx["epsilon"])
    L.set_double_draws(fx["double_u"], fx["double_rand_act"])
    L.load_batch(fx["states"], fx["actions"], fx["rewards"], fx["next_states"], fx["dones"], fx["is_weight"])
    L.train_step(L._obs_buf, L._obs_buf)
    torch.cuda.synchronize()
    np.testing.assert_allclose(float(L.loss.item()), float(fx["loss"]), rtol=1e-4)
    np.testing.assert_allclose(L.td_last.cpu().numpy(), fx["new_td"], rtol=1e-4, atol=1e-4)
    coef = min(1.0, float(fx["grad_clip"]) / (float(L.norm[0].item()) + 1e-6))

    def gidx(i, k):   # vdn parameters() order: feature_net[*], gru_net[*], action_net[*]
        return 4 * i + k if k < 4 else (4 * N + 4 * i + k - 4 if k < 8 else 8 * N + 2 * i + k - 8)

    after = nets.agent_from_state(fx, "after.", "vdn")
    for k, key in enumerate(nets.AGENT_KEYS):
        g_all = np.stack([fx[f"g0.{gidx(i, k)}"] for i in range(N)])
        _check_grads(_grad_view(L, key).cpu().numpy() * coef, g_all)
        sel = np.abs(g_all) > 1e-4 * np.abs(g_all).max()
        np.testing.assert_allclose(L.beh.view(key).cpu().numpy()[sel], after[key].numpy()[sel], atol=2e-6)


@pytest.mark.parametrize("mode,f1,g,h,hm", [("qmix", 64, 64, 64, 64), ("vdn", 64, 32, 32, 32),
                                            ("qmix_min", 128, 32, 32, 64)])
def test_chunk_sequence_launches_match_per_step(mode, f1, g, h, hm):
    """REC / mixer fwd / mixer bwd / agent bwd as one launch each for all C steps: bit-identical to
    the per-step launches."""
    from minimarl.learner import Mixer, QLearner
    from minimarl.qnet import AgentQNet
    N, D, A, B, C = 4, 47, 5, 32, 10
    gen = torch.Generator().manual_seed(3)
    st, ns = torch.rand(B, C, N, D, generator=gen), torch.rand(B, C, N, D, generator=gen)
    act = torch.randint(0, A, (B, C, N), generator=gen).float()
    rew = torch.randn(B, C, N, generator=gen)
    dn = (torch.rand(B, C, 1, generator=gen) < 0.25).float()
    w = torch.rand(B, 1, generator=gen) + 0.5
    out = []
    for seq in (True, False):
        beh = AgentQNet(N, D, A, f1, g, h, DEV, seed=1)
        tgt = AgentQNet(N, D, A, f1, g, h, DEV, seed=2)
        mix = tmix = None
        if mode != "vdn":
            mix, tmix = Mixer(N, N * D, hm, 32, DEV, seed=3), Mixer(N, N * D, hm, 32, DEV, seed=4)
        L = QLearner(beh, tgt, mix, tmix, batch=B, chunk=C, mode=mode, device=DEV)
        L.seq = seq
        L.load_batch(st, act, rew, ns, dn, w)
        L.train_step(L._obs_buf, L._obs_buf)
        torch.cuda.synchronize()
        out.append((L.P.clone(), L.Gr.clone(), L.loss.clone(), L.qa.clone(), L.maxq.clone(), L.dqa.clone()))
    for x, y in zip(*out):
        assert torch.equal(x, y)


@pytest.mark.parametrize("M,fn", [(320, "mm_outer_reduce_batch"), (4096 * 10 + 17, "mm_outer_reduce_batch"),
                                  (4096 * 10 + 17, "mm_outer_reduce_batch_bf3")])
def test_outer_reduce_batch_large_rows(M, fn):
    """The batched weight-gradient reduction (mm_outer_reduce_batch) at the learner's row counts for
    B = 32 and B = 4096 (multi-chunk slices) against a float64 torch reference; the fast mode's bf16x3-split
    variant within the same bounds (its ~2^-16 per-product error averages out over the 40977-row sums; tiny
    and huge magnitudes mixed in to exercise the fp32 exponent range that f16 would lose)."""
    import ctypes
    from minimarl._lib import OuterArgs, check, lib
    from minimarl.qnet import ptr, stream_handle
    g = torch.Generator(device=DEV).manual_seed(1)
    G, R, Cc = 3, 70, 45
    U = torch.randn(G, M, R, device=DEV, generator=g)
    V = torch.randn(G, M, Cc, device=DEV, generator=g)
    if fn.endswith("bf3"):
        U[0] *= 1e-9          # gradient-sized values far below f16's normal range
        V[1] *= 1e6
    dW = torch.zeros(G, R, Cc, device=DEV)
    db = torch.zeros(G, R, device=DEV)
    a = OuterArgs()
    a.U, a.u_g, a.u_m = ptr(U), M * R, R
    a.V, a.v_g, a.v_m = ptr(V), M * Cc, Cc
    a.dW, a.w_g, a.db, a.b_g = ptr(dW), R * Cc, ptr(db), R
    a.M, a.R, a.Cc, a.accumulate, a.groups = M, R, Cc, 0, G
    L = lib()
    n = int(L.mm_outer_reduce_batch_partial(ctypes.byref(a), 1))
    part = torch.zeros(n, device=DEV)
    check(getattr(L, fn)(ctypes.byref(a), 1, ptr(part), n, stream_handle()), fn)
    torch.cuda.synchronize()
    ref = torch.einsum("gmr,gmc->grc", U.double(), V.double())
    for k in range(G):   # per group: atol scaled by that group's magnitude (sqrt(M) random-sign growth)
        scale = float(U[k].abs().max()) * float(V[k].abs().max())
        np.testing.assert_allclose(dW[k].double().cpu().numpy(), ref[k].cpu().numpy(), rtol=1e-4,
                                   atol=1e-3 * scale * np.sqrt(M / 320))
        np.testing.assert_allclose(db[k].double().cpu().numpy(), U[k].double().sum(0).cpu().numpy(), rtol=1e-4,
                                   atol=1e-3 * float(U[k].abs().max()) * np.sqrt(M / 320))


@pytest.mark.parametrize("knob", ["mixer", "agent_bwd"])
def test_multi_sample_blocks_bit_identical(knob):
    """B >= 512 runs the mixer forward with 8 samples per block and the agent backward with 8
    samples per wave (shared weight reads); each must give exactly the one-sample kernel's results
    (mm_learner_set_multi_sample with that kernel's flag 0)."""
    from minimarl._lib import lib
    from minimarl.learner import Mixer, QLearner
    from minimarl.qnet import AgentQNet
    N, D, A, B, C = 4, 47, 5, 600, 4
    res = []
    for multi in (1, 0):
        lib().mm_learner_set_multi_sample(multi if knob == "mixer" else 1, multi if knob == "agent_bwd" else 1)
        try:
            beh = AgentQNet(N, D, A, 64, 64, 64, DEV, seed=1)
            tgt = AgentQNet(N, D, A, 64, 64, 64, DEV, seed=2)
            mix = Mixer(N, N * D, 64, 32, DEV, seed=3)
            tmix = Mixer(N, N * D, 64, 32, DEV, seed=4)
            L = QLearner(beh, tgt, mix, tmix, batch=B, chunk=C, mode="qmix", device=DEV)
            g = torch.Generator().manual_seed(0)
            st = torch.rand(B, C, N, D, generator=g)
            ns = torch.rand(B, C, N, D, generator=g)
            act = torch.randint(0, A, (B, C, N), generator=g).float()
            rew = torch.randn(B, C, N, generator=g) * 0.5
            dn = (torch.rand(B, C, 1, generator=g) < 0.2).float()
            w = torch.rand(B, 1, generator=g) * 0.5 + 0.5
            L.load_batch(st, act, rew, ns, dn, w)
            L.train_step(L._obs_buf, L._obs_buf)
            torch.cuda.synchronize()
            res.append((L.loss.clone(), L.P.clone(), L.td_last.clone()))
        finally:
            lib().mm_learner_set_multi_sample(1, 1)
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][2], res[1][2])


@pytest.mark.parametrize("fwd_side", [True, False])
def test_paired_bwd_launch_matches_side_stream(fwd_side):
    """The agent BPTT and the mixer recurrence's backward sharing one launch (mm_agent_mixer_bwd_seq, the default
    on the split mixer path) against the side-stream version (QLearner(pair_bwd=False)), with the mixer's forward
    on its side stream or in line (fwd_side): bit-identical parameters and loss after three captured updates at
    the bench's B = 32 shape."""
    from minimarl.engine import RolloutEngine
    from minimarl.learner import Mixer, QLearner
    res = []
    for v in ("1", "0"):
        eng = RolloutEngine(2048, 8, f1=64, g=64, h=64, chunk=10, capacity=4096, seed=3, device="cuda")
        for _ in range(2):
            eng.run_graph(0.5)
        N, D = eng.N, eng.D
        mix, tmix = Mixer(N, N * D, 64, 32, "cuda", seed=7), Mixer(N, N * D, 64, 32, "cuda", seed=7)
        lrn = QLearner(eng.behavior, eng.target, mix, tmix, batch=32, chunk=10, mode="qmix", device="cuda",
                       pair_bwd=v == "1", fwd_side=fwd_side)
        assert lrn._pair_bwd == (v == "1") and lrn._mixer_split()
        lrn.capture_update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=1)
        for _ in range(3):
            lrn.replay_update()
        torch.cuda.synchronize()
        res.append((eng.behavior.flat.clone(), mix.flat.clone(), lrn.loss.clone()))
    for x, y in zip(*res):
        assert torch.equal(x, y)


def test_paired_fwd_launches_bit_identical():
    """The forward's agent and mixer chains in shared grids (mm_agent_mixer_pre: agent PRE + mixer state projection,
    mm_agent_mixer_rec_seq: agent recurrence + mixer recurrence; the default at the bench's B = 32 shape) against the
    separate launches on a side stream (QLearner(pair_fwd=False)) and in line (fwd_side=False): bit-identical
    parameters, Adam moments and loss after three captured updates."""
    from minimarl._lib import lib
    from minimarl.engine import RolloutEngine
    from minimarl.learner import Mixer, QLearner
    res = []
    for pair, side in ((True, True), (False, True), (False, False)):
        eng = RolloutEngine(2048, 8, f1=64, g=64, h=64, chunk=10, capacity=4096, seed=3, device="cuda")
        for _ in range(2):
            eng.run_graph(0.5)
        N, D = eng.N, eng.D
        mix, tmix = Mixer(N, N * D, 64, 32, "cuda", seed=7), Mixer(N, N * D, 64, 32, "cuda", seed=7)
        lrn = QLearner(eng.behavior, eng.target, mix, tmix, batch=32, chunk=10, mode="qmix", device="cuda",
                       pair_fwd=pair, fwd_side=side)
        assert lrn._fwd_pair() == pair
        if pair:
            assert lib().mm_agent_mixer_pair_supported(ctypes.byref(eng.behavior.dims), 32, 10, N, N * D, 64, 32) == 3
        lrn.capture_update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=1)
        for _ in range(3):
            lrn.replay_update()
        torch.cuda.synchronize()
        res.append((eng.behavior.flat.clone(), mix.flat.clone(), lrn.m.clone(), lrn.v.clone(), lrn.loss.clone()))
    for other in res[1:]:
        for x, y in zip(res[0], other):
            assert torch.equal(x, y)


@pytest.mark.parametrize("two_groups", [0, 1])
def test_clip_adam_pack_matches_separate_calls(two_groups):
    """mm_clip_adam_pack (the Adam step writing the behavior net's exact-f32 image, the priority update one more
    block of the same launch) against mm_clip_adam / mm_clip2_adam + mm_qnet_pack_f32 + mm_per_update: bit-identical
    parameters, moments, step, norms, image and sum tree (random gradients large enough that the clip engages)."""
    from minimarl._lib import check, lib
    from minimarl.qnet import AgentQNet, ptr, stream_handle
    from minimarl.replay import DevicePER
    L = lib()
    N, D, A = 8, 47, 5
    net = AgentQNet(N, D, A, 64, 64, 64, DEV, seed=5)
    n_agent, n_mix = net.n_params, 9000
    n = n_agent + n_mix
    g = torch.Generator().manual_seed(11)
    P0 = torch.randn(n, generator=g) * 0.1
    G0 = torch.randn(n, generator=g) * 0.05
    m0 = torch.randn(n, generator=g) * 1e-3
    v0 = torch.rand(n, generator=g) * 1e-4
    B, cap = 32, 4096
    nodes = torch.randint(cap - 1, 2 * cap - 1, (B,), generator=g).to(DEV)
    td = torch.rand(B, generator=g).to(DEV)
    outs = []
    for fused in (False, True):
        P, G, m, v = (x.clone().to(DEV) for x in (P0, G0, m0, v0))
        step = torch.full((1,), 2.0, device=DEV)
        partials = torch.zeros(512, device=DEV)
        norm = torch.zeros(2, device=DEV)
        packed = torch.zeros_like(net.packed)
        per = DevicePER(cap, "qmix", device=DEV)
        per.add(torch.rand(cap, generator=torch.Generator().manual_seed(3)).to(DEV))
        s = stream_handle(torch.device(DEV))
        args = (ptr(P), ptr(G), ptr(m), ptr(v), n, n_agent)   # clip group(s): the agent net [, the rest]
        hyp = (5.0, 1e-3, 0.9, 0.999, 1e-8, ptr(step), ptr(partials), ptr(norm), 1.0)
        if fused:
            check(L.mm_clip_adam_pack(*args, two_groups, *hyp, ctypes.byref(net.dims), ptr(packed), per._h,
                                      ptr(nodes), ptr(td), B, None, 0, 0, None, None, None, s), "clip_adam_pack")
        else:
            fn = L.mm_clip2_adam if two_groups else L.mm_clip_adam
            check(fn(*args, *hyp, s), "clip_adam")
            check(L.mm_qnet_pack_f32(ctypes.byref(net.dims), ptr(P), ptr(packed), s), "pack_f32")
            check(L.mm_per_update(per._h, ptr(nodes), ptr(td), B, s), "per_update")
        torch.cuda.synchronize()
        img = (net.packed.numel() - ((N + 63) & ~63)) // 2   # the f32 image: the first N agent strides
        outs.append((P, m, v, step, norm, packed[:img], per.tree()))
    for x, y in zip(*outs):
        assert torch.equal(x, y)
    assert outs[1][4][0] > 5.0           # the clip engaged (norm above max_norm)


def test_hyper_bwd_per_block_matches_separate_update():
    """mm_mixer_bwd_seq_hyper_per (the small priority update as one more block of the hypernet backward, what a
    sampled B = 32 QMIX update issues) against mm_mixer_bwd_seq_hyper + mm_per_update on the same inputs:
    bit-identical hypernet outputs and sum trees."""
    from minimarl._lib import check, lib
    from minimarl.engine import RolloutEngine
    from minimarl.learner import Mixer, QLearner
    from minimarl.qnet import ptr, stream_handle
    from minimarl.replay import DevicePER
    L = lib()
    eng = RolloutEngine(2048, 8, f1=64, g=64, h=64, chunk=10, capacity=4096, seed=3, device="cuda")
    for _ in range(2):
        eng.run_graph(0.5)
    N, D = eng.N, eng.D
    mix, tmix = Mixer(N, N * D, 64, 32, "cuda", seed=7), Mixer(N, N * D, 64, 32, "cuda", seed=7)
    lrn = QLearner(eng.behavior, eng.target, mix, tmix, batch=32, chunk=10, mode="qmix", device="cuda")
    assert lrn._mixer_split()
    lrn.sample_and_grads(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=1)
    torch.cuda.synchronize()
    ts, _ = eng.per.checkpoint_tensors()
    outs = (lrn.dhm, lrn.dqa, lrn.mdelta, lrn.mxws)
    snap = [t.clone() for t in outs]
    s = stream_handle(torch.device(DEV))
    mx = lrn.mix
    margs = (lrn.B, N, mx.S, mx.Hm, mx.K1, ptr(mx.flat), ptr(lrn.msave), ptr(lrn.qa), ptr(lrn.dq), ptr(lrn.done),
             ptr(lrn.ones_f), ptr(lrn.dhm), ptr(lrn.dqa), ptr(lrn.mdelta), ptr(lrn.mxws), lrn.C)
    td = lrn.td_last * 1.5 + 0.25      # other priorities than the ones sample_and_grads already wrote
    res = []
    for fused in (False, True):
        for t, v in zip(outs, snap):
            t.copy_(v)
        per = DevicePER(4096, "qmix", device=DEV)
        per.restore_tensors(ts)
        if fused:
            check(L.mm_mixer_bwd_seq_hyper_per(*margs, per._h, ptr(lrn.nodes), ptr(td), lrn.B, s), "hyp+per")
        else:
            check(L.mm_mixer_bwd_seq_hyper(*margs, s), "hyper")
            check(L.mm_per_update(per._h, ptr(lrn.nodes), ptr(td), lrn.B, s), "per_update")
        torch.cuda.synchronize()
        res.append([t.clone() for t in outs] + [per.tree()])
    for x, y in zip(*res):
        assert torch.equal(x, y)
    assert not torch.equal(res[0][-1], ts["tree"])       # the update changed the tree




def test_multi_update_graph_matches_single_replays():
    """capture_update(per_replay=5) + replay_updates(10) (two launches of a 5-update graph) against ten replays of
    the one-update graph from the same state: bit-identical parameters, Adam moments, PER tree and loss."""
    from minimarl.engine import RolloutEngine
    from minimarl.learner import Mixer, QLearner
    res = []
    for k in (1, 5):
        eng = RolloutEngine(2048, 8, f1=64, g=64, h=64, chunk=10, capacity=4096, seed=3, device="cuda")
        for _ in range(2):
            eng.run_graph(0.5)
        N, D = eng.N, eng.D
        mix, tmix = Mixer(N, N * D, 64, 32, "cuda", seed=7), Mixer(N, N * D, 64, 32, "cuda", seed=7)
        lrn = QLearner(eng.behavior, eng.target, mix, tmix, batch=32, chunk=10, mode="qmix", device="cuda")
        lrn.capture_update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=1, per_replay=k)
        lrn.replay_updates(10)
        torch.cuda.synchronize()
        assert lrn.updates == 10
        res.append((lrn.P.clone(), lrn.m.clone(), lrn.v.clone(), eng.per.tree(), lrn.loss.clone(),
                    eng.behavior.packed.clone()))
    for x, y in zip(*res):
        assert torch.equal(x, y)
