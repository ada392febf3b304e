"""GPU: the PyTorch custom ops (torch.ops.minimarl.*, torch.classes.minimarl.*; csrc/torch_ops.cpp)
against the oracle and the golden vectors, their argument checks and HIP-graph capture."""
import numpy as np
import pytest
import torch

from oracle import nets
from oracle.env import EnvSpec, VecEnvOracle
from oracle.sumtree import SumTreeOracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    from minimarl.ops import load
    return load()


def _net(N=8, D=47, A=5, f1=64, g=64, h=64, seed=3):
    from minimarl.qnet import AgentQNet
    net = AgentQNet(N, D, A, f1, g, h, DEV, seed=seed)
    return net, {k: v.detach().cpu().clone() for k, v in net.params().items()}


@pytest.mark.parametrize("E", [96, 2304])
def test_agent_q_ops_vs_oracle(ops, E):
    from minimarl.ops import dims
    net, P = _net()
    packed = torch.empty_like(net.packed)
    ops.qnet_pack(net.flat, dims(net), packed)
    g = torch.Generator().manual_seed(2)
    obs, hid = torch.rand(E, 8, 47, generator=g), torch.randn(E, 8, 64, generator=g) * 0.5
    o, h = obs.to(DEV), hid.to(DEV)
    q, h2 = torch.empty(E, 8, 5, device=DEV), torch.empty(E, 8, 64, device=DEV)
    ops.agent_q_fwd(packed, dims(net), o, h, h2, q)
    qo, ho = nets.agent_forward(P, obs, hid)
    np.testing.assert_allclose(q.cpu().numpy(), qo.numpy(), rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(h2.cpu().numpy(), ho.numpy(), rtol=1e-5, atol=2e-5)
    mq = torch.empty(E, 8, device=DEV)
    ops.agent_q_max(packed, dims(net), o, h, h2, mq)
    np.testing.assert_allclose(mq.cpu().numpy(), qo.max(2)[0].numpy(), rtol=1e-5, atol=2e-5)
    # injected draws: the reference's epsilon_greedy (vdn/_network.py:52-58) exactly
    u = torch.rand(E, generator=g)
    ra = torch.randint(0, 5, (E, 8), generator=g, dtype=torch.int32)
    act, qt = torch.empty(E, 8, dtype=torch.int32, device=DEV), torch.empty(E, 8, device=DEV)
    q2 = torch.empty_like(q)
    ops.agent_q_act(packed, dims(net), o, h, 0.3, u.to(DEV), ra.to(DEV), 0, 0, h2, act, qt, q2)
    ref = nets.epsilon_greedy(qo, 0.3, u, ra).long()
    a = act.cpu().long()
    greedy = (u > 0.3)
    np.testing.assert_array_equal(a[~greedy].numpy(), ref[~greedy].numpy())
    gap = qo.max(2)[0] - qo.gather(2, a.unsqueeze(-1)).squeeze(-1)
    assert float(gap[greedy].max()) <= 2e-5
    np.testing.assert_allclose(q2.cpu().numpy(), qo.numpy(), rtol=1e-5, atol=2e-5)


def test_td_error_op(ops):
    E, N = 300, 8
    g = torch.Generator().manual_seed(4)
    rew, qt, mq = (torch.randn(E, N, generator=g) for _ in range(3))
    done = (torch.rand(E, generator=g) < 0.2).to(torch.uint8)
    td = torch.empty(E, device=DEV)
    ops.td_error(rew.to(DEV), done.to(DEV), qt.to(DEV), mq.to(DEV), 0.99, td)
    ref = (rew.sum(1) + (1 - done.float()) * 0.99 * mq.sum(1) - qt.sum(1)).abs()     # vdn/_utils.py:44-52
    np.testing.assert_allclose(td.cpu().numpy(), ref.numpy(), rtol=1e-6, atol=1e-5)


def test_gae_scan_op_golden(ops, golden):
    fx = golden("mappo_gae")
    T, E, N = fx["rewards"].shape[:3]
    vp = fx["value_preds"].copy()
    vp[-1] = fx["next_value"]
    vn = torch.tensor([float(fx["vn_mean"][0]), float(fx["vn_mean_sq"][0]), float(fx["vn_debias"])], device=DEV)
    ret = torch.zeros(T + 1, E * N, device=DEV)
    ops.gae_scan(torch.from_numpy(fx["rewards"].reshape(T, E * N)).to(DEV), torch.from_numpy(vp.reshape(T + 1, -1)).to(DEV),
                 torch.from_numpy(fx["masks"].reshape(T + 1, -1)).to(DEV), vn, float(fx["gamma"]),
                 float(fx["gae_lambda"]), ret)
    np.testing.assert_allclose(ret[:T].cpu().numpy(), fx["returns"][:T].reshape(T, E * N), rtol=1e-6, atol=1e-6)


def test_env_class_bit_exact(ops):
    from minimarl.ops import Env
    E, N = 200, 8
    env = Env(E, N, 100, -0.01, False, DEV)
    D = env.obs_dim()
    ora = VecEnvOracle(EnvSpec(N, 100), E)
    obs = torch.empty(E, N, D, device=DEV)
    env.reset(obs)
    np.testing.assert_array_equal(obs.cpu().numpy(), ora.observe())
    nxt, cur = torch.empty_like(obs), torch.empty_like(obs)
    rew, done = torch.empty(E, N, device=DEV), torch.empty(E, dtype=torch.uint8, device=DEV)
    rng = np.random.default_rng(0)
    for _ in range(130):
        a = rng.integers(0, 5, (E, N)).astype(np.int32)
        env.step(torch.from_numpy(a).to(DEV), nxt, cur, rew, done)
        on, orew, od = ora.step(a)
        np.testing.assert_array_equal(nxt.cpu().numpy(), on)
        np.testing.assert_array_equal(rew.cpu().numpy(), orew)
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), od)
        ora.reset_envs(od)
        np.testing.assert_array_equal(cur.cpu().numpy(), ora.observe())


def test_per_class_vs_oracle(ops):
    from minimarl.ops import PER
    cap = 4096
    per = PER(cap, "vdn", 0.4, 0.4, 1e-6, 0.99, True, 0.0, 0.0, DEV)
    ora = SumTreeOracle(cap, "vdn", 0.4, 0.4)
    rng = np.random.default_rng(3)
    for _ in range(5):
        td = (rng.random(1500) * 2).astype(np.float32)
        slots = torch.empty(1500, dtype=torch.int64, device=DEV)
        per.insert(torch.from_numpy(td).to(DEV), slots)
        np.testing.assert_array_equal(slots.cpu().numpy(), ora.add_batch([float(x) for x in td]))
        fr = rng.random(64)
        nodes, s2, w = (torch.empty(64, dtype=torch.int64, device=DEV), torch.empty(64, dtype=torch.int64, device=DEV),
                        torch.empty(64, device=DEV))
        per.sample(torch.from_numpy(fr).to(DEV), 0, 0, nodes, s2, w)
        on, _, _, ow = ora.sample(64, fr)
        np.testing.assert_array_equal(nodes.cpu().numpy(), on)
        np.testing.assert_allclose(w.cpu().numpy(), ow, rtol=1e-5)
        np.testing.assert_allclose(per.tree().cpu().numpy(), ora.tree, rtol=1e-6, atol=1e-9)
    assert per.size() == cap and per.capacity() == cap


def test_ops_argument_errors(ops):
    from minimarl.ops import dims
    net, _ = _net(N=2, D=47, A=5, g=32, h=32)
    o = torch.rand(4, 2, 47, device=DEV)
    h = torch.zeros(4, 2, 32, device=DEV)
    with pytest.raises(RuntimeError, match="obs shape"):
        ops.agent_q_fwd(net.packed, dims(net), torch.rand(4, 3, 47, device=DEV), h, h.clone(),
                        torch.empty(4, 3, 5, device=DEV))
    with pytest.raises(RuntimeError, match="must be float"):
        ops.agent_q_fwd(net.packed, dims(net), o, h.double(), h, torch.empty(4, 2, 5, device=DEV))
    with pytest.raises(RuntimeError, match="'CPU' backend"):   # no CPU kernel is registered: no fallback
        ops.td_error(torch.zeros(4, 2), torch.zeros(4, dtype=torch.uint8), torch.zeros(4, 2), torch.zeros(4, 2), 0.99,
                     torch.zeros(4))


def test_ops_capture_in_hip_graph(ops):
    """The ops enqueue on torch's current stream: a captured forward replays like an eager one."""
    from minimarl.ops import dims
    net, _ = _net()
    packed = net.packed
    net.pack()
    E = 512
    o = torch.rand(E, 8, 47, device=DEV)
    h = torch.randn(E, 8, 64, device=DEV)
    q1, h1 = torch.empty(E, 8, 5, device=DEV), torch.empty(E, 8, 64, device=DEV)
    ops.agent_q_fwd(packed, dims(net), o, h, h1, q1)
    q2, h2 = torch.zeros_like(q1), torch.zeros_like(h1)
    gph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(gph):
            ops.agent_q_fwd(packed, dims(net), o, h, h2, q2)
    torch.cuda.current_stream().wait_stream(s)
    gph.replay()
    torch.cuda.synchronize()
    assert torch.equal(q1, q2) and torch.equal(h1, h2)


def _mixer_golden(golden):
    from minimarl.learner import Mixer
    fx = golden("mixnet")
    B, N, D = fx["obs"].shape
    mix = Mixer(N, N * D, 32, 32, DEV)
    mix.load_reference_state({k[2:]: fx[k] for k in fx if k.startswith("p.")})
    M = nets.mixer_from_state({k[2:]: fx[k] for k in fx if k.startswith("p.")})
    return fx, mix, M, B, N, D


def test_qmix_mixer_ops_golden_and_autograd(ops, golden):
    """qmix_mixer_fwd = Mix_Net.forward (qmix/_network.py:199-217) on the reference's golden inputs;
    qmix_mixer_bwd = torch autograd of the oracle mixer for an arbitrary dQ_tot and incoming hidden
    gradient (dropped on 'done' rows): dQ_i, dh and every Mix_Net parameter gradient.
    Tolerances: forward rtol 1e-5; gradients |g - g_ref| <= 1e-5 * max|g_ref| + 1e-4 * |g_ref|."""
    from minimarl.learner import MIX_KEYS
    fx, mix, M, B, N, D = _mixer_golden(golden)
    dims = [N, N * D, 32, 32]
    state = torch.from_numpy(fx["obs"]).reshape(B, N * D).to(DEV)
    q = torch.from_numpy(fx["q"]).to(DEV)
    h = torch.from_numpy(fx["hidden"]).to(DEV)
    qtot, h2 = torch.empty(B, device=DEV), torch.empty(B, 32, device=DEV)
    save = torch.empty(B, ops_save_dim(N), device=DEV)
    ops.qmix_mixer_fwd(mix.flat, dims, q, state, h, None, qtot, h2, save)
    np.testing.assert_allclose(qtot.cpu().numpy(), fx["q_tot"][:, 0], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(h2.cpu().numpy(), fx["next_hidden"], rtol=1e-5, atol=1e-5)
    g = torch.Generator().manual_seed(9)
    dqt = torch.randn(B, generator=g)
    dh_next = torch.randn(B, 32, generator=g)
    drop = (torch.rand(B, generator=g) < 0.25).float()
    # oracle autograd: d/dparams of sum(dqt * Q_tot) + sum(dh_next * (1 - drop) * h')
    Mg = {k: v.clone().requires_grad_(True) for k, v in M.items()}
    qg = torch.from_numpy(fx["q"]).clone().requires_grad_(True)
    hg = torch.from_numpy(fx["hidden"]).clone().requires_grad_(True)
    qt_ref, h_ref = nets.mixer_forward(Mg, qg, torch.from_numpy(fx["obs"]), hg)
    obj = (qt_ref.view(B) * dqt).sum() + (h_ref * dh_next * (1 - drop).view(B, 1)).sum()
    grads = torch.autograd.grad(obj, [qg, hg] + [Mg[k] for k in MIX_KEYS])
    dh = dh_next.clone().to(DEV)
    dq = torch.empty(B, N, device=DEV)
    dP = torch.empty_like(mix.flat)
    ws = torch.empty(ops.qmix_mixer_workspace(dims, B), device=DEV)
    ops.qmix_mixer_bwd(mix.flat, dims, state, save, q, dqt.to(DEV), drop.to(DEV), dh, dq, dP, ws)
    torch.cuda.synchronize()

    def close(a, b, what):
        b = b.detach().numpy()
        np.testing.assert_array_less(np.abs(a - b), 1e-5 * np.abs(b).max() + 1e-4 * np.abs(b) + 1e-12, err_msg=what)

    close(dq.cpu().numpy(), grads[0], "dq")
    close(dh.cpu().numpy(), grads[1], "dh")
    for k, gr in zip(MIX_KEYS, grads[2:]):
        close(mix.view(k, dP).cpu().numpy(), gr, k)


def ops_save_dim(N, Hm=32, K1=32):
    return 6 * Hm + N * K1 + 4 * K1 + 1


@pytest.mark.parametrize("mode", ["qmix", "vdn"])
def test_td_target_loss_and_vdn_sum_golden(ops, golden, mode):
    """td_target_loss (+ vdn_sum for VDN) on the Q_tot sequences of the reference's golden update, recomputed
    by the oracle nets from the golden weights and batch: the loss and the new priorities equal the
    reference's (qmix/_train.py:75-84,118-121; vdn/_train.py:73-79,96-99), rtol 1e-4; dQ_tot = 2 (Q_tot - y) / B."""
    fx = golden(mode + "_train")
    s, a, r, s2, d = (torch.from_numpy(fx[k]) for k in ("states", "actions", "rewards", "next_states", "dones"))
    B, C, N, D = s.shape
    style = "qmix" if mode == "qmix" else "vdn"
    pre = ("before_q.", "target_q.") if mode == "qmix" else ("before.", "target.")
    P, T = nets.agent_from_state(fx, pre[0], style), nets.agent_from_state(fx, pre[1], style)
    H = P["Whh"].shape[2]
    h, ht = torch.zeros(B, N, H), torch.zeros(B, N, H)
    qtot, qtot_t = torch.empty(C, B, device=DEV), torch.empty(C, B, device=DEV)
    if mode == "qmix":
        M, TM = nets.mixer_from_state(fx, "before_m."), nets.mixer_from_state(fx, "target_m.")
        hm, hmt = torch.zeros(B, 32), torch.zeros(B, 32)
    with torch.no_grad():
        for t in range(C):
            q, nh = nets.agent_forward(P, s[:, t], h)
            tq, nht = nets.agent_forward(T, s2[:, t], ht)
            if mode == "qmix":
                qa = q.gather(2, a[:, t].unsqueeze(-1).long()).squeeze(-1)
                qt_, nhm = nets.mixer_forward(M, qa, s[:, t], hm)
                tt_, nhmt = nets.mixer_forward(TM, tq.max(2)[0], s2[:, t], hmt)
                qtot[t], qtot_t[t] = qt_.view(B).to(DEV), tt_.view(B).to(DEV)
                hm, hmt = nhm * (1 - d[:, t]), nhmt * (1 - d[:, t])
            else:     # the VDN mixer on the device: sum_i Q_i(a_i) and sum_i max_a Q'_i
                ops.vdn_sum(q.contiguous().to(DEV), a[:, t].to(torch.int32).to(DEV), qtot[t])
                ops.vdn_sum(tq.contiguous().to(DEV), None, qtot_t[t])
                torch.cuda.synchronize()
                ref = q.gather(2, a[:, t].unsqueeze(-1).long()).squeeze(-1).sum(1)
                np.testing.assert_allclose(qtot[t].cpu().numpy(), ref.numpy(), rtol=1e-6, atol=1e-6)
                np.testing.assert_allclose(qtot_t[t].cpu().numpy(), tq.max(2)[0].sum(1).numpy(), rtol=1e-6, atol=1e-6)
            keep = (1 - d[:, t]).view(B, 1, 1)
            h, ht = nh * keep, nht * keep
    rew = r.permute(1, 0, 2).contiguous().to(DEV)                 # [C, B, N]
    done = d.view(B, C).t().contiguous().to(DEV)
    isw = torch.from_numpy(fx["is_weight"]).view(B).to(DEV)
    dqt, td_last = torch.empty(C, B, device=DEV), torch.empty(B, device=DEV)
    loss, parts = torch.empty(1, device=DEV), torch.empty(C, B, device=DEV)
    ops.td_target_loss(rew, done, isw, qtot, qtot_t, float(fx["gamma"]), 0, dqt, td_last, loss, parts)
    torch.cuda.synchronize()
    np.testing.assert_allclose(float(loss), float(fx["loss"]), rtol=1e-4)
    np.testing.assert_allclose(td_last.cpu().numpy(), fx["new_td"], rtol=1e-4, atol=1e-4)
    w = isw.view(1, B)
    y = w * (rew.sum(2) + N * float(fx["gamma"]) * (1 - done) * qtot_t)
    np.testing.assert_allclose(dqt.cpu().numpy(), (2 * (qtot - y) / B).cpu().numpy(), rtol=1e-4, atol=1e-6)
    with pytest.raises(RuntimeError, match="vdn_sum"):
        ops.td_target_loss(rew, done, isw, qtot, qtot_t, 0.99, 1, dqt, td_last, loss, parts)


def _mappo_policy(fx):
    from minimarl.mappo import MappoPolicy
    D = fx["obs"].shape[1]
    pol = MappoPolicy(D, 5, 32, DEV)
    pol.actor.load_reference_state(fx, "actor.")
    pol.critic.load_reference_state(fx, "critic.")
    return pol, D


def test_mappo_ops_golden(ops, golden):
    """mappo_get_actions / mappo_evaluate_actions (R_MAPPOPolicy.get_actions / act / evaluate_actions,
    rmappo_policy.py:57-136: MLPBase -> masked GRU -> LayerNorm -> Categorical, critic value) vs the
    reference's golden outputs: values, hiddens, log-probs, the recurrent minibatch's values / log-probs /
    masked entropy, rtol 1e-5; sampled actions = the oracle's inverse-CDF sampler on the same injected
    uniforms; deterministic actions = the argmax."""
    from oracle import mappo as om
    fx = golden("mappo_fwd")
    pol, D = _mappo_policy(fx)
    dims = [D, 32, 5]
    t = lambda k: torch.from_numpy(fx[k]).contiguous()  # noqa: E731
    R = fx["obs"].shape[0]
    obs, ha, hc, m = t("obs").to(DEV), t("ha").view(R, 32).to(DEV), t("hc").view(R, 32).to(DEV), t("masks").view(R).to(DEV)
    u = torch.rand(R, generator=torch.Generator().manual_seed(3))
    ha2, hc2 = torch.empty(R, 32, device=DEV), torch.empty(R, 32, device=DEV)
    act = torch.empty(R, dtype=torch.int32, device=DEV)
    lp, v = torch.empty(R, device=DEV), torch.empty(R, device=DEV)
    ops.mappo_get_actions(pol.actor.flat, pol.critic.flat, dims, obs, ha, hc, m, u.to(DEV), 0, 0, False, ha2, hc2, act,
                          lp, v)
    torch.cuda.synchronize()
    np.testing.assert_allclose(v.cpu().numpy(), fx["values"][:, 0], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(ha2.cpu().numpy(), fx["ha_out"][:, 0], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(hc2.cpu().numpy(), fx["hc_out"][:, 0], rtol=1e-5, atol=2e-6)
    PA = om.net_from_state(fx, "actor.", "actor")
    logits, _ = om.net_step(PA, t("obs"), t("ha")[:, 0], t("masks"))
    np.testing.assert_array_equal(act.cpu().numpy(), om.sample_actions(logits, u).numpy())
    lpo = torch.log_softmax(logits, -1).gather(1, act.cpu().long().view(-1, 1))
    np.testing.assert_allclose(lp.cpu().numpy(), lpo[:, 0].numpy(), rtol=1e-5, atol=2e-6)
    ops.mappo_get_actions(pol.actor.flat, pol.critic.flat, dims, obs, ha, hc, m, None, 0, 0, True, ha2, hc2, act, lp, v)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(act.cpu().numpy(), logits.argmax(-1).numpy())
    # the recurrent minibatch: n chunks of L steps, masks zero inside chunks (RNNLayer segments)
    L, n = int(fx["seq_L"]), int(fx["seq_n"])
    rows = L * n
    vals, lps, ent = torch.empty(rows, device=DEV), torch.empty(rows, device=DEV), torch.empty(1, device=DEV)
    ws = torch.empty(ops.mappo_evaluate_workspace(dims, rows), device=DEV)
    ops.mappo_evaluate_actions(pol.actor.flat, pol.critic.flat, dims, t("seq_obs").to(DEV),
                               t("seq_ha").view(n, 32).to(DEV), t("seq_hc").view(n, 32).to(DEV),
                               t("seq_actions").view(rows).to(torch.int32).to(DEV), t("seq_masks").view(rows).to(DEV),
                               t("seq_active").view(rows).to(DEV), L, vals, lps, ent, ws)
    torch.cuda.synchronize()
    np.testing.assert_allclose(vals.cpu().numpy(), fx["seq_values"][:, 0], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(lps.cpu().numpy(), fx["seq_logp"][:, 0], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(float(ent), float(fx["seq_entropy"]), rtol=1e-5)


def test_new_ops_capture_in_hip_graph(ops, golden):
    """The mixer forward + backward, TD loss, VDN sum and the MAPPO pair captured in ONE HIP graph (all
    enqueued on torch's current stream, caller-allocated outputs, no host sync) replay bit-identically to
    their eager launches."""
    fx, mix, M, B, N, D = _mixer_golden(golden)
    dims = [N, N * D, 32, 32]
    state = torch.from_numpy(fx["obs"]).reshape(B, N * D).to(DEV)
    q, h = torch.from_numpy(fx["q"]).to(DEV), torch.from_numpy(fx["hidden"]).to(DEV)
    reset = (torch.arange(B, device=DEV) % 5 == 0).to(torch.uint8)
    dqt, drop = torch.randn(B, device=DEV), (torch.arange(B, device=DEV) % 3 == 0).float()
    dh0 = torch.randn(B, 32, device=DEV)
    qv = torch.randn(B, N, 5, device=DEV)
    av = torch.randint(0, 5, (B, N), device=DEV, dtype=torch.int32)
    C = 3
    rew, done = torch.randn(C, B, N, device=DEV), (torch.rand(C, B, device=DEV) < 0.2).float()
    fm = golden("mappo_fwd")
    pol, Dm = _mappo_policy(fm)
    tm = {k: torch.from_numpy(fm[k]).contiguous().to(DEV) for k in ("obs", "ha", "hc", "masks", "seq_obs", "seq_ha",
                                                                    "seq_hc", "seq_masks", "seq_active")}
    seq_act = torch.from_numpy(fm["seq_actions"]).view(-1).to(torch.int32).to(DEV)
    Rm = fm["obs"].shape[0]
    L, n = int(fm["seq_L"]), int(fm["seq_n"])
    ws_m = torch.empty(ops.mappo_evaluate_workspace([Dm, 32, 5], L * n), device=DEV)
    ws = torch.empty(ops.qmix_mixer_workspace(dims, B), device=DEV)

    def outs():
        return dict(qtot=torch.empty(B, device=DEV), h2=torch.empty(B, 32, device=DEV),
                    save=torch.empty(B, ops_save_dim(N), device=DEV), dh=torch.empty(B, 32, device=DEV),
                    dq=torch.empty(B, N, device=DEV), dP=torch.empty_like(mix.flat), vs=torch.empty(B, device=DEV),
                    dqt=torch.empty(C, B, device=DEV), tdl=torch.empty(B, device=DEV), loss=torch.empty(1, device=DEV),
                    parts=torch.empty(C, B, device=DEV), ha2=torch.empty(Rm, 32, device=DEV),
                    hc2=torch.empty(Rm, 32, device=DEV), act=torch.empty(Rm, dtype=torch.int32, device=DEV),
                    lp=torch.empty(Rm, device=DEV), v=torch.empty(Rm, device=DEV),
                    sv=torch.empty(L * n, device=DEV), slp=torch.empty(L * n, device=DEV),
                    sent=torch.empty(1, device=DEV), qt3=torch.empty(C, B, device=DEV))

    def run(o):
        ops.qmix_mixer_fwd(mix.flat, dims, q, state, h, reset, o["qtot"], o["h2"], o["save"])
        o["dh"].copy_(dh0)
        ops.qmix_mixer_bwd(mix.flat, dims, state, o["save"], q, dqt, drop, o["dh"], o["dq"], o["dP"], ws)
        ops.vdn_sum(qv, av, o["vs"])
        o["qt3"].copy_(o["qtot"].view(1, B).expand(C, B))
        ops.td_target_loss(rew, done, None, o["qt3"], o["qt3"], 0.99, 4, o["dqt"], o["tdl"], o["loss"], o["parts"])
        ops.mappo_get_actions(pol.actor.flat, pol.critic.flat, [Dm, 32, 5], tm["obs"], tm["ha"].view(Rm, 32),
                              tm["hc"].view(Rm, 32), tm["masks"].view(Rm), None, 7, 11, False, o["ha2"], o["hc2"],
                              o["act"], o["lp"], o["v"])
        ops.mappo_evaluate_actions(pol.actor.flat, pol.critic.flat, [Dm, 32, 5], tm["seq_obs"], tm["seq_ha"].view(n, 32),
                                   tm["seq_hc"].view(n, 32), seq_act, tm["seq_masks"].view(-1),
                                   tm["seq_active"].view(-1), L, o["sv"], o["slp"], o["sent"], ws_m)

    eager = outs()
    run(eager)
    torch.cuda.synchronize()
    cap = outs()
    gph = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        with torch.cuda.graph(gph):
            run(cap)
    torch.cuda.current_stream().wait_stream(st)
    gph.replay()
    torch.cuda.synchronize()
    for k in eager:
        assert torch.equal(eager[k], cap[k]), k
