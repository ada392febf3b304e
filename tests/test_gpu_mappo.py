"""GPU parity of the MAPPO HIP path (csrc/mappo.hip via minimarl.mappo) against the reference's
golden vectors (tests/golden/mappo_*.npz) and the oracle (oracle/mappo.py).

Tolerances (fp32; the device uses hardware exp/rcp for the GRU gates, ~1e-6 relative):
values / log-probs / hiddens rtol 1e-5 atol 2e-6; returns rtol 1e-6.

Training (gradients, post-Adam parameters, loss logs) is held to a bar DERIVED per test from the oracle on
the same data (``_fp32_spread``): the oracle is run three times, in fp32 in the device's chunk order, in fp32
in a random chunk order (the reference's randperm) and in float64; per tensor, the fp32 spread is
max(|fp32 chunk - fp32 permuted|, |fp32 - f64|, 2^-23 max|f64|) (inf-norm), i.e. how far two legitimate fp32
evaluations of the same sums land from each other and from the exact value. The device (different summation
trees: MFMA k-accumulation, 128 block partials; hardware exp / rcp) must land within K_FP32 = 16 spreads of
the f64 value. Measured spreads are ~1e-7 .. 8e-7 of a tensor's max at the golden size and at 512 x 8 x 100
(tools/mappo_tol.py), so the bars are ~1e-5 of max|g| instead of the round-3 fixed 1e-3 .. 2e-3.
"""
import numpy as np
import pytest
import torch

from oracle import mappo as om

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = dict(rtol=1e-5, atol=2e-6)
K_FP32 = 16


def _ppo_oracle(PA, PC, data, vn0, epochs, L, dtype=torch.float32, perms=None):
    """om.ppo_train in the given float dtype (params, buffer and ValueNorm cast); -> (record, PA2, PC2, vn2)."""
    old = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        npd = np.float64 if dtype == torch.float64 else np.float32
        d = {k: (v.astype(npd) if v.dtype in (np.float32, np.float64) else v) for k, v in data.items()}
        pa = {k: torch.as_tensor(v).to(dtype) for k, v in PA.items()}
        pc = {k: torch.as_tensor(v).to(dtype) for k, v in PC.items()}
        rec = []
        PA2, PC2, vn2 = om.ppo_train(pa, pc, d, om.ValueNorm(*vn0), epochs, L, perms=perms, record=rec)
    finally:
        torch.set_default_dtype(old)
    return rec, PA2, PC2, vn2


def _fp32_spread(f, n_chunks):
    """f(dtype, perms) -> {name: array}; -> (f64 values, {name: fp32 spread}) (module docstring)."""
    a = f(torch.float32, None)
    b = f(torch.float32, np.random.default_rng(123).permutation(n_chunks)[None].repeat(64, 0))
    c = f(torch.float64, None)
    sp = {}
    for k in c:
        x, y, z = (np.asarray(v[k], np.float64) for v in (a, b, c))
        sp[k] = max(np.abs(x - y).max(), np.abs(x - z).max(), 2.0 ** -23 * np.abs(z).max(), 1e-30)
    return c, sp


def _ppo_oracle_self_old(PA, PC, data, vn0, epochs, L, dtype=torch.float32):
    """The oracle with the rollout's old log-probs / values replaced by its OWN epoch-0 training forward
    (evaluate_chunks on the same chunk batch): its epoch-0 ratio is then exactly 1, as on the device, whose rollout
    and training forwards are the same MFMA code (so the device's old log-probs carry no rounding the training
    forward does not share). -> _train_outputs of that run."""
    old = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        npd = np.float64 if dtype == torch.float64 else np.float32
        d = {k: (v.astype(npd) if v.dtype in (np.float32, np.float64) else v) for k, v in data.items()}
        PA2 = {k: torch.as_tensor(v).to(dtype) for k, v in PA.items()}
        PC2 = {k: torch.as_tensor(v).to(dtype) for k, v in PC.items()}
        vn = om.ValueNorm(*vn0)
        adv = om.normalized_advantages(d, vn)
        b = om.chunk_batch(d, adv, L, None)
        with torch.no_grad():
            lp, _ = om.evaluate_chunks(PA2, b["obs"], b["ha0"], b["masks"], L, "actor", b["actions"],
                                       b["active_masks"])
            v = om.evaluate_chunks(PC2, b["obs"], b["hc0"], b["masks"], L, "critic")
        b["action_log_probs"], b["value_preds"] = lp.detach(), v.detach()
        sa, sc, rec = {}, {}, []
        for _ in range(epochs):
            pa = {k: t.detach().clone().requires_grad_(True) for k, t in PA2.items()}
            pc = {k: t.detach().clone().requires_grad_(True) for k, t in PC2.items()}
            vn.update(b["returns"])
            pol, ent, vloss, _ = om.ppo_losses(pa, pc, b, L, vn, entropy_coef=0.01)
            ga = torch.autograd.grad(pol - ent * 0.01, [pa[k] for k in om.NET_KEYS])
            gc = torch.autograd.grad(vloss * 0.5, [pc[k] for k in om.NET_KEYS])
            ga, na = om.clip_grads(list(ga), 0.5)
            gc, nc = om.clip_grads(list(gc), 0.5)
            rec.append(dict(ga=dict(zip(om.NET_KEYS, ga)), gc=dict(zip(om.NET_KEYS, gc)), na=float(na), nc=float(nc),
                            pol=float(pol.detach()), ent=float(ent.detach()), vloss=float(vloss.detach())))
            PA2 = om.adam(PA2, dict(zip(om.NET_KEYS, ga)), sa, 1e-4, 1e-5)
            PC2 = om.adam(PC2, dict(zip(om.NET_KEYS, gc)), sc, 1e-4, 1e-5)
    finally:
        torch.set_default_dtype(old)
    return _train_outputs(rec, PA2, PC2, vn)


def _unclipped_grads(rec, ep=0):
    """{(net, key): gradient before clip_grad_norm_} of epoch ep of an om.ppo_train record."""
    out = {}
    for n, tag, nk in ((0, "ga", "na"), (1, "gc", "nc")):
        coef = min(1.0, 0.5 / (rec[ep][nk] + 1e-6))
        for k in om.NET_KEYS:
            out[(n, k)] = rec[ep][tag][k].double().numpy() / coef
    return out


def _assert_within(got, want, spread, what):
    err = float(np.abs(np.asarray(got, np.float64) - want).max())
    assert err <= K_FP32 * spread, f"{what}: |dev - f64| = {err:.3e} > {K_FP32} x spread {spread:.3e}"


def _policy(fx, prefix=""):
    from minimarl.mappo import MappoPolicy
    D = fx[prefix + "actor.base.feature_norm.weight"].shape[0]
    A = fx[prefix + "actor.act.action_out.linear.bias"].shape[0]
    p = MappoPolicy(D, A, 32, DEV)
    p.actor.load_reference_state(fx, prefix + "actor.")
    p.critic.load_reference_state(fx, prefix + "critic.")
    return p


def _soa_field(buf, nf, f, rows):
    return buf.view(-1, nf, 64)[:, f, :].reshape(-1)[:rows]


def test_get_actions_matches_reference(golden):
    fx = golden("mappo_fwd")
    p = _policy(fx)
    t = lambda k: torch.from_numpy(fx[k]).to(DEV)
    v, a, lp, ha, hc = p.get_actions(t("obs"), t("ha")[:, 0], t("hc")[:, 0], t("masks"), actions=t("actions"))
    torch.cuda.synchronize()
    np.testing.assert_allclose(v.cpu().numpy(), fx["values"], **TOL)
    np.testing.assert_allclose(lp.cpu().numpy(), fx["logp"], **TOL)
    np.testing.assert_allclose(ha.cpu().numpy(), fx["ha_out"][:, 0], **TOL)
    np.testing.assert_allclose(hc.cpu().numpy(), fx["hc_out"][:, 0], **TOL)


def test_sampler_matches_oracle(golden):
    fx = golden("mappo_fwd")
    p = _policy(fx)
    PA = om.net_from_state(fx, "actor.", "actor")
    PC = om.net_from_state(fx, "critic.", "critic")
    rng = np.random.default_rng(5)
    R = 4096
    obs = torch.from_numpy(np.concatenate([fx["obs"]] * (R // fx["obs"].shape[0] + 1))[:R].copy())
    obs[:, :2] = torch.rand(R, 2, generator=torch.Generator().manual_seed(3))
    ha = torch.from_numpy(rng.standard_normal((R, 32)).astype(np.float32) * 0.5)
    hc = torch.from_numpy(rng.standard_normal((R, 32)).astype(np.float32) * 0.5)
    m = torch.from_numpy((rng.random(R) > 0.1).astype(np.float32))
    u = torch.from_numpy(rng.random(R).astype(np.float32))
    v, a, lp, ha2, hc2 = p.get_actions(obs.to(DEV), ha.to(DEV), hc.to(DEV), m.to(DEV), u=u.to(DEV))
    torch.cuda.synchronize()
    vo, ao, lpo, hao, hco = om.get_actions(PA, PC, obs, ha, hc, m.view(-1, 1), u=u)
    # the inverse CDF is discontinuous: allow disagreement only where u sits within 1e-5 of a boundary
    logits, _ = om.net_step(PA, obs, ha, m.view(-1, 1))
    c = torch.cumsum(torch.softmax(logits, -1), -1)
    near = ((c - u.view(-1, 1)).abs() < 1e-5).any(-1).numpy()
    agree = a.cpu().numpy()[:, 0] == ao.numpy()[:, 0]
    assert np.all(agree | near) and agree.mean() > 0.999
    ok = agree
    np.testing.assert_allclose(lp.cpu().numpy()[ok], lpo.numpy()[ok], **TOL)
    np.testing.assert_allclose(v.cpu().numpy(), vo.numpy(), **TOL)
    np.testing.assert_allclose(ha2.cpu().numpy(), hao.numpy(), **TOL)
    # every action occurs (u uniform, near-uniform policy at gain 0.01)
    assert len(np.unique(a.cpu().numpy())) == 5


def test_device_rng_sampling_rate():
    from minimarl.mappo import MappoPolicy
    p = MappoPolicy(47, 5, 32, DEV, seed=3)
    R = 1 << 16
    obs = torch.rand(R, 47, device=DEV)
    h = torch.zeros(R, 32, device=DEV)
    _, a, lp, _, _ = p.get_actions(obs, h, h, None, seed=11, counter=7)
    # Wo gain 0.01 -> probabilities ~0.2 each: empirical frequencies within 1.5% (binomial 6 sigma)
    freq = torch.bincount(a.view(-1).long(), minlength=5).float().cpu().numpy() / R
    probs = torch.exp(lp).mean().item()
    assert np.all(np.abs(freq - 0.2) < 0.015), freq
    assert 0.15 < probs < 0.25
    _, a2, _, _, _ = p.get_actions(obs, h, h, None, seed=11, counter=8)
    assert (a2 != a).float().mean().item() > 0.5      # a new counter draws new samples


def test_train_forward_chunks_match_reference(golden):
    """Training path (rnn.py:30-77 masked segments) on L-step chunks from stored hiddens."""
    from minimarl.mappo import MappoBuffer, MappoTrainer
    from minimarl._lib import lib
    fx = golden("mappo_fwd")
    p = _policy(fx)
    L, n = int(fx["seq_L"]), int(fx["seq_n"])
    buf = MappoBuffer(L, n, 1, p.D, 32, DEV)
    buf.obs[:L] = torch.from_numpy(fx["seq_obs"].reshape(L, n, -1)).to(DEV)
    buf.masks[:L] = torch.from_numpy(fx["seq_masks"].reshape(L, n)).to(DEV)
    buf.rnn_states[0] = torch.from_numpy(fx["seq_ha"][:, 0]).to(DEV)
    buf.rnn_states_critic[0] = torch.from_numpy(fx["seq_hc"][:, 0]).to(DEV)
    tr = MappoTrainer(p, L, n, L=L, ppo_epoch=1, fused=False)
    import ctypes
    fa = tr.fwd_args(buf)
    assert lib().mm_mappo_fwd(ctypes.byref(p.dims), ctypes.byref(fa), None) == 0
    torch.cuda.synchronize()
    ns0 = lib().mm_mappo_save_fields(ctypes.byref(p.dims), 0)
    ns1 = lib().mm_mappo_save_fields(ctypes.byref(p.dims), 1)
    rows = L * n
    logp_all = torch.stack([_soa_field(tr.save[0], ns0, ns0 - 5 + q, rows) for q in range(5)], -1).cpu()
    act = torch.from_numpy(fx["seq_actions"]).long().view(-1)
    lp = logp_all.gather(-1, act.view(-1, 1)).numpy()
    val = _soa_field(tr.save[1], ns1, ns1 - 1, rows).cpu().numpy()
    np.testing.assert_allclose(lp, fx["seq_logp"], **TOL)
    np.testing.assert_allclose(val, fx["seq_values"][:, 0], **TOL)
    ent = -(logp_all.exp() * logp_all).sum(-1)
    act_m = torch.from_numpy(fx["seq_active"]).view(-1)
    np.testing.assert_allclose(float((ent * act_m).sum() / act_m.sum()), float(fx["seq_entropy"]), rtol=1e-5)


def test_gae_matches_reference(golden):
    from minimarl.mappo import MappoBuffer, MappoPolicy, MappoTrainer
    fx = golden("mappo_gae")
    T, E, N = fx["rewards"].shape[:3]
    buf = MappoBuffer(T, E, N, 47, 32, DEV)
    buf.rewards.copy_(torch.from_numpy(fx["rewards"].reshape(T, E * N)))
    vp = fx["value_preds"].copy()
    vp[-1] = fx["next_value"]
    buf.value_preds.copy_(torch.from_numpy(vp.reshape(T + 1, E * N)))
    buf.masks.copy_(torch.from_numpy(fx["masks"].reshape(T + 1, E * N)))
    vn = torch.tensor([float(fx["vn_mean"][0]), float(fx["vn_mean_sq"][0]), float(fx["vn_debias"])],
                      dtype=torch.float32, device=DEV)
    buf.compute_returns(vn, float(fx["gamma"]), float(fx["gae_lambda"]))
    torch.cuda.synchronize()
    np.testing.assert_allclose(buf.returns[:T].cpu().numpy(), fx["returns"][:T].reshape(T, E * N), rtol=1e-6,
                               atol=1e-6)


def _trainer_from_fixture(fx, fused=True):
    from minimarl.mappo import MappoBuffer, MappoTrainer
    p = _policy(fx, "before.")
    E, N, T, L = (int(fx[k]) for k in ("E", "N", "T", "L"))
    buf = MappoBuffer(T, E, N, p.D, 32, DEV)
    buf.load_reference({k[5:]: fx[k] for k in fx if k.startswith("data.")})
    tr = MappoTrainer(p, T, E * N, L=L, ppo_epoch=int(fx["epochs"]), fused=fused)
    tr.load_value_normalizer(float(fx["vn0.running_mean"][0]), float(fx["vn0.running_mean_sq"][0]),
                             float(fx["vn0.debiasing_term"]))
    return p, buf, tr


def _golden_oracle_inputs(fx):
    sd = {k[len("before."):]: fx[k] for k in fx if k.startswith("before.")}
    PA, PC = om.net_from_state(sd, "actor.", "actor"), om.net_from_state(sd, "critic.", "critic")
    data = {k[5:]: fx[k] for k in fx if k.startswith("data.")}
    vn0 = (float(fx["vn0.running_mean"][0]), float(fx["vn0.running_mean_sq"][0]), float(fx["vn0.debiasing_term"]))
    n_chunks = int(fx["T"]) * int(fx["E"]) * int(fx["N"]) // int(fx["L"])
    return PA, PC, data, vn0, n_chunks


@pytest.mark.parametrize("fused", [True, False], ids=["fused_mfma", "saves_wgrad"])
def test_first_epoch_gradients_match_reference(golden, fused):
    """Unclipped gradients of PPO epoch 0: the fused MFMA pass (mm_mappo_grad, a partial tile of chunks) and
    the saves + wgrad path, each tensor within K_FP32 fp32 spreads (module docstring) of the f64 oracle, and the
    reference's own fp32 gradients (golden, clipped -> divided by its clip coefficient) within the same bar
    plus their own distance to f64."""
    from minimarl._lib import lib
    fx = golden("mappo_train")
    p, buf, tr = _trainer_from_fixture(fx, fused)
    PA, PC, data, vn0, nch = _golden_oracle_inputs(fx)
    L = int(fx["L"])
    g64, spread = _fp32_spread(lambda dt, pm: _unclipped_grads(_ppo_oracle(PA, PC, data, vn0, 1, L, dt, pm)[0]), nch)
    tr.prepare(buf)
    assert lib().mm_mappo_vn_update(tr.vn.data_ptr(), tr.stats.data_ptr(), 0.99999, None) == 0
    if fused:
        tr.grad[0].fill_(float("nan"))      # the fused pass writes every entry (pads included)
        tr.grad[1].fill_(float("nan"))
    tr.gradients(buf)
    torch.cuda.synchronize()
    for n, (net, tag) in enumerate(((p.actor, "a"), (p.critic, "c"))):
        coef = min(1.0, 0.5 / (float(fx["norms"][n]) + 1e-6))
        kind = "actor" if n == 0 else "critic"
        for k in om.NET_KEYS:
            g = net.view(k, tr.grad[n]).cpu().numpy()
            ref = fx[f"grad{tag}0.{om.ref_name(k, kind)}"] / coef
            _assert_within(g, g64[(n, k)], spread[(n, k)], f"{kind} {k} vs f64")
            ref_err = float(np.abs(ref - g64[(n, k)]).max())
            assert np.abs(g - ref).max() <= K_FP32 * spread[(n, k)] + ref_err, f"{kind} {k} vs golden"
        # pads of the flat layout carry zero gradient
        assert float(tr.grad[n].abs().sum()) == pytest.approx(
            sum(float(net.view(k, tr.grad[n]).abs().sum()) for k in om.NET_KEYS), rel=1e-6)


def _train_outputs(rec, PA2, PC2, vn2):
    """post-train parameters and the train() log of an om.ppo_train run (R_MAPPO.train averages the per-epoch
    losses / norms, ramppo_network.py:245-287)"""
    out = {("actor", k): PA2[k].double().numpy() for k in om.NET_KEYS}
    out.update({("critic", k): PC2[k].double().numpy() for k in om.NET_KEYS})
    E = len(rec)
    out["value_loss"] = np.array(sum(r["vloss"] for r in rec) / E)
    out["policy_loss"] = np.array(sum(r["pol"] for r in rec) / E)
    out["dist_entropy"] = np.array(sum(r["ent"] for r in rec) / E)
    out["actor_grad_norm"] = np.array(sum(r["na"] for r in rec) / E)
    out["critic_grad_norm"] = np.array(sum(r["nc"] for r in rec) / E)
    out["vn_mean"] = vn2.m.double().numpy()
    out["vn_mean_sq"] = vn2.msq.double().numpy()
    return out


@pytest.mark.parametrize("fused", [True, False], ids=["fused_mfma", "saves_wgrad"])
def test_ppo_train_matches_reference(golden, fused):
    """The golden train() (3 epochs): post-Adam parameters, ValueNorm state and the train_info log within K_FP32
    fp32 spreads of the f64 oracle (a parameter's spread includes Adam's sign sensitivity: a near-zero gradient
    whose sign differs between two fp32 orders moves the coordinate by ~lr either way, and the permuted fp32
    run shows exactly that); and within the same bar plus the reference's own fp32 distance of its golden
    values. The mean ratio is identically 1 at epoch 0 and tested at rtol 1e-5."""
    fx = golden("mappo_train")
    p, buf, tr = _trainer_from_fixture(fx, fused)
    PA, PC, data, vn0, nch = _golden_oracle_inputs(fx)
    EP, L = int(fx["epochs"]), int(fx["L"])
    o64, spread = _fp32_spread(lambda dt, pm: _train_outputs(*_ppo_oracle(PA, PC, data, vn0, EP, L, dt, pm)), nch)
    info = tr.train(buf)
    torch.cuda.synchronize()
    for net, kind in ((p.actor, "actor"), (p.critic, "critic")):
        for k in om.NET_KEYS:
            got = net.view(k).cpu().numpy()
            after = fx[f"after.{kind}.{om.ref_name(k, kind)}"]
            _assert_within(got, o64[(kind, k)], spread[(kind, k)], f"{kind} {k} vs f64")
            ref_err = float(np.abs(after - o64[(kind, k)]).max())
            assert np.abs(got - after).max() <= K_FP32 * spread[(kind, k)] + ref_err, f"{kind} {k} vs golden"
    vn = tr.value_normalizer_state()
    _assert_within(vn["running_mean"], o64["vn_mean"], spread["vn_mean"], "vn mean")
    _assert_within(vn["running_mean_sq"], o64["vn_mean_sq"], spread["vn_mean_sq"], "vn mean_sq")
    for key in ("value_loss", "policy_loss", "dist_entropy", "actor_grad_norm", "critic_grad_norm"):
        _assert_within(info[key], o64[key], spread[key], key)
        ref_err = abs(float(fx["info." + key]) - float(o64[key]))
        assert abs(info[key] - float(fx["info." + key])) <= K_FP32 * spread[key] + ref_err, key
    np.testing.assert_allclose(info["ratio"], float(fx["info.ratio"]), rtol=1e-5)


def test_runner_episode_end_to_end():
    """Rollout (env kernel + fused actor/critic + insert) -> GAE -> 2 PPO epochs on device; checks
    the buffer against the oracle env and a CPU recomputation of the GAE."""
    from minimarl.env import VecEnv
    from minimarl.mappo import MappoPolicy, MappoRunner
    E, N, T = 64, 8, 20
    env = VecEnv(E, N, max_steps=12, device=DEV)
    p = MappoPolicy(env.obs_dim, 5, 32, DEV, seed=0)
    r = MappoRunner(env, p, T=T, L=5, ppo_epoch=2, seed=1)
    r.warmup()
    r.rollout()
    r.compute()
    torch.cuda.synchronize()
    b = r.buf
    masks = b.masks.cpu().numpy()
    # max_steps 12: every env finishes at t = 11 (or earlier when the apples run out)
    assert masks[12].sum() < E * N and np.all(masks[0] == 1)
    # zeroed hiddens exactly where the env finished
    hz = b.rnn_states.abs().sum(-1).cpu().numpy() == 0
    assert np.all(hz[1:][masks[1:] == 0])
    vn = r.trainer.vn
    ret_ref, _ = om.compute_returns(b.rewards.cpu().numpy()[..., None], b.value_preds.cpu().numpy()[..., None],
                                    masks[..., None], b.value_preds[T].cpu().numpy()[..., None],
                                    om.ValueNorm(*[float(x) for x in vn.cpu().numpy()]), 0.99, 0.95)
    np.testing.assert_allclose(b.returns[:T].cpu().numpy(), ret_ref[:T, :, 0], rtol=1e-5, atol=1e-5)
    before = p.actor.flat.clone()
    info = r.train()
    torch.cuda.synchronize()
    assert all(np.isfinite(v) for v in info.values()), info
    assert float((p.actor.flat - before).abs().max()) > 0
    assert np.all(b.obs[0].cpu().numpy() == b.obs[T].cpu().numpy())


def _ref_layout(b, E, N):
    """MappoBuffer [T(+1), E*N, ...] -> the reference SharedReplayBuffer layout [T(+1), E, N, ..., 1]."""
    c = lambda t: t.detach().cpu().numpy()  # noqa: E731
    T1 = b.obs.shape[0]
    d = {"obs": c(b.obs).reshape(T1, E, N, -1),
         "rnn_states": c(b.rnn_states).reshape(T1, E, N, 1, -1),
         "rnn_states_critic": c(b.rnn_states_critic).reshape(T1, E, N, 1, -1),
         "actions": c(b.actions).astype(np.float32).reshape(T1 - 1, E, N, 1)}
    for k in ("action_log_probs", "rewards"):
        d[k] = c(getattr(b, k)).reshape(T1 - 1, E, N, 1)
    for k in ("value_preds", "returns", "masks", "active_masks"):
        d[k] = c(getattr(b, k)).reshape(T1, E, N, 1)
    return d


def test_cfg3_scale_rollout_and_epoch_gradients_vs_oracle():
    """cfg3-scale MAPPO (512 envs x 8 agents x T = 100 = 409,600 row-steps; bench.py times 4096 envs with
    the same kernels and the same tiled-SoA / multi-slice wgrad path) against the oracle:
    * rollout (magym_runner.py:114-195): every step's obs / rewards / masks bit-exact vs the env oracle
      driven with the stored actions; log-probs, values and next hiddens vs ``om.get_actions`` from the
      device's stored input hiddens (rtol 1e-5 atol 2e-6); hiddens zeroed where the env finished;
    * GAE + ValueNorm (shared_buffer.py:131-157) vs ``om.compute_returns`` (rtol 1e-5 atol 1e-5);
    * PPO epoch 0 (ramppo_network.py:103-209): every gradient of actor and critic within K_FP32 fp32 spreads
      (module docstring) of the f64 oracle's autograd on the full recurrent minibatch."""
    import ctypes
    from minimarl._lib import lib
    from minimarl.env import VecEnv
    from minimarl.mappo import MappoPolicy, MappoRunner
    from oracle.env import EnvSpec, VecEnvOracle
    E, N, T, L = 512, 8, 100, 5
    env = VecEnv(E, N, max_steps=100, device=DEV)
    p = MappoPolicy(env.obs_dim, 5, 32, DEV, seed=3)
    PA = {k: p.actor.view(k).detach().cpu().clone() for k in om.NET_KEYS}
    PC = {k: p.critic.view(k).detach().cpu().clone() for k in om.NET_KEYS}
    r = MappoRunner(env, p, T=T, L=L, ppo_epoch=1, seed=11)
    r.warmup()
    r.rollout()
    r.compute()
    torch.cuda.synchronize()
    b = r.buf
    EN = E * N
    obs, acts = b.obs.cpu().numpy(), b.actions.cpu().numpy().astype(np.int64)
    ha, hc = b.rnn_states.cpu(), b.rnn_states_critic.cpu()
    masks, rew = b.masks.cpu().numpy(), b.rewards.cpu().numpy()
    ora = VecEnvOracle(EnvSpec(N, 100), E)
    np.testing.assert_array_equal(obs[0].reshape(E, N, -1), ora.observe())
    for t in range(T):
        _, rw, dn = ora.step(acts[t].reshape(E, N))
        ora.reset_envs(dn)
        np.testing.assert_array_equal(obs[t + 1].reshape(E, N, -1), ora.observe())
        np.testing.assert_array_equal(rew[t].reshape(E, N), rw)
        np.testing.assert_array_equal(masks[t + 1].reshape(E, N), np.repeat((~dn)[:, None], N, 1).astype(np.float32))
        if t % 9 == 0 or t == T - 1:
            v, _, lp, ha2, hc2 = om.get_actions(PA, PC, torch.from_numpy(obs[t]), ha[t], hc[t],
                                                torch.from_numpy(masks[t]).view(-1, 1),
                                                actions=torch.from_numpy(acts[t]).view(-1, 1))
            np.testing.assert_allclose(b.action_log_probs[t].cpu().numpy(), lp.numpy()[:, 0], rtol=1e-5, atol=2e-6)
            np.testing.assert_allclose(b.value_preds[t].cpu().numpy(), v.numpy()[:, 0], rtol=1e-5, atol=2e-6)
            keep = torch.from_numpy(masks[t + 1]).view(-1, 1)
            np.testing.assert_allclose(ha[t + 1].numpy(), (ha2 * keep).numpy(), rtol=1e-5, atol=2e-6)
            np.testing.assert_allclose(hc[t + 1].numpy(), (hc2 * keep).numpy(), rtol=1e-5, atol=2e-6)
    assert masks[1:].min() == 0.0          # episodes finished inside the window
    tr = r.trainer
    vn0 = [float(x) for x in tr.vn.cpu().numpy()]
    data = _ref_layout(b, E, N)
    ret_ref, _ = om.compute_returns(data["rewards"], data["value_preds"], data["masks"], data["value_preds"][T],
                                    om.ValueNorm(*vn0), 0.99, 0.95)
    np.testing.assert_allclose(data["returns"][:T], ret_ref[:T], rtol=1e-5, atol=1e-5)
    # ---- PPO epoch 0 gradients through the fused MFMA pass (mm_mappo_grad: 819 tiles of 32 chunks
    # over 1024 waves, per-block partials) -- the trainer bench.py runs
    tr.prepare(b)
    assert tr.fused
    assert lib().mm_mappo_vn_update(tr.vn.data_ptr(), tr.stats.data_ptr(), 0.99999, None) == 0
    tr.gradients(b)
    torch.cuda.synchronize()
    g64, spread = _fp32_spread(lambda dt, pm: _unclipped_grads(_ppo_oracle(PA, PC, data, vn0, 1, L, dt, pm)[0]),
                               T * EN // L)
    for n, net in enumerate((p.actor, p.critic)):
        for k in om.NET_KEYS:
            _assert_within(net.view(k, tr.grad[n]).cpu().numpy(), g64[(n, k)], spread[(n, k)], f"net {n} {k}")


@pytest.mark.parametrize("L", [5, 10, 1])
def test_fused_gradients_match_saves_path_and_are_deterministic(L):
    """mm_mappo_grad (forward recomputed in the backward, MFMA weight gradients) vs the saves + BPTT +
    wgrad kernels on the same rollout, several chunk lengths (ragged last tile: 330 chunks at L = 10),
    |g_fused - g_saves| <= 1e-4 max|g| + 1e-4 |g|; two fused runs are bit-identical."""
    from minimarl._lib import lib
    from minimarl.env import VecEnv
    from minimarl.mappo import MappoPolicy, MappoRunner, MappoTrainer
    E, N, T = 66, 5, 20
    env = VecEnv(E, N, max_steps=100, device=DEV)
    p = MappoPolicy(env.obs_dim, 5, 32, DEV, seed=5)
    r = MappoRunner(env, p, T=T, L=L, ppo_epoch=1, seed=2)
    r.warmup()
    r.rollout()
    r.compute()
    b = r.buf
    grads = {}
    for fused in (True, False, True):
        tr = MappoTrainer(p, T, E * N, L=L, ppo_epoch=1, fused=fused)
        tr.vn.copy_(r.trainer.vn)
        tr.prepare(b)
        assert lib().mm_mappo_vn_update(tr.vn.data_ptr(), tr.stats.data_ptr(), 0.99999, None) == 0
        tr.gradients(b)
        torch.cuda.synchronize()
        g = [x.cpu().numpy().copy() for x in tr.grad]
        if fused and fused in grads:
            for n in (0, 1):
                np.testing.assert_array_equal(g[n], grads[True][n])
        grads.setdefault(fused, g)
    for n in (0, 1):
        a, ref = grads[True][n], grads[False][n]
        assert np.isfinite(a).all()
        np.testing.assert_array_less(np.abs(a - ref), 1e-4 * np.abs(ref).max() + 1e-4 * np.abs(ref) + 1e-9)


def test_data_parallel_hooks_match_single_replica():
    """The data-parallel train() (raw advantage / return sums all-reduced, stats from the global sums,
    per-epoch gradient all-reduce averaged in clip/Adam) with a stand-in all-reduce for TWO identical
    replicas (x2, world 2) equals the single-replica train(): same global statistics and mean gradients.
    Tolerance rtol 1e-4: the replicated path's advantage std is the one-pass form over f64 sums, the
    single-GPU path's the two-pass form."""
    from minimarl.env import VecEnv
    from minimarl.mappo import MappoPolicy, MappoRunner

    def run(allreduce):
        E, N, T = 64, 8, 20
        env = VecEnv(E, N, max_steps=12, device=DEV)
        p = MappoPolicy(env.obs_dim, 5, 32, DEV, seed=0)
        r = MappoRunner(env, p, T=T, L=5, ppo_epoch=3, seed=1, grad_allreduce=allreduce)
        r.warmup()
        r.rollout()
        r.compute()
        info = r.train()
        torch.cuda.synchronize()
        return p, info

    def twice(g):
        g.mul_(2.0)
        return 2

    p1, i1 = run(None)
    p2, i2 = run(twice)
    assert all(np.isfinite(v) for v in i2.values()), i2
    np.testing.assert_allclose(p2.actor.flat.cpu().numpy(), p1.actor.flat.cpu().numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(p2.critic.flat.cpu().numpy(), p1.critic.flat.cpu().numpy(), rtol=1e-4, atol=1e-6)


def test_full_train_15_epochs_vs_oracle_at_scale():
    """R_MAPPO.train as benched (15 PPO epochs, one full-batch minibatch each, ValueNorm updated per epoch,
    advantages normalised once, clip 0.5 + Adam per net; ramppo_network.py:211-287) at 128 envs x 8 agents x
    T = 40 (the golden covers E = 4, N = 2, T = 10 only): post-train parameters and ValueNorm state within K_FP32
    fp32 spreads (module docstring; over 15 epochs the spread carries Adam's sign-flip steps of near-zero
    gradients) of the f64 oracle on the same rollout whose old log-probs / values are its own epoch-0 forward
    (_ppo_oracle_self_old: the device's rollout and training forwards are the same MFMA code, so its epoch-0 ratio
    is exactly 1)."""
    from minimarl.env import VecEnv
    from minimarl.mappo import MappoPolicy, MappoRunner
    E, N, T, L, EP = 128, 8, 40, 5, 15
    env = VecEnv(E, N, max_steps=100, device=DEV)
    p = MappoPolicy(env.obs_dim, 5, 32, DEV, seed=5)
    r = MappoRunner(env, p, T=T, L=L, ppo_epoch=EP, seed=13)
    r.warmup()
    r.rollout()
    r.compute()
    torch.cuda.synchronize()
    PA = {k: p.actor.view(k).detach().cpu().clone() for k in om.NET_KEYS}
    PC = {k: p.critic.view(k).detach().cpu().clone() for k in om.NET_KEYS}
    vn0 = [float(x) for x in r.trainer.vn.cpu().numpy()]
    data = _ref_layout(r.buf, E, N)
    r.train()
    torch.cuda.synchronize()
    _, spread = _fp32_spread(lambda dt, pm: _train_outputs(*_ppo_oracle(PA, PC, data, vn0, EP, L, dt, pm)),
                             T * E * N // L)
    # the reference: the f64 oracle whose old log-probs / values are its own epoch-0 training forward (ratio exactly 1
    # at epoch 0, as on the device, whose rollout and training forwards are one MFMA code path); the spread also
    # covers the fp32 run of that variant
    o64 = _ppo_oracle_self_old(PA, PC, data, vn0, EP, L, torch.float64)
    o_32 = _ppo_oracle_self_old(PA, PC, data, vn0, EP, L, torch.float32)
    for k in o64:
        spread[k] = max(spread[k], float(np.abs(np.asarray(o_32[k], np.float64) - np.asarray(o64[k], np.float64)).max()))
    for net, kind in ((p.actor, "actor"), (p.critic, "critic")):
        for k in om.NET_KEYS:
            _assert_within(net.view(k).detach().cpu().numpy(), o64[(kind, k)], spread[(kind, k)], f"{kind} {k}")
    vn = r.trainer.value_normalizer_state()
    _assert_within(vn["running_mean"], o64["vn_mean"], spread["vn_mean"], "vn mean")
    _assert_within(vn["running_mean_sq"], o64["vn_mean_sq"], spread["vn_mean_sq"], "vn mean_sq")


def test_cfg3_full_size_rollout_returns_and_epoch():
    """cfg3 at its own size (4096 envs x 8 agents x T = 100, the shape bench.py times), checked through properties
    the oracle can afford at that size (magym_runner.py:30-105):
    * the env: obs / rewards / masks bit-exact vs the env oracle for the first 5 steps, driven with the stored actions;
      every later step's masks are exactly 0 / 1 per env and all agents of an env share them;
    * GAE + ValueNorm returns (shared_buffer.py:131-157) vs ``om.compute_returns`` on the device's own rewards,
      values and masks (rtol 1e-5 atol 1e-5);
    * one full PPO epoch (ramppo_network.py:211-287): finite losses and gradient norms, ratio 1 at epoch 0 (the
      policy has not moved: every active row's exp(logp - logp_old) = 1 up to fp32 rounding), parameters changed
      and finite."""
    from minimarl.env import VecEnv
    from minimarl.mappo import MappoPolicy, MappoRunner
    from oracle.env import EnvSpec, VecEnvOracle
    E, N, T, L = 4096, 8, 100, 5
    env = VecEnv(E, N, max_steps=100, device=DEV)
    p = MappoPolicy(env.obs_dim, 5, 32, DEV, seed=3)
    r = MappoRunner(env, p, T=T, L=L, ppo_epoch=1, seed=11)
    r.warmup()
    r.rollout()
    r.compute()
    torch.cuda.synchronize()
    b = r.buf
    obs, acts = b.obs.cpu().numpy(), b.actions.cpu().numpy().astype(np.int64)
    masks, rew = b.masks.cpu().numpy(), b.rewards.cpu().numpy()
    ora = VecEnvOracle(EnvSpec(N, 100), E)
    np.testing.assert_array_equal(obs[0].reshape(E, N, -1), ora.observe())
    for t in range(5):
        _, rw, dn = ora.step(acts[t].reshape(E, N))
        ora.reset_envs(dn)
        np.testing.assert_array_equal(obs[t + 1].reshape(E, N, -1), ora.observe())
        np.testing.assert_array_equal(rew[t].reshape(E, N), rw)
        np.testing.assert_array_equal(masks[t + 1].reshape(E, N), np.repeat((~dn)[:, None], N, 1).astype(np.float32))
    m = masks.reshape(T + 1, E, N)
    assert set(np.unique(m)) <= {0.0, 1.0} and (m == m[:, :, :1]).all()
    assert m[1:].min() == 0.0                       # envs finished inside the episode
    tr = r.trainer
    vn0 = [float(x) for x in tr.vn.cpu().numpy()]
    data = _ref_layout(b, E, N)
    ret_ref, _ = om.compute_returns(data["rewards"], data["value_preds"], data["masks"], data["value_preds"][T],
                                    om.ValueNorm(*vn0), 0.99, 0.95)
    np.testing.assert_allclose(data["returns"][:T], ret_ref[:T], rtol=1e-5, atol=1e-5)
    a0, c0 = p.actor.flat.clone(), p.critic.flat.clone()
    info = r.train()
    torch.cuda.synchronize()
    for k in ("value_loss", "policy_loss", "dist_entropy", "actor_grad_norm", "critic_grad_norm", "ratio"):
        assert np.isfinite(info[k]), k
    assert abs(info["ratio"] - 1.0) < 1e-3          # (an f32 atomic sum over 3.3M rows)
    assert torch.isfinite(p.actor.flat).all() and torch.isfinite(p.critic.flat).all()
    assert not torch.equal(p.actor.flat, a0) and not torch.equal(p.critic.flat, c0)
