"""GPU parity of the MAPPO HIP path (csrc/mappo.hip via minimarl.mappo) against the reference's
golden vectors (tests/golden/mappo_*.npz) and the oracle (oracle/mappo.py).

Tolerances (fp32; the device uses hardware exp/rcp for the GRU gates, ~1e-6 relative):
values / log-probs / hiddens rtol 1e-5 atol 2e-6; returns rtol 1e-6; gradients
|g - g_ref| <= 1e-3 * max|g_ref| + 1e-3 * |g_ref|; post-Adam params atol 3e-5 (a tenth of the
three Adam steps' ~3e-4 travel) where |g_ref| is not negligible.
"""
import numpy as np
import pytest
import torch

from oracle import mappo as om

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = dict(rtol=1e-5, atol=2e-6)


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
    tr = MappoTrainer(p, L, n, L=L, ppo_epoch=1)
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


def _trainer_from_fixture(fx):
    from minimarl.mappo import MappoBuffer, MappoTrainer
    p = _policy(fx, "before.")
    E, N, T, L = (int(fx[k]) for k in ("E", "N", "T", "L"))
    buf = MappoBuffer(T, E, N, p.D, 32, DEV)
    buf.load_reference({k[5:]: fx[k] for k in fx if k.startswith("data.")})
    tr = MappoTrainer(p, T, E * N, L=L, ppo_epoch=int(fx["epochs"]))
    tr.load_value_normalizer(float(fx["vn0.running_mean"][0]), float(fx["vn0.running_mean_sq"][0]),
                             float(fx["vn0.debiasing_term"]))
    return p, buf, tr


def test_first_epoch_gradients_match_reference(golden):
    """Unclipped gradients of PPO epoch 0 vs the reference's (clipped) ones / its clip coefficient."""
    import ctypes
    from minimarl._lib import lib
    fx = golden("mappo_train")
    p, buf, tr = _trainer_from_fixture(fx)
    tr.prepare(buf)
    L_, d = lib(), ctypes.byref(p.dims)
    assert L_.mm_mappo_vn_update(tr.vn.data_ptr(), tr.stats.data_ptr(), 0.99999, None) == 0
    fa, ba = tr.fwd_args(buf), tr.bwd_args(buf)
    assert L_.mm_mappo_fwd(d, ctypes.byref(fa), None) == 0
    assert L_.mm_mappo_bwd(d, ctypes.byref(ba), None) == 0
    for n in (0, 1):
        assert L_.mm_mappo_wgrad(d, n, tr.gsoa[n].data_ptr(), tr.rs, tr.grad[n].data_ptr(),
                                 tr.partial.data_ptr(), None) == 0
    torch.cuda.synchronize()
    for n, (net, tag) in enumerate(((p.actor, "a"), (p.critic, "c"))):
        coef = min(1.0, 0.5 / (float(fx["norms"][n]) + 1e-6))
        kind = "actor" if n == 0 else "critic"
        for k in om.NET_KEYS:
            g = net.view(k, tr.grad[n]).cpu().numpy()
            ref = fx[f"grad{tag}0.{om.ref_name(k, kind)}"] / coef
            scale = np.abs(ref).max()
            np.testing.assert_array_less(np.abs(g - ref), 1e-3 * scale + 1e-3 * np.abs(ref) + 1e-9,
                                         err_msg=f"{kind} {k}")
        # pads of the flat layout carry zero gradient
        assert float(tr.grad[n].abs().sum()) == pytest.approx(
            sum(float(net.view(k, tr.grad[n]).abs().sum()) for k in om.NET_KEYS), rel=1e-6)


def test_ppo_train_matches_reference(golden):
    fx = golden("mappo_train")
    p, buf, tr = _trainer_from_fixture(fx)
    info = tr.train(buf)
    torch.cuda.synchronize()
    for n, (net, kind) in enumerate(((p.actor, "actor"), (p.critic, "critic"))):
        tag = "a" if n == 0 else "c"
        for k in om.NET_KEYS:
            name = om.ref_name(k, kind)
            after = fx[f"after.{kind}.{name}"]
            g = np.abs(fx[f"grad{tag}0.{name}"])
            sel = g > 1e-3 * g.max()
            got = net.view(k).cpu().numpy()
            np.testing.assert_allclose(got[sel], after[sel], atol=3e-5, err_msg=f"{kind} {k}")
            np.testing.assert_allclose(got, after, atol=4e-4, err_msg=f"{kind} {k} (all)")
    vn = tr.value_normalizer_state()
    np.testing.assert_allclose(vn["running_mean"], fx["vn1.running_mean"], rtol=1e-5)
    np.testing.assert_allclose(vn["running_mean_sq"], fx["vn1.running_mean_sq"], rtol=1e-5)
    np.testing.assert_allclose(info["value_loss"], float(fx["info.value_loss"]), rtol=1e-3)
    np.testing.assert_allclose(info["policy_loss"], float(fx["info.policy_loss"]), rtol=1e-2, atol=1e-5)
    np.testing.assert_allclose(info["dist_entropy"], float(fx["info.dist_entropy"]), rtol=1e-5)
    np.testing.assert_allclose(info["actor_grad_norm"], float(fx["info.actor_grad_norm"]), rtol=1e-3)
    np.testing.assert_allclose(info["critic_grad_norm"], float(fx["info.critic_grad_norm"]), rtol=1e-3)
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
