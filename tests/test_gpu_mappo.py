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


@pytest.mark.parametrize("fused", [True, False], ids=["fused_mfma", "saves_wgrad"])
def test_first_epoch_gradients_match_reference(golden, fused):
    """Unclipped gradients of PPO epoch 0 vs the reference's (clipped) ones / its clip coefficient:
    the fused MFMA pass (mm_mappo_grad, a partial tile of chunks) and the saves + wgrad path."""
    from minimarl._lib import lib
    fx = golden("mappo_train")
    p, buf, tr = _trainer_from_fixture(fx, fused)
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
            scale = np.abs(ref).max()
            np.testing.assert_array_less(np.abs(g - ref), 1e-3 * scale + 1e-3 * np.abs(ref) + 1e-9,
                                         err_msg=f"{kind} {k}")
        # pads of the flat layout carry zero gradient
        assert float(tr.grad[n].abs().sum()) == pytest.approx(
            sum(float(net.view(k, tr.grad[n]).abs().sum()) for k in om.NET_KEYS), rel=1e-6)


@pytest.mark.parametrize("fused", [True, False], ids=["fused_mfma", "saves_wgrad"])
def test_ppo_train_matches_reference(golden, fused):
    fx = golden("mappo_train")
    p, buf, tr = _trainer_from_fixture(fx, fused)
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
    * PPO epoch 0 (ramppo_network.py:103-209): every gradient of actor and critic vs the oracle's
      autograd on the full recurrent minibatch, |g - g_ref| <= 2e-3 max|g_ref| + 2e-3 |g_ref|."""
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
    rec = []
    om.ppo_train(PA, PC, data, om.ValueNorm(*vn0), 1, L, record=rec)
    for n, (net, tag) in enumerate(((p.actor, "ga"), (p.critic, "gc"))):
        nrm = rec[0]["na" if n == 0 else "nc"]
        coef = min(1.0, 0.5 / (nrm + 1e-6))
        for k in om.NET_KEYS:
            g = net.view(k, tr.grad[n]).cpu().numpy()
            ref = rec[0][tag][k].numpy() / coef
            np.testing.assert_array_less(np.abs(g - ref), 2e-3 * np.abs(ref).max() + 2e-3 * np.abs(ref) + 1e-9,
                                         err_msg=f"net {n} {k}")


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
    T = 40 (the golden covers E = 4, N = 2, T = 10 only): post-train parameters vs ``om.ppo_train`` on the same
    rollout. Coordinates whose epoch-0 gradient is significant (> 1e-3 of the tensor's max) within 5e-5;
    every coordinate within 15 epochs x 2 lr (Adam steps of near-zero gradients follow rounding noise)."""
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
    rec = []
    PA2, PC2, vn2 = om.ppo_train(PA, PC, data, om.ValueNorm(*vn0), EP, L, record=rec)
    lr = 1e-4
    for n, (net, ref, tag) in enumerate(((p.actor, PA2, "ga"), (p.critic, PC2, "gc"))):
        for k in om.NET_KEYS:
            got = net.view(k).detach().cpu().numpy()
            want = ref[k].detach().numpy()
            g = np.abs(rec[0][tag][k].numpy())
            sel = g > 1e-3 * g.max()
            np.testing.assert_allclose(got[sel], want[sel], atol=5e-5, err_msg=f"net {n} {k}")
            np.testing.assert_allclose(got, want, atol=2 * EP * lr, err_msg=f"net {n} {k} (all)")
    vn = r.trainer.value_normalizer_state()
    np.testing.assert_allclose(vn["running_mean"], vn2.m.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(vn["running_mean_sq"], vn2.msq.numpy(), rtol=1e-5, atol=1e-6)
