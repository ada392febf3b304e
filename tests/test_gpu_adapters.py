"""GPU: the reference-signature adapters (minimarl/adapters.py) driven exactly as the
reference calls its own classes, against the reference's golden vectors."""
import random
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import mappo as om
from oracle import nets

pytestmark = pytest.mark.gpu
DEV = "cuda"


class _Space:
    def __init__(self, shape=None, n=None):
        self.shape, self.n = shape, n


class FixtureReplay:
    """A duck-typed Replay_buffer (the interface Train_dqn / Target_Dqn use: sample + update) that
    hands out the golden update's sampled batch and records the priority updates."""

    def __init__(self, fx):
        self.fx, self.updates = fx, []

    def sample(self, batch_size, chunk_size):
        f = self.fx
        t = lambda k: torch.tensor(f[k])  # noqa: E731
        return (t("states"), t("actions"), t("rewards"), t("next_states"), t("dones"), list(f["idx"]),
                t("is_weight"))

    def update(self, idx, td):
        self.updates.append((int(idx), float(td.reshape(-1)[0])))


def _args(fx, **kw):
    a = SimpleNamespace(batch_size=32, update_iter=1, chunk_size=10, use_recurrent=True, gamma=float(fx["gamma"]),
                        grad_clip_norm=float(fx["grad_clip"]))
    a.__dict__.update(kw)
    return a


def _check_updates(rep, fx):
    idx = [u[0] for u in rep.updates]
    td = np.array([u[1] for u in rep.updates])
    np.testing.assert_array_equal(idx, fx["upd_idx"])
    np.testing.assert_allclose(td, fx["new_td"], rtol=1e-4, atol=1e-4)


def test_train_dqn_adapter_matches_reference(golden):
    """Train_dqn(args, device).train(Replay_buffer, bq, bm, tq, tm, optimizer, epsilon), qmix/_train.py:19-121."""
    from minimarl.adapters import Mix_Net, Q_Net, Train_dqn
    fx = golden("qmix_train")
    N, D = fx["states"].shape[2:]
    obs_sp, act_sp = [_Space((D,))] * N, [_Space(n=5)] * N
    args = _args(fx)
    bq, tq = Q_Net(obs_sp, act_sp, args), Q_Net(obs_sp, act_sp, args)
    bm, tm = Mix_Net(obs_sp, args), Mix_Net(obs_sp, args)
    sd = lambda p: {k[len(p):]: fx[k] for k in fx if k.startswith(p)}  # noqa: E731
    bq.load_state_dict(sd("before_q."))
    tq.load_state_dict(sd("target_q."))
    bm.load_state_dict(sd("before_m."))
    tm.load_state_dict(sd("target_m."))
    optimizer = torch.optim.Adam(params=[torch.zeros(1)], lr=float(fx["lr"]))
    rep = FixtureReplay(fx)
    out = Train_dqn(args, DEV).train(rep, bq, bm, tq, tm, optimizer, 0.1)
    torch.cuda.synchronize()
    assert out is None
    _check_updates(rep, fx)
    after = nets.agent_from_state(fx, "after_q.", "qmix")
    got = nets.agent_from_state(bq.state_dict(), "", "qmix")
    for i, key in enumerate(nets.AGENT_KEYS):
        g_all = np.stack([fx[f"g0.{10 * a + i}"] for a in range(N)])
        sel = np.abs(g_all) > 1e-4 * np.abs(g_all).max()
        np.testing.assert_allclose(got[key].numpy()[sel], after[key].numpy()[sel], atol=2e-6)
    afterM = nets.mixer_from_state(fx, "after_m.")
    gotM = nets.mixer_from_state({"m." + k: v for k, v in bm.state_dict().items()}, "m.")
    for j, key in enumerate(nets.MIXER_KEYS):
        g_ref = fx[f"g1.{j}"]
        sel = np.abs(g_ref) > 1e-4 * np.abs(g_ref).max()
        np.testing.assert_allclose(gotM[key].numpy()[sel], afterM[key].numpy()[sel], atol=2e-6)
    # the behavior nets keep working as reference-shaped modules after the update
    q, h = bq(torch.tensor(fx["states"][:, 0]), bq.init_hidden(32))
    assert q.shape == (32, N, 5) and torch.isfinite(q).all()


def test_target_dqn_adapter_matches_reference(golden):
    """Target_Dqn(buffer, behavior, target, args, device).train(target_network, optimizer, epsilon) -> loss."""
    from minimarl.adapters import Q_Net, Target_Dqn
    fx = golden("vdn_train")
    N, D = fx["states"].shape[2:]
    obs_sp, act_sp = [_Space((D,))] * N, [_Space(n=5)] * N
    args = _args(fx)
    beh, tgt = Q_Net(obs_sp, act_sp, args), Q_Net(obs_sp, act_sp, args)
    sd = lambda p: {k[len(p):]: fx[k] for k in fx if k.startswith(p)}  # noqa: E731
    beh.load_state_dict(sd("before."), style="vdn")
    tgt.load_state_dict(sd("target."), style="vdn")
    rep = FixtureReplay(fx)
    tm = Target_Dqn(rep, beh, tgt, args, DEV)
    loss = tm.train(tgt, torch.optim.Adam(params=[torch.zeros(1)], lr=float(fx["lr"])), 0.1)
    torch.cuda.synchronize()
    assert loss.shape == ()
    np.testing.assert_allclose(float(loss), float(fx["loss"]), rtol=1e-4)
    _check_updates(rep, fx)


def test_learner_adapter_rebinds(golden):
    """A new target object or a changed optimizer lr rebuilds the adapter's learner over the same nets
    (the old one releases them first; the Adam moments carry over); a second adapter over the same
    behavior nets also binds."""
    from minimarl.adapters import Mix_Net, Q_Net, Train_dqn
    fx = golden("qmix_train")
    N, D = fx["states"].shape[2:]
    obs_sp, act_sp = [_Space((D,))] * N, [_Space(n=5)] * N
    args = _args(fx)
    bq, tq, tq2 = (Q_Net(obs_sp, act_sp, args) for _ in range(3))
    bm, tm = Mix_Net(obs_sp, args), Mix_Net(obs_sp, args)
    opt = torch.optim.Adam(params=[torch.zeros(1)], lr=1e-3)
    tr = Train_dqn(args, DEV)
    tr.train(FixtureReplay(fx), bq, bm, tq, tm, opt, 0.1)
    L1 = tr._learner
    m1 = L1.m.clone()
    tr.train(FixtureReplay(fx), bq, bm, tq2, tm, opt, 0.1)          # new target net
    assert tr._learner is not L1 and tr._learner.updates == 2
    assert not torch.equal(tr._learner.m, m1)                       # moments continued, then stepped
    opt.param_groups[0]["lr"] = 5e-4
    tr.train(FixtureReplay(fx), bq, bm, tq2, tm, opt, 0.1)          # lr change
    assert tr._learner.lr == 5e-4 and tr._learner.updates == 3
    tr._learner.release()
    Train_dqn(args, DEV).train(FixtureReplay(fx), bq, bm, tq2, tm, opt, 0.1)   # second adapter, same nets
    q, _ = bq(torch.tensor(fx["states"][:, 0]), bq.init_hidden(32))
    assert torch.isfinite(q).all()


def test_adapter_large_batch_forward_after_update_uses_new_weights(golden):
    """After an adapter train step (the learner repacks only the exact-f32 image, pack_f32), a large-batch
    forward (B >= 2048: the fp16x3 LDS kernel and its range flags) must see the updated weights: equal to a
    fresh Q_Net loaded with the same state_dict (full pack). ADVICE r4: _packed() ignored _h3_stale."""
    from minimarl.adapters import Mix_Net, Q_Net, Train_dqn
    fx = golden("qmix_train")
    N, D = fx["states"].shape[2:]
    obs_sp, act_sp = [_Space((D,))] * N, [_Space(n=5)] * N
    args = _args(fx)
    bq, tq = Q_Net(obs_sp, act_sp, args), Q_Net(obs_sp, act_sp, args)
    bm, tm = Mix_Net(obs_sp, args), Mix_Net(obs_sp, args)
    sd = lambda p: {k[len(p):]: fx[k] for k in fx if k.startswith(p)}  # noqa: E731
    bq.load_state_dict(sd("before_q."))
    tq.load_state_dict(sd("target_q."))
    bm.load_state_dict(sd("before_m."))
    tm.load_state_dict(sd("target_m."))
    B = 4096
    g = torch.Generator().manual_seed(5)
    obs = (torch.rand(B, N, D, generator=g) < 0.2).float()
    obs[..., :2] = torch.rand(B, N, 2, generator=g)
    h = torch.randn(B, N, bq.net.H, generator=g) * 0.3
    q_before, _ = bq(obs, h)                      # packs both images at the initial weights
    Train_dqn(args, DEV).train(FixtureReplay(fx), bq, bm, tq, tm,
                               torch.optim.Adam(params=[torch.zeros(1)], lr=float(fx["lr"])), 0.1)
    q_after, h_after = bq(obs, h)
    fresh = Q_Net(obs_sp, act_sp, args)
    fresh.load_state_dict(bq.state_dict())
    q_ref, h_ref = fresh(obs, h)
    torch.cuda.synchronize()
    assert not torch.equal(q_after, q_before)
    assert torch.equal(q_after, q_ref) and torch.equal(h_after, h_ref)


def test_mix_net_adapter_golden(golden):
    from minimarl.adapters import Mix_Net
    fx = golden("mixnet")
    B, N, D = fx["obs"].shape
    m = Mix_Net([_Space((D,))] * N, SimpleNamespace(use_recurrent=True))
    m.load_state_dict({k[2:]: fx[k] for k in fx if k.startswith("p.")})
    qt, h = m(torch.tensor(fx["q"]), torch.tensor(fx["obs"]), torch.tensor(fx["hidden"]))
    np.testing.assert_allclose(qt.cpu().numpy(), fx["q_tot"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(h.cpu().numpy(), fx["next_hidden"], rtol=1e-5, atol=1e-5)
    assert m.init_hidden(7).shape == (7, 32)


@pytest.mark.parametrize("flavor", ["vdn", "qmix"])
def test_per_adapter_golden_sequence(golden, flavor, monkeypatch):
    """Prioritized_Experience_Replay(args).collect_sample / sample / update replaying the reference's own
    op sequence; sample() consumes random.random() per stratum like the reference (fractions fed from
    the fixture)."""
    from minimarl.adapters import Prioritized_Experience_Replay
    fx = golden("per_" + flavor)
    cap, b, C = int(fx["capacity"]), int(fx["batch"]), int(fx["chunk"])
    if flavor == "vdn":
        args = SimpleNamespace(buffer_limit=cap, alpha=0.4, beta=0.4, eps=1e-6, step_weight=0.99,
                               use_step_weight=True, update_alpha_beta=True, max_episodes=30000, update_iter=10)
    else:
        args = SimpleNamespace(buffer_limit=cap, alpha=0.8, beta=0.2, eps=1e-6, update_alpha_beta=True,
                               max_episodes=100000, update_iter=10)
    per = Prioritized_Experience_Replay(args, flavor=flavor, device=DEV)
    payload = [np.zeros((C, 2, 3), np.float32), np.zeros((C, 1, 2), np.float32), np.zeros((C, 2), np.float32),
               np.zeros((C, 2, 3), np.float32), np.zeros(C, np.int64)]
    for k in range(int(fx["n_ops"])):
        kind = int(fx[f"op{k}.kind"])
        if kind == 0:
            n = per.collect_sample(payload, float(fx[f"op{k}.td"]), warm_up=True)
            assert n == len(per)
        elif kind == 1:
            it = iter(fx[f"op{k}.fracs"].tolist())
            monkeypatch.setattr(random, "random", lambda: next(it))
            s, a, r, s2, d, idx, w = per.sample(b, C)
            monkeypatch.undo()
            assert s.shape == (b, C, 2, 3) and d.shape == (b, C, 1) and w.shape == (b, 1)
            np.testing.assert_array_equal(idx.cpu().numpy(), fx[f"op{k}.idx"])
            np.testing.assert_allclose(w.cpu().numpy().ravel(), fx[f"op{k}.is_weight"].ravel(), rtol=1e-5)
            last = idx
        else:
            per.update(last, torch.tensor(fx[f"op{k}.td"]))
        np.testing.assert_allclose(per.per.tree().cpu().numpy(), fx[f"op{k}.tree"], rtol=2e-6, atol=1e-9)


def _mappo_args():
    return SimpleNamespace(hidden_size=32, actor_lr=1e-4, critic_lr=1e-4, opti_eps=1e-5, weight_decay=0, seed=1)


def test_r_mappo_policy_adapter_golden(golden):
    """R_MAPPOPolicy(args, obs_space, cent_obs_space, act_space, device): get_values / evaluate_actions vs
    the reference's outputs; get_actions' values and hiddens vs the reference, its log-probs those of the
    actions it sampled (device RNG)."""
    from minimarl.adapters import R_MAPPOPolicy
    fx = golden("mappo_fwd")
    D = fx["obs"].shape[1]
    pol = R_MAPPOPolicy(_mappo_args(), _Space((D,)), _Space((D,)), _Space(n=5), DEV)
    pol.actor.load_reference_state(fx, "actor.")
    pol.critic.load_reference_state(fx, "critic.")
    t = lambda k: torch.from_numpy(fx[k])  # noqa: E731
    v = pol.get_values(t("obs"), t("hc"), t("masks"))
    np.testing.assert_allclose(v.cpu().numpy(), fx["values"], rtol=1e-5, atol=2e-6)
    obs = t("obs").to(DEV)
    v, a, lp, ha, hc = pol.get_actions(obs, obs, t("ha"), t("hc"), t("masks"))
    assert a.shape == (12, 1) and ha.shape == (12, 1, 32)
    np.testing.assert_allclose(v.cpu().numpy(), fx["values"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(ha.cpu().numpy(), fx["ha_out"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(hc.cpu().numpy(), fx["hc_out"], rtol=1e-5, atol=2e-6)
    PA = om.net_from_state(fx, "actor.", "actor")
    logits, _ = om.net_step(PA, t("obs"), t("ha")[:, 0], t("masks"))
    lpo = torch.log_softmax(logits, -1).gather(1, a.cpu())
    np.testing.assert_allclose(lp.cpu().numpy(), lpo.numpy(), rtol=1e-5, atol=2e-6)
    # evaluate_actions on the golden recurrent minibatch (rnn.py:30-77 segments inside each chunk)
    so = t("seq_obs")
    vals, lps, ent = pol.evaluate_actions(so, so, t("seq_ha"), t("seq_hc"), t("seq_actions"), t("seq_masks"),
                                          active_masks=t("seq_active"))
    np.testing.assert_allclose(vals.cpu().numpy(), fx["seq_values"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(lps.cpu().numpy(), fx["seq_logp"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(float(ent), float(fx["seq_entropy"]), rtol=1e-5)
    act, ha2 = pol.act(t("obs"), t("ha"), t("masks"), deterministic=True)
    np.testing.assert_array_equal(act.cpu().numpy()[:, 0], logits.argmax(-1).numpy())
    with pytest.raises(NotImplementedError):
        R_MAPPOPolicy(_mappo_args(), _Space((D,)), _Space((D * 8,)), _Space(n=5), DEV)
