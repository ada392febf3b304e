"""GPU: the offpolicy episode QMix / VDN trainer (csrc/offq.hip via minimarl.offq.OffQMix) against
the reference's own train_policy_on_batch (tests/golden/offq_*.npz) and the CPU oracle."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
from make_golden_offq import target_perturbation  # noqa: E402

from oracle import offq as ref  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load_case(name):
    f = np.load(os.path.join(GOLD, f"offq_{name}.npz"))
    d = {k: f[k] for k in f.files}
    N, T, B, D, A, dq, per, hub, tseed = [int(x) for x in d["meta"]]
    base = [k for k in f.files if k.startswith("q.") or k.startswith("m.")]
    pert = target_perturbation([(k, d[k].shape) for k in base], tseed)
    tgt = {k: d[k] + pert[k] for k in base}
    return d, tgt, dict(N=N, T=T, B=B, D=D, A=A, double_q=bool(dq), use_per=bool(per), huber=bool(hub))


def sub(sd, prefix):
    return {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}


def make_trainer(name, d, tgt, meta):
    from minimarl.offq import OffQMix
    g, lr, eps, mx, hd, nu, pe = [float(x) for x in d["hyper"]]
    K, Hh = [int(x) for x in d["mixer_dims"]]
    tr = OffQMix(meta["N"], meta["D"], meta["A"], meta["T"], meta["B"], mixer=name, mixer_hidden=K, hyper_hidden=Hh,
                 gamma=g, lr=lr, opti_eps=eps, max_grad_norm=mx, use_double_q=meta["double_q"],
                 use_per=meta["use_per"], use_huber_loss=meta["huber"], huber_delta=hd, per_nu=nu, per_eps=pe)
    tr.load_reference_state(sub(d, "q."), sub(d, "m."), sub(tgt, "q."), sub(tgt, "m."))
    return tr


def ref_batch(d):
    pid = "policy_0"
    isw = d.get("is_weight")
    return ({pid: d["obs"]}, {pid: d["share_obs"]}, {pid: d["acts"]}, {pid: d["rewards"]}, {pid: d["dones"]},
            {pid: d["dones_env"]}, {pid: None}, isw, np.arange(d["obs"].shape[2]))


@pytest.mark.parametrize("name", ["qmix", "vdn"])
def test_offq_train_matches_reference(name):
    d, tgt, meta = load_case(name)
    tr = make_trainer(name, d, tgt, meta)
    info, prio, _ = tr.train_policy_on_batch(ref_batch(d))
    torch.cuda.synchronize()
    np.testing.assert_allclose(float(info["loss"]), d["loss"], rtol=2e-5)
    np.testing.assert_allclose(float(info["Q_tot"]), d["q_tot"], rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(float(info["grad_norm"]), d["grad_norm"], rtol=2e-5)
    coef = min(1.0, float(d["hyper"][3]) / (float(info["grad_norm"]) + 1e-6))
    for k in ref.NET_KEYS:
        rn = "q." + ref.AGENT_REF[k]
        g = tr.agent_view(k, tr.grad).cpu().numpy() * coef
        np.testing.assert_allclose(g, d["grad." + rn], rtol=1e-4, atol=2e-6, err_msg=k)
        np.testing.assert_allclose(tr.agent_view(k).cpu().numpy(), d["post." + rn], rtol=1e-5, atol=2e-6, err_msg=k)
    if name == "qmix":
        for k in ref.MIXER_KEYS:
            g = tr.mixer_view(k, tr.grad).cpu().numpy() * coef
            np.testing.assert_allclose(g, d["grad.m." + k], rtol=1e-4, atol=2e-6, err_msg=k)
            np.testing.assert_allclose(tr.mixer_view(k).cpu().numpy(), d["post.m." + k], rtol=1e-5, atol=2e-6,
                                       err_msg=k)
    if meta["use_per"]:
        np.testing.assert_allclose(prio.cpu().numpy(), d["new_priorities"], rtol=2e-5)
    else:
        assert prio is None


def test_offq_q_values_vs_oracle():
    d, tgt, meta = load_case("qmix")
    tr = make_trainer("qmix", d, tgt, meta)
    P = ref.agent_from_state(d)
    g = torch.Generator().manual_seed(3)
    L, R, D = 7, 300, meta["D"]
    x = (torch.rand(L, R, D, generator=g) < 0.2).float()
    x[..., :2] = torch.rand(L, R, 2, generator=g)
    h0 = torch.randn(R, 64, generator=g) * 0.3
    q_ref, h_ref = ref.agent_q_seq(P, x, h0)
    q, h = tr.get_q_values(x.cuda(), h0.cuda())
    np.testing.assert_allclose(q.cpu().numpy(), q_ref.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(h.cpu().numpy(), h_ref.numpy(), rtol=1e-4, atol=1e-5)
    # single step, zero hidden (rollout shape) and greedy actions
    q1, _ = tr.get_q_values(x[0].cuda())
    q1_ref, _ = ref.agent_q_seq(P, x[:1])
    np.testing.assert_allclose(q1.cpu().numpy(), q1_ref[0].numpy(), rtol=1e-4, atol=1e-5)
    oh, _, gq = tr.get_actions(x[0].cuda())
    assert torch.equal(oh.argmax(-1).cpu(), q1.argmax(-1).cpu())


@pytest.mark.parametrize("name", ["qmix", "vdn"])
def test_offq_multi_update_with_soft_target(name):
    """Three updates with a soft target update after each (runner batch_train_q, base_runner.py:
    273-298) against the oracle's chain; fresh synthetic batches, B = 6, T = 9."""
    d, tgt, meta = load_case(name)
    meta = dict(meta, T=9, B=6)
    from minimarl.offq import OffQMix
    tr = OffQMix(meta["N"], meta["D"], meta["A"], meta["T"], meta["B"], mixer=name, use_double_q=meta["double_q"],
                 use_per=meta["use_per"], use_huber_loss=meta["huber"])
    tr.load_reference_state(sub(d, "q."), sub(d, "m."), sub(tgt, "q."), sub(tgt, "m."))
    P, PT = ref.agent_from_state(d), ref.agent_from_state(tgt)
    M = ref.mixer_from_state(d) if name == "qmix" else {}
    MT = ref.mixer_from_state(tgt) if name == "qmix" else {}
    rng = np.random.default_rng(11)
    st = {}
    from minimarl.synth import offq_episode_batch as make_batch
    for it in range(3):
        obs, share, acts, rew, dones, dones_env = make_batch(rng, meta["N"], meta["T"], meta["B"], meta["D"],
                                                             meta["A"])
        isw = (0.5 + rng.random(meta["B"])).astype(np.float32) if meta["use_per"] else None
        b = {"obs": obs, "share_obs": share, "acts": acts, "rewards": rew, "dones_env": dones_env, "is_weight": isw}
        P, M, info = ref.train_batch(P, M, PT, MT, b, mixer=name, double_q=meta["double_q"],
                                     use_per=meta["use_per"], huber=meta["huber"], adam_state=st)
        PT = ref.soft_update(PT, P, 0.005)
        if name == "qmix":
            MT = ref.soft_update(MT, M, 0.005)
        pid = "policy_0"
        out, prio, _ = tr.train_policy_on_batch(({pid: obs}, {pid: share}, {pid: acts}, {pid: rew}, {pid: dones},
                                                 {pid: dones_env}, {pid: None}, isw, None))
        tr.soft_target_updates()
        torch.cuda.synchronize()
        np.testing.assert_allclose(float(out["loss"]), info["loss"], rtol=1e-4, err_msg=f"iter {it}")
    for k in ref.NET_KEYS:
        np.testing.assert_allclose(tr.agent_view(k).cpu().numpy(), P[k].numpy(), rtol=1e-4, atol=2e-6, err_msg=k)
        np.testing.assert_allclose(tr.agent_view(k, tr.PT).cpu().numpy(), PT[k].numpy(), rtol=1e-4, atol=2e-6,
                                   err_msg="target " + k)
    if name == "qmix":
        for k in ref.MIXER_KEYS:
            np.testing.assert_allclose(tr.mixer_view(k).cpu().numpy(), M[k].numpy(), rtol=1e-4, atol=2e-6, err_msg=k)


def test_offq_grad_allreduce_hook():
    """Data-parallel hook: a stand-in all-reduce that sums two identical replicas' gradients (x2,
    returns world = 2) must leave the update bit-identical to the single-replica one."""
    d, tgt, meta = load_case("qmix")
    a = make_trainer("qmix", d, tgt, meta)
    b = make_trainer("qmix", d, tgt, meta)

    def fake_allreduce(g):
        g.mul_(2.0)
        return 2

    b.allreduce = fake_allreduce
    for tr in (a, b):
        tr.train_policy_on_batch(ref_batch(d))
    torch.cuda.synchronize()
    assert torch.equal(a.P, b.P) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v)
