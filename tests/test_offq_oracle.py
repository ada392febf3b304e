"""CPU: the offpolicy QMix / VDN trainer oracle (oracle/offq.py) against the reference's own
train_policy_on_batch (fixtures tests/golden/offq_*.npz, made by tests/golden/make_golden_offq.py)."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
from make_golden_offq import target_perturbation  # noqa: E402

from oracle import offq  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load_case(name):
    f = np.load(os.path.join(GOLD, f"offq_{name}.npz"))
    d = {k: f[k] for k in f.files}
    N, T, B, D, A, dq, per, hub, tseed = [int(x) for x in d["meta"]]
    base = [k for k in f.files if k.startswith("q.") or k.startswith("m.")]
    pert = target_perturbation([(k, d[k].shape) for k in base], tseed)
    tgt = {k: d[k] + pert[k] for k in base}
    return d, tgt, dict(N=N, T=T, B=B, D=D, A=A, double_q=bool(dq), use_per=bool(per), huber=bool(hub))


def run_oracle(name):
    d, tgt, meta = load_case(name)
    mixer = "qmix" if name == "qmix" else "vdn"
    P = offq.agent_from_state(d)
    PT = offq.agent_from_state(tgt)
    M = offq.mixer_from_state(d) if mixer == "qmix" else {}
    MT = offq.mixer_from_state(tgt) if mixer == "qmix" else {}
    g, lr, eps, mx, hd, nu, pe = [float(x) for x in d["hyper"]]
    K = int(d["mixer_dims"][0])
    P2, M2, info = offq.train_batch(P, M, PT, MT, d, mixer=mixer, double_q=meta["double_q"],
                                    use_per=meta["use_per"], huber=meta["huber"], gamma=g, huber_delta=hd,
                                    per_nu=nu, per_eps=pe, K=K, max_norm=mx, lr=lr, eps=eps)
    return d, P2, M2, info, mixer


@pytest.mark.parametrize("name", ["qmix", "vdn"])
def test_offq_oracle_matches_reference(name):
    d, P2, M2, info, mixer = run_oracle(name)
    np.testing.assert_allclose(info["loss"], d["loss"], rtol=1e-5)
    np.testing.assert_allclose(info["grad_norm"], d["grad_norm"], rtol=1e-5)
    np.testing.assert_allclose(info["q_tot"], d["q_tot"], rtol=1e-5, atol=1e-6)
    for k in offq.NET_KEYS:
        ref = "q." + offq.AGENT_REF[k]
        np.testing.assert_allclose(info["grads"][k].numpy(), d["grad." + ref], rtol=1e-4, atol=1e-6, err_msg=k)
        np.testing.assert_allclose(P2[k].numpy(), d["post." + ref], rtol=1e-5, atol=1e-6, err_msg=k)
    if mixer == "qmix":
        for k in offq.MIXER_KEYS:
            np.testing.assert_allclose(info["grads"][k].numpy(), d["grad.m." + k], rtol=1e-4, atol=1e-6, err_msg=k)
            np.testing.assert_allclose(M2[k].numpy(), d["post.m." + k], rtol=1e-5, atol=1e-6, err_msg=k)
    if "new_priorities" in d:
        np.testing.assert_allclose(info["priorities"], d["new_priorities"], rtol=1e-5)


def test_offq_soft_update():
    a = {"x": torch.randn(100)}
    b = {"x": torch.randn(100)}
    out = offq.soft_update(a, b, 0.005)
    ref = a["x"] * np.float32(0.995) + b["x"] * np.float32(0.005)
    assert torch.equal(out["x"], ref)
