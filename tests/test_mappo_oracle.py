"""CPU: the MAPPO oracle (oracle/mappo.py) against the reference's golden vectors."""
import numpy as np
import pytest
import torch

from oracle import mappo as om


def _nets(fx, prefix=""):
    sd = {k[len(prefix):]: fx[k] for k in fx if k.startswith(prefix)}
    return om.net_from_state(sd, "actor.", "actor"), om.net_from_state(sd, "critic.", "critic")


def test_get_actions_golden(golden):
    fx = golden("mappo_fwd")
    PA, PC = _nets(fx)
    t = lambda k: torch.from_numpy(fx[k])
    v, a, lp, ha, hc = om.get_actions(PA, PC, t("obs"), t("ha")[:, 0], t("hc")[:, 0], t("masks"),
                                      actions=t("actions"))
    np.testing.assert_allclose(v.numpy(), fx["values"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(lp.numpy(), fx["logp"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ha.numpy(), fx["ha_out"][:, 0], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(hc.numpy(), fx["hc_out"][:, 0], rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(fx["draws"][0], fx["actions"])   # the recorded sample is the action


def test_evaluate_chunks_golden(golden):
    fx = golden("mappo_fwd")
    PA, PC = _nets(fx)
    t = lambda k: torch.from_numpy(fx[k])
    L = int(fx["seq_L"])
    lp, ent = om.evaluate_chunks(PA, t("seq_obs"), t("seq_ha")[:, 0], t("seq_masks"), L, "actor",
                                 t("seq_actions"), t("seq_active"))
    v = om.evaluate_chunks(PC, t("seq_obs"), t("seq_hc")[:, 0], t("seq_masks"), L, "critic")
    np.testing.assert_allclose(lp.numpy(), fx["seq_logp"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(v.numpy(), fx["seq_values"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(float(ent), float(fx["seq_entropy"]), rtol=1e-6)


def test_sampler_inverse_cdf():
    logits = torch.tensor([[0.0, 1.0, -1.0, 2.0, 0.5]])
    p = torch.softmax(logits, -1)[0]
    c = torch.cumsum(p, 0)
    for a in range(5):
        lo = 0.0 if a == 0 else float(c[a - 1])
        u = torch.tensor([(lo + float(c[a])) / 2])
        assert int(om.sample_actions(logits, u)) == a
    assert int(om.sample_actions(logits, torch.tensor([0.99999994]))) == 4


def test_compute_returns_golden(golden):
    fx = golden("mappo_gae")
    vn = om.ValueNorm(float(fx["vn_mean"][0]), float(fx["vn_mean_sq"][0]), float(fx["vn_debias"]))
    ret, _ = om.compute_returns(fx["rewards"], fx["value_preds"], fx["masks"], fx["next_value"], vn,
                                float(fx["gamma"]), float(fx["gae_lambda"]))
    np.testing.assert_allclose(ret[:-1], fx["returns"][:-1], rtol=1e-6, atol=1e-6)


def _train_data(fx):
    return {k[5:]: fx[k] for k in fx if k.startswith("data.")}


@pytest.mark.parametrize("use_perm", [True, False])
def test_ppo_train_golden(golden, use_perm):
    fx = golden("mappo_train")
    PA, PC = _nets(fx, "before.")
    vn = om.ValueNorm(float(fx["vn0.running_mean"][0]), float(fx["vn0.running_mean_sq"][0]),
                      float(fx["vn0.debiasing_term"]))
    rec = []
    E = int(fx["epochs"])
    PA2, PC2, vn = om.ppo_train(PA, PC, _train_data(fx), vn, E, int(fx["L"]),
                                perms=fx["perms"] if use_perm else None, record=rec)
    # clipped gradients fed to each Adam step (reference names via om.ref_name)
    tol = dict(rtol=2e-4, atol=1e-7) if use_perm else dict(rtol=2e-3, atol=1e-6)
    for ep in range(E):
        for k in om.NET_KEYS:
            np.testing.assert_allclose(rec[ep]["ga"][k].numpy(), fx[f"grada{ep}.{om.ref_name(k, 'actor')}"],
                                       err_msg=f"actor {k} epoch {ep}", **tol)
            np.testing.assert_allclose(rec[ep]["gc"][k].numpy(), fx[f"gradc{ep}.{om.ref_name(k, 'critic')}"],
                                       err_msg=f"critic {k} epoch {ep}", **tol)
        np.testing.assert_allclose(rec[ep]["na"], fx["norms"][2 * ep], rtol=1e-5)
        np.testing.assert_allclose(rec[ep]["nc"], fx["norms"][2 * ep + 1], rtol=1e-5)
    for k in om.NET_KEYS:
        np.testing.assert_allclose(PA2[k].numpy(), fx[f"after.actor.{om.ref_name(k, 'actor')}"], rtol=1e-5,
                                   atol=2e-6)
        np.testing.assert_allclose(PC2[k].numpy(), fx[f"after.critic.{om.ref_name(k, 'critic')}"], rtol=1e-5,
                                   atol=2e-6)
    np.testing.assert_allclose(vn.m.numpy(), fx["vn1.running_mean"], rtol=1e-6)
    np.testing.assert_allclose(vn.msq.numpy(), fx["vn1.running_mean_sq"], rtol=1e-6)
