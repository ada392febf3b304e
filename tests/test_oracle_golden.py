"""Pin the CPU oracle to the reference's own outputs (golden vectors from tests/golden)."""
import numpy as np
import torch

from oracle import nets
from oracle.sumtree import SumTreeOracle


def _t(x):
    return torch.tensor(x)


def test_qnet_forward_matches_reference(golden):
    for tag, style in [("qmix_n2", "qmix"), ("qmix_n8", "qmix"), ("vdn_n2", "vdn")]:
        fx = golden("qnet_" + tag)
        P = nets.agent_from_state(fx, "p.", style)
        q, h = nets.agent_forward(P, _t(fx["obs"]), _t(fx["hidden"]))
        np.testing.assert_allclose(q.numpy(), fx["q"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(h.numpy(), fx["next_hidden"], rtol=1e-5, atol=1e-6)


def test_sample_action_replay(golden):
    for tag, style in [("qmix", "qmix"), ("vdn", "vdn")]:
        fx = golden("sample_action_" + tag)
        P = nets.agent_from_state(fx, "p.", style)
        q, h = nets.agent_forward(P, _t(fx["obs"]), _t(fx["hidden"]))
        act = nets.epsilon_greedy(q, float(fx["epsilon"]), fx["u"], fx["rand_actions"])
        np.testing.assert_array_equal(act.numpy(), fx["action"])


def test_td_error(golden):
    fx = golden("td_error")
    for i in range(int(fx["n_cases"])):
        td = nets.cal_td_error(_t(fx[f"c{i}.action"]), list(fx[f"c{i}.reward"]), int(fx[f"c{i}.done"]),
                               _t(fx[f"c{i}.behavior_q"]), _t(fx[f"c{i}.target_q"]), float(fx["gamma"]))
        assert abs(td - float(fx[f"c{i}.td"])) <= 1e-5 * max(1.0, abs(float(fx[f"c{i}.td"])))


def test_mixer_forward(golden):
    fx = golden("mixnet")
    M = nets.mixer_from_state(fx, "p.")
    qt, h = nets.mixer_forward(M, _t(fx["q"]), _t(fx["obs"]), _t(fx["hidden"]))
    np.testing.assert_allclose(qt.numpy(), fx["q_tot"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(h.numpy(), fx["next_hidden"], rtol=1e-5, atol=1e-6)


def _replay_per(fx, flavor):
    cap = int(fx["capacity"])
    b = int(fx["batch"])
    if flavor == "vdn":
        st = SumTreeOracle(cap, "vdn", alpha=0.4, beta=0.4, alpha_inc=(1 - 0.4) / (30000 * 10),
                           beta_inc=(1 - 0.4) / (30000 * 10))
    else:
        st = SumTreeOracle(cap, "qmix", alpha=0.8, beta=0.2, alpha_inc=(1 - 0.8) / (100000 * 10),
                           beta_inc=(1 - 0.2) / (100000 * 10))
    slot_chunk = {}
    for k in range(int(fx["n_ops"])):
        kind = int(fx[f"op{k}.kind"])
        if kind == 0:
            slot = st.add(float(fx[f"op{k}.td"]))
            slot_chunk[slot] = int(fx[f"op{k}.chunk_id"])
        elif kind == 1:
            nodes, slots, _, w = st.sample(b, fx[f"op{k}.fracs"])
            np.testing.assert_array_equal(nodes, fx[f"op{k}.idx"])
            np.testing.assert_allclose(w, fx[f"op{k}.is_weight"].ravel(), rtol=1e-6)
            np.testing.assert_array_equal([slot_chunk[s] for s in slots], fx[f"op{k}.chunk_ids"])
            assert abs(st.beta - float(fx[f"op{k}.beta"])) < 1e-15
        else:
            for node, td in zip(fx[f"op{k}.idx"], fx[f"op{k}.td"]):
                # the reference feeds a float32 tensor: priority computed in f32 (App. A 9)
                p32 = (np.float32(td) + np.float32(st.eps)) ** np.float32(st.alpha)
                st.update_leaf(int(node), float(np.float32(p32)))
        np.testing.assert_allclose(st.tree, fx[f"op{k}.tree"], rtol=2e-6, atol=1e-9)


def test_per_vdn_sequence(golden):
    _replay_per(golden("per_vdn"), "vdn")


def test_per_qmix_sequence(golden):
    _replay_per(golden("per_qmix"), "qmix")


def test_vdn_train_step(golden):
    fx = golden("vdn_train")
    P = nets.agent_from_state(fx, "before.", "vdn")
    T = nets.agent_from_state(fx, "target.", "vdn")
    batch = nets.batch_from_fixture(fx)
    newP, g, loss, new_td = nets.vdn_train_step(P, T, batch, float(fx["gamma"]), float(fx["lr"]),
                                                float(fx["grad_clip"]))
    np.testing.assert_allclose(float(loss), float(fx["loss"]), rtol=1e-5)
    after = nets.agent_from_state(fx, "after.", "vdn")
    for k in nets.AGENT_KEYS:
        np.testing.assert_allclose(newP[k].numpy(), after[k].numpy(), rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(new_td.numpy(), fx["new_td"], rtol=1e-4, atol=1e-5)


def test_qmix_train_step(golden):
    fx = golden("qmix_train")
    P = nets.agent_from_state(fx, "before_q.", "qmix")
    M = nets.mixer_from_state(fx, "before_m.")
    T = nets.agent_from_state(fx, "target_q.", "qmix")
    TM = nets.mixer_from_state(fx, "target_m.")
    batch = nets.batch_from_fixture(fx)
    newP, newM, g, loss, new_td = nets.qmix_train_step(P, M, T, TM, batch, float(fx["gamma"]),
                                                       float(fx["lr"]), float(fx["grad_clip"]))
    np.testing.assert_allclose(float(loss), float(fx["loss"]), rtol=1e-5)
    after = nets.agent_from_state(fx, "after_q.", "qmix")
    for k in nets.AGENT_KEYS:
        np.testing.assert_allclose(newP[k].numpy(), after[k].numpy(), rtol=1e-5, atol=2e-6)
    afterM = nets.mixer_from_state(fx, "after_m.")
    for k in nets.MIXER_KEYS:
        np.testing.assert_allclose(newM[k].numpy(), afterM[k].numpy(), rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(new_td.numpy(), fx["new_td"], rtol=1e-4, atol=1e-4)


def test_vdn_double_train_step(golden):
    """Oracle of Target_Double_Dqn (vdn/_train.py:104-158) vs the reference's update."""
    fx = golden("vdn_double_train")
    P = nets.agent_from_state(fx, "before.", "vdn")
    T = nets.agent_from_state(fx, "target.", "vdn")
    batch = nets.batch_from_fixture(fx)
    newP, g, loss, new_td = nets.vdn_double_train_step(P, T, batch, float(fx["gamma"]), float(fx["lr"]),
                                                       float(fx["grad_clip"]), float(fx["epsilon"]),
                                                       fx["double_u"], fx["double_rand_act"])
    np.testing.assert_allclose(float(loss), float(fx["loss"]), rtol=1e-5)
    np.testing.assert_allclose(new_td.numpy(), fx["new_td"], rtol=1e-4, atol=1e-5)
    after = nets.agent_from_state(fx, "after.", "vdn")
    for k in nets.AGENT_KEYS:
        np.testing.assert_allclose(newP[k].numpy(), after[k].numpy(), rtol=1e-5, atol=2e-6)


def _qmix_min_fixture(golden):
    fx = golden("qmix_min_train")
    P = nets.agent_from_state(fx, "q.", "min")
    T = nets.agent_from_state(fx, "qt.", "min")
    M = nets.mixer_from_state(fx, "m.")
    TM = nets.mixer_from_state(fx, "mt.")
    batch = tuple(torch.tensor(fx[k]) for k in ("s", "a", "r", "s2", "done"))
    gamma, lr = (float(x) for x in fx["gamma_lr"])
    return fx, P, T, M, TM, batch, gamma, lr


def test_qmix_min_train_step(golden):
    """Oracle of the minimal QMIX (qmix/qmix.py train, row a15) vs the reference's own update."""
    fx, P, T, M, TM, batch, gamma, lr = _qmix_min_fixture(golden)
    newP, newM, g, loss = nets.qmix_min_train_step(P, M, T, TM, batch, gamma, lr, 5.0)
    gref = nets.agent_from_state(fx, "grad.q.", "min")
    post = nets.agent_from_state(fx, "post.q.", "min")
    for k in nets.AGENT_KEYS:
        np.testing.assert_allclose(g[k].numpy(), gref[k].numpy(), rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(newP[k].numpy(), post[k].numpy(), rtol=1e-5, atol=2e-6)
    gmref = nets.mixer_from_state(fx, "grad.m.")
    postM = nets.mixer_from_state(fx, "post.m.")
    for k in nets.MIXER_KEYS:
        np.testing.assert_allclose(g["m." + k].numpy(), gmref[k].numpy(), rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(newM[k].numpy(), postM[k].numpy(), rtol=1e-5, atol=2e-6)


def test_per_batched_insert_equals_sequential_when_no_self_eviction():
    rng = np.random.default_rng(0)
    a = SumTreeOracle(13, "vdn")
    b = SumTreeOracle(13, "vdn")
    init = rng.random(9) * 0.1
    for td in init:
        a.add(td)
        b.add(td)
    new = 1.0 + rng.random(8)           # all larger than any existing priority
    for td in new:
        a.add(td)
    b.add_batch(new)
    np.testing.assert_allclose(np.sort(a.tree[12:]), np.sort(b.tree[12:]))
    np.testing.assert_allclose(a.tree[0], b.tree[0], rtol=1e-12)
