"""Oracle (test infrastructure only): the episode-level recurrent QMix / VDN trainer of the
reference's ``offpolicy/`` fork restated in torch-CPU fp32 (autograd for the gradients only).

Pinned against tests/golden/offq_*.npz (tests/golden/make_golden_offq.py runs the reference).

  agent_q_seq   AgentQFunction over a whole episode (offpolicy/algorithms/qmix/algorithm/
                agent_q_function.py:24-57): LN(D) -> [Linear, ReLU, LN] x 2 (mlp.py:7-29,52-89;
                fc_h is built but unused) -> GRU from h = 0 (rnn.py:4-23, no masks) -> LN ->
                Linear (act.py:21-37). One net shared by all agents, rows stacked agent-major
                (qmix.py:108-124: row = agent * B + b).
  qmixer        QMixer with 2-layer hypernets (q_mixer.py:20-94): w1 = |hyper_w1(s)| viewed
                [N, K] (w1[i][k] = out[i*K + k]), b1 = hyper_b1(s), hidden = elu(q w1 + b1),
                w2 = |hyper_w2(s)|, b2 = hyper_b2(s), Q_tot = hidden . w2 + b2.  VDN: sum_i q_i.
  train_batch   QMix.train_policy_on_batch (qmix.py:80-210): Q(s_t, a_t) for t < T; target
                Q'(s_{t+1}) at the behavior net's greedy actions (double Q) or the max; targets
                r^(agent 0) + (1 - done_env) gamma Q'_tot; error masked by the previous step's
                done_env; loss = sum_b w_b sum_t err^2 / sum(mask) (PER) or sum err^2 / sum(mask);
                new priorities (1 - nu) mean_t |err| + nu max_t |err| + eps; clip_grad_norm_ over
                agent + mixer (max 10); Adam(lr 5e-4, eps 1e-5).
  soft_update   utils/util.py:123-134: target <- target * (1 - tau) + source * tau.
"""
import numpy as np
import torch

from .mappo import LN_EPS, adam, clip_grads, gru_cell, layer_norm

NET_KEYS = ["ln0_w", "ln0_b", "W1", "b1", "ln1_w", "ln1_b", "W2", "b2", "ln2_w", "ln2_b",
            "Wih", "Whh", "bih", "bhh", "lnr_w", "lnr_b", "Wo", "bo"]
# AgentQFunction state_dict names (rnn = RNNBase: feature_norm, mlp, rnn (RNNLayer: rnn, norm); q)
AGENT_REF = {
    "ln0_w": "rnn.feature_norm.weight", "ln0_b": "rnn.feature_norm.bias",
    "W1": "rnn.mlp.fc1.0.weight", "b1": "rnn.mlp.fc1.0.bias",
    "ln1_w": "rnn.mlp.fc1.2.weight", "ln1_b": "rnn.mlp.fc1.2.bias",
    "W2": "rnn.mlp.fc2.0.0.weight", "b2": "rnn.mlp.fc2.0.0.bias",
    "ln2_w": "rnn.mlp.fc2.0.2.weight", "ln2_b": "rnn.mlp.fc2.0.2.bias",
    "Wih": "rnn.rnn.rnn.weight_ih_l0", "Whh": "rnn.rnn.rnn.weight_hh_l0",
    "bih": "rnn.rnn.rnn.bias_ih_l0", "bhh": "rnn.rnn.rnn.bias_hh_l0",
    "lnr_w": "rnn.rnn.norm.weight", "lnr_b": "rnn.rnn.norm.bias",
    "Wo": "q.action_out.weight", "bo": "q.action_out.bias",
}
# QMixer parameters in named_parameters() order (q_mixer.py:39-67, hypernet_layers = 2)
MIXER_KEYS = ["hyper_w1.0.weight", "hyper_w1.0.bias", "hyper_w1.2.weight", "hyper_w1.2.bias",
              "hyper_w2.0.weight", "hyper_w2.0.bias", "hyper_w2.2.weight", "hyper_w2.2.bias",
              "hyper_b1.weight", "hyper_b1.bias",
              "hyper_b2.0.weight", "hyper_b2.0.bias", "hyper_b2.2.weight", "hyper_b2.2.bias"]


def agent_from_state(sd, prefix="q."):
    return {k: torch.tensor(np.asarray(sd[prefix + AGENT_REF[k]]), dtype=torch.float32) for k in NET_KEYS}


def mixer_from_state(sd, prefix="m."):
    return {k: torch.tensor(np.asarray(sd[prefix + k]), dtype=torch.float32) for k in MIXER_KEYS}


def agent_q_seq(P, x, h0=None):
    """x [L, R, D] -> q [L, R, A], final hidden [R, H]."""
    L, R, _ = x.shape
    H = P["Whh"].shape[1]
    h = torch.zeros(R, H) if h0 is None else h0
    f = layer_norm(x, P["ln0_w"], P["ln0_b"])
    f = layer_norm(torch.relu(f @ P["W1"].t() + P["b1"]), P["ln1_w"], P["ln1_b"])
    f = layer_norm(torch.relu(f @ P["W2"].t() + P["b2"]), P["ln2_w"], P["ln2_b"])
    hs = []
    for t in range(L):
        h = gru_cell(f[t], h, P["Wih"], P["Whh"], P["bih"], P["bhh"])
        hs.append(h)
    y = layer_norm(torch.stack(hs), P["lnr_w"], P["lnr_b"])
    return y @ P["Wo"].t() + P["bo"], h


def qmixer(M, q, s, K):
    """q [T, B, N], s [T, B, S] -> Q_tot [T, B]."""
    T, B, N = q.shape
    relu = torch.relu

    def two(k, x):
        return relu(x @ M[k + ".0.weight"].t() + M[k + ".0.bias"]) @ M[k + ".2.weight"].t() + M[k + ".2.bias"]

    w1 = two("hyper_w1", s).abs().view(T, B, N, K)
    b1 = (s @ M["hyper_b1.weight"].t() + M["hyper_b1.bias"]).view(T, B, 1, K)
    hid = torch.nn.functional.elu(q.view(T, B, 1, N) @ w1 + b1)
    w2 = two("hyper_w2", s).abs().view(T, B, K, 1)
    b2 = two("hyper_b2", s).view(T, B, 1, 1)
    return (hid @ w2 + b2).view(T, B)


def stack_agents(x):
    """[N, L, B, ...] -> [L, N*B, ...] (torch.cat(list(x), dim=-2), qmix.py:112-113)."""
    return torch.cat(list(x), dim=-2) if x.dim() == 4 else torch.cat(list(x), dim=1)


def train_batch(P, M, PT, MT, batch, mixer="qmix", double_q=True, use_per=True, huber=False, gamma=0.99,
                huber_delta=10.0, per_nu=0.9, per_eps=1e-6, K=32, max_norm=10.0, lr=5e-4, eps=1e-5, adam_state=None):
    """One QMix.train_policy_on_batch. batch: dict of arrays (reference sample layout).
    Returns (new P, new M, info dict with grads / loss / priorities)."""
    obs = torch.tensor(batch["obs"])                   # [N, T+1, B, D]
    N, T1, B, _ = obs.shape
    T = T1 - 1
    xs = stack_agents(obs)                             # [T+1, N*B, D]
    acts = stack_agents(torch.tensor(batch["acts"]))   # [T, N*B, A]
    share = torch.tensor(batch["share_obs"])           # [T+1, B, S]
    rew = torch.tensor(batch["rewards"])[0, :, :, 0]   # [T, B] (agent 0's reward)
    dn = torch.tensor(batch["dones_env"])[:, :, 0]     # [T, B]
    p = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    m = {k: v.detach().clone().requires_grad_(True) for k, v in M.items()} if mixer == "qmix" else {}
    q_all, _ = agent_q_seq(p, xs)                      # [T+1, NB, A]
    a_idx = acts.max(-1)[1]
    q_taken = q_all[:-1].gather(2, a_idx.unsqueeze(-1))[..., 0]   # [T, NB]
    with torch.no_grad():
        qt_all, _ = agent_q_seq(PT, xs)
        if double_q:
            g = q_all.max(-1)[1]
            nq = qt_all.gather(2, g.unsqueeze(-1))[..., 0]
        else:
            nq = qt_all.max(-1)[0]
        nq = nq[1:]                                      # [T, NB]
    qa = q_taken.view(T, N, B).permute(0, 2, 1)        # [T, B, N]
    nqa = nq.view(T, N, B).permute(0, 2, 1)
    if mixer == "qmix":
        qtot = qmixer(m, qa, share[:-1], K)
        with torch.no_grad():
            nqtot = qmixer(MT, nqa, share[1:], K)
    else:
        qtot, nqtot = qa.sum(-1), nqa.sum(-1)
    bad = torch.cat([torch.zeros(1, B), dn[:T - 1]], 0)
    y = rew + (1 - dn) * gamma * nqtot
    err = (qtot - y.detach()) * (1 - bad)
    if huber:
        ae = err.abs()
        le = torch.where(ae <= huber_delta, err ** 2 / 2, huber_delta * (ae - huber_delta / 2))
    else:
        le = err ** 2
    if use_per:
        w = torch.tensor(batch["is_weight"])
        loss = (le.sum(0) * w).sum() / (1 - bad).sum()
        td = err.abs().detach().numpy().astype(np.float32)
        prio = ((1 - per_nu) * td.mean(0) + per_nu * td.max(0)) + per_eps
    else:
        loss = le.sum() / (1 - bad).sum()
        prio = None
    keys = list(p) + list(m)
    tens = [p[k] for k in p] + [m[k] for k in m]
    grads = torch.autograd.grad(loss, tens)
    gc, total = clip_grads(list(grads), max_norm)
    G = dict(zip(keys, gc))
    state = {} if adam_state is None else adam_state
    new = adam({**P, **{("m:" + k): v for k, v in M.items()}} if mixer == "qmix" else dict(P),
               {**{k: G[k] for k in p}, **{("m:" + k): G[k] for k in m}}, state, lr, eps)
    P2 = {k: new[k] for k in P}
    M2 = {k: new["m:" + k] for k in M} if mixer == "qmix" else M
    info = {"loss": float(loss.detach()), "grad_norm": float(total), "q_tot": float((qtot.detach() * (1 - bad)).mean()),
            "grads": G, "priorities": prio, "err": err.detach()}
    return P2, M2, info


def soft_update(target, source, tau):
    c1, c2 = np.float32(1.0 - tau), np.float32(tau)
    return {k: target[k] * float(c1) + source[k] * float(c2) for k in target}


__all__ = ["NET_KEYS", "AGENT_REF", "MIXER_KEYS", "agent_from_state", "mixer_from_state", "agent_q_seq", "qmixer",
           "train_batch", "soft_update", "LN_EPS"]
