"""Oracle (test infrastructure only): per-agent Q-networks, QMIX mixer, TD error, learners.

Restated from the reference in functional torch-CPU fp32 (autograd is used only
for the learner gradients). Parameters are plain stacked tensors (see
``AGENT_KEYS`` / ``MIXER_KEYS``); converters from the reference state_dict
naming live in ``from_qmix_state`` / ``from_vdn_state`` / ``mixer_from_state``.
"""
import numpy as np
import torch
import torch.nn.functional as F

# per-agent stacked parameters, leading dim = agent
#   W1 [N,F1,D] b1 [N,F1]   W2 [N,G,F1] b2 [N,G]          qmix/_network.py:20-26
#   Wih [N,3H,G] Whh [N,3H,H] bih [N,3H] bhh [N,3H]       qmix/_network.py:31-33 (GRUCell, gates r,z,n)
#   Wq [N,A,H] bq [N,A]                                   qmix/_network.py:41
AGENT_KEYS = ["W1", "b1", "W2", "b2", "Wih", "Whh", "bih", "bhh", "Wq", "bq"]
# mixer (qmix/_network.py:172-197)
MIXER_KEYS = ["gWih", "gWhh", "gbih", "gbhh", "w1W", "w1b", "w2W", "w2b", "b1W", "b1b",
              "b2aW", "b2ab", "b2bW", "b2bb"]

_QMIX_FMT = {
    "W1": "feature_network_{i}.0.weight", "b1": "feature_network_{i}.0.bias",
    "W2": "feature_network_{i}.2.weight", "b2": "feature_network_{i}.2.bias",
    "Wih": "gru_network_{i}.weight_ih", "Whh": "gru_network_{i}.weight_hh",
    "bih": "gru_network_{i}.bias_ih", "bhh": "gru_network_{i}.bias_hh",
    "Wq": "action_network_{i}.0.weight", "bq": "action_network_{i}.0.bias",
}
_VDN_FMT = {
    "W1": "feature_net.{i}.0.weight", "b1": "feature_net.{i}.0.bias",
    "W2": "feature_net.{i}.2.weight", "b2": "feature_net.{i}.2.bias",
    "Wih": "gru_net.{i}.weight_ih", "Whh": "gru_net.{i}.weight_hh",
    "bih": "gru_net.{i}.bias_ih", "bhh": "gru_net.{i}.bias_hh",
    "Wq": "action_net.{i}.0.weight", "bq": "action_net.{i}.0.bias",
}
# minimal QMIX QNet (qmix/qmix.py:102-131): agent_feature_i = Linear(D,128) ReLU Linear(128,32) ReLU
_MIN_FMT = {
    "W1": "agent_feature_{i}.0.weight", "b1": "agent_feature_{i}.0.bias",
    "W2": "agent_feature_{i}.2.weight", "b2": "agent_feature_{i}.2.bias",
    "Wih": "agent_gru_{i}.weight_ih", "Whh": "agent_gru_{i}.weight_hh",
    "bih": "agent_gru_{i}.bias_ih", "bhh": "agent_gru_{i}.bias_hh",
    "Wq": "agent_q_{i}.weight", "bq": "agent_q_{i}.bias",
}
_FMTS = {"qmix": _QMIX_FMT, "vdn": _VDN_FMT, "min": _MIN_FMT}
_MIX_FMT = {
    "gWih": "gru.weight_ih", "gWhh": "gru.weight_hh", "gbih": "gru.bias_ih", "gbhh": "gru.bias_hh",
    "w1W": "hyper_net_weight_1.weight", "w1b": "hyper_net_weight_1.bias",
    "w2W": "hyper_net_weight_2.weight", "w2b": "hyper_net_weight_2.bias",
    "b1W": "hyper_net_bias_1.weight", "b1b": "hyper_net_bias_1.bias",
    "b2aW": "hyper_net_bias_2.0.weight", "b2ab": "hyper_net_bias_2.0.bias",
    "b2bW": "hyper_net_bias_2.2.weight", "b2bb": "hyper_net_bias_2.2.bias",
}


def _n_agents(sd, fmt):
    n = 0
    while fmt["W1"].format(i=n) in sd:
        n += 1
    return n


def agent_from_state(sd, prefix="", style="qmix"):
    """Stack a reference Q_Net / QNet state_dict (dict of arrays) into AGENT_KEYS tensors."""
    fmt = _FMTS[style]
    sd = {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}
    n = _n_agents(sd, fmt)
    return {k: torch.tensor(np.stack([np.asarray(sd[f.format(i=i)]) for i in range(n)]), dtype=torch.float32)
            for k, f in fmt.items()}


def agent_to_state(P, style="qmix"):
    fmt = _QMIX_FMT if style == "qmix" else _VDN_FMT
    out = {}
    for k, f in fmt.items():
        for i in range(P[k].shape[0]):
            out[f.format(i=i)] = P[k][i].detach().numpy()
    return out


def mixer_from_state(sd, prefix=""):
    return {k: torch.tensor(np.asarray(sd[prefix + f]), dtype=torch.float32) for k, f in _MIX_FMT.items()}


def mixer_to_state(M):
    return {f: M[k].detach().numpy() for k, f in _MIX_FMT.items()}


def gru_cell(x, h, Wih, Whh, bih, bhh):
    """torch.nn.GRUCell semantics (gate order r, z, n); h' = n + z*(h-n)."""
    gi = F.linear(x, Wih, bih)
    gh = F.linear(h, Whh, bhh)
    ir, iz, inn = gi.chunk(3, dim=1)
    hr, hz, hn = gh.chunk(3, dim=1)
    r = torch.sigmoid(ir + hr)
    z = torch.sigmoid(iz + hz)
    n = torch.tanh(inn + r * hn)
    return n + z * (h - n)


def agent_forward(P, obs, hidden):
    """Q_Net.forward: per-agent MLP D->F1->G (ReLU) -> GRUCell(G,H) -> Linear(H->A).

    qmix/_network.py:44-64, vdn/_network.py:71-83. obs [B,N,D], hidden [B,N,H]
    -> q [B,N,A], next_hidden [B,N,H].
    """
    n = P["W1"].shape[0]
    qs, hs = [], []
    for i in range(n):
        x = F.relu(F.linear(obs[:, i, :], P["W1"][i], P["b1"][i]))
        x = F.relu(F.linear(x, P["W2"][i], P["b2"][i]))
        h = gru_cell(x, hidden[:, i, :], P["Wih"][i], P["Whh"][i], P["bih"][i], P["bhh"][i])
        hs.append(h)
        qs.append(F.linear(h, P["Wq"][i], P["bq"][i]))
    return torch.stack(qs, 1), torch.stack(hs, 1)


def epsilon_greedy(q, epsilon, u, rand_actions):
    """vdn/_network.py:52-58 with the RNG draws injected.

    One uniform u[b] per env row (mask = u <= eps: all agents of a row random or
    all greedy); random rows take rand_actions[b, :]; greedy rows take the first
    argmax. Returns float actions [B,N] like the reference.
    """
    u = torch.as_tensor(u)
    mask = (u <= epsilon)
    greedy = q.argmax(dim=2)
    ra = torch.as_tensor(rand_actions).long()
    return torch.where(mask[:, None], ra, greedy).float()


def cal_td_error(action, reward, done, behavior_q, target_q, gamma):
    """vdn/_utils.py:44-52: |sum(r) + (1-d)*gamma*sum_i max_a Q'_i - sum_i Q_{i,a_i}| (float)."""
    action_index = torch.as_tensor(action).long().reshape(-1, 1)
    behavior_value = torch.gather(behavior_q[0], 1, action_index).reshape(1, -1)[0].sum(dim=0)
    target_max_q = target_q.max(dim=2)[0][0].sum(dim=0)
    target_value = sum(reward) + (1 - done) * gamma * target_max_q
    return abs(target_value - behavior_value).item()


def mixer_forward(M, q, obs, hidden, hidden_dim=32):
    """Mix_Net.forward, qmix/_network.py:199-217. q [B,N], obs [B,N,D], hidden [B,Hm]."""
    b, n, d = obs.shape
    state = obs.reshape(b, n * d)
    h = gru_cell(state, hidden, M["gWih"], M["gWhh"], M["gbih"], M["gbhh"])
    w1 = torch.abs(F.linear(h, M["w1W"], M["w1b"])).view(b, hidden_dim, n)   # W1[b,k,i] = out[b, k*N+i]
    b1 = F.linear(h, M["b1W"], M["b1b"]).unsqueeze(-1)
    w2 = torch.abs(F.linear(h, M["w2W"], M["w2b"]))
    b2 = F.linear(F.relu(F.linear(h, M["b2aW"], M["b2ab"])), M["b2bW"], M["b2bb"])
    y = torch.relu(torch.bmm(w1, q.unsqueeze(-1)) + b1)
    return (w2.unsqueeze(-1) * y).sum(dim=1) + b2, h


def _requires(P):
    return {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}


def clip_grad_norm(tensors, max_norm):
    """torch.nn.utils.clip_grad_norm_ semantics: coef = max_norm/(total+1e-6), clamped to 1."""
    total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g, 2) for g in tensors]), 2)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    return [g * coef for g in tensors], total


def adam_step(params, grads, state, lr, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam (no amsgrad, no weight decay) single step; state: dict name->(m, v, t)."""
    out = {}
    for k, p in params.items():
        g = grads[k]
        m, v, t = state.get(k, (torch.zeros_like(p), torch.zeros_like(p), 0))
        t += 1
        m = m * betas[0] + g * (1 - betas[0])
        v = v * betas[1] + g * g * (1 - betas[1])
        bc1 = 1 - betas[0] ** t
        bc2 = 1 - betas[1] ** t
        denom = (v.sqrt() / (bc2 ** 0.5)) + eps
        out[k] = p - (lr / bc1) * (m / denom)
        state[k] = (m, v, t)
    return out


def vdn_loss(P, T, batch, gamma):
    """Target_Dqn.train inner loop, vdn/_train.py:197-221 (one update, hidden zero at chunk start).

    batch: states [B,C,N,D], actions [B,C,N], rewards [B,C,N], next_states, dones [B,C,1], is_weight [B,1].
    Returns (loss, last-step target_values, last-step sum_q).
    """
    s, a, r, s2, d, w = batch
    B, C, N, _ = s.shape
    H = P["Whh"].shape[2]
    h = torch.zeros(B, N, H)
    ht = torch.zeros(B, N, H)
    loss = 0.0
    for t in range(C):
        q, nh = agent_forward(P, s[:, t], h)
        sum_q = q.gather(2, a[:, t].unsqueeze(-1).long()).squeeze(-1).sum(1, keepdim=True)
        tq, nht = agent_forward(T, s2[:, t], ht.detach())
        sum_tq = tq.max(dim=2)[0].sum(1, keepdim=True)
        # quirk (App. A 1-2): w * (r[B,N] + gamma*(1-d)*Q'[B,1]).sum(1)  => sum r + N*gamma*(1-d)*Q'
        target = w * (r[:, t] + gamma * (1 - d[:, t]) * sum_tq).sum(dim=1, keepdim=True)
        loss = loss + F.mse_loss(target.detach(), sum_q)
        keep = (1.0 - d[:, t]).view(B, 1, 1)
        h = nh * keep
        ht = nht * keep
    return loss, target.detach(), sum_q


def vdn_train_step(P, T, batch, gamma, lr, grad_clip, adam_state=None):
    """One Target_Dqn update (vdn/_train.py:190-233): loss, backward, clip (all params), Adam."""
    Pg = _requires(P)
    loss, target, sum_q = vdn_loss(Pg, T, batch, gamma)
    grads = torch.autograd.grad(loss, [Pg[k] for k in AGENT_KEYS])
    grads, _ = clip_grad_norm(list(grads), grad_clip)
    g = dict(zip(AGENT_KEYS, grads))
    state = {} if adam_state is None else adam_state
    newP = adam_step({k: P[k] for k in AGENT_KEYS}, g, state, lr)
    new_td = (target - sum_q.detach()).abs().view(-1)
    return newP, g, loss.detach(), new_td


def vdn_double_loss(P, T, batch, gamma, epsilon, draws_u, draws_ra):
    """Target_Double_Dqn.train inner loop, vdn/_train.py:112-141 (one update).

    The double network (a copy of the behavior net, :110) picks eps-greedy actions on s' with its
    own hidden chain (draws injected: u [C,B], rand actions [C,B,N]); the bootstrap is
    sum_i Q_tgt(s')_{i, a*_i} (:127-129); target and loss as Target_Dqn (xN quirk, IS weight).
    """
    s, a, r, s2, d, w = batch
    B, C, N, _ = s.shape
    H = P["Whh"].shape[2]
    Pd = {k: v.detach() for k, v in P.items()}
    h = torch.zeros(B, N, H)
    ht = torch.zeros(B, N, H)
    hd = torch.zeros(B, N, H)
    loss = 0.0
    for t in range(C):
        q, nh = agent_forward(P, s[:, t], h)
        sum_q = q.gather(2, a[:, t].unsqueeze(-1).long()).squeeze(-1).sum(1, keepdim=True)
        tq, nht = agent_forward(T, s2[:, t], ht.detach())
        dq, nhd = agent_forward(Pd, s2[:, t], hd)
        act = epsilon_greedy(dq, epsilon, draws_u[t], draws_ra[t])
        sum_dq = tq.gather(2, act.long().unsqueeze(-1)).squeeze(-1).sum(1, keepdim=True)
        target = w * (r[:, t] + gamma * (1 - d[:, t]) * sum_dq).sum(dim=1, keepdim=True)
        loss = loss + F.mse_loss(target.detach(), sum_q)
        keep = (1.0 - d[:, t]).view(B, 1, 1)
        h, ht, hd = nh * keep, nht * keep, nhd * keep
    return loss, target.detach(), sum_q


def vdn_double_train_step(P, T, batch, gamma, lr, grad_clip, epsilon, draws_u, draws_ra, adam_state=None):
    """One Target_Double_Dqn update: loss, backward, clip (behavior params), Adam (vdn/_train.py:143-147)."""
    Pg = _requires(P)
    loss, target, sum_q = vdn_double_loss(Pg, T, batch, gamma, epsilon, draws_u, draws_ra)
    grads = torch.autograd.grad(loss, [Pg[k] for k in AGENT_KEYS])
    grads, _ = clip_grad_norm(list(grads), grad_clip)
    g = dict(zip(AGENT_KEYS, grads))
    state = {} if adam_state is None else adam_state
    newP = adam_step({k: P[k] for k in AGENT_KEYS}, g, state, lr)
    return newP, g, loss.detach(), (target - sum_q.detach()).abs().view(-1)


def qmix_loss(P, M, T, TM, batch, gamma, hidden_dim=32):
    """Train_dqn.train inner loop, qmix/_train.py:39-103 (one update).

    Hidden reset "rows where done" for every batch size (the reference indexes
    mix hidden with a [B]-mask on a [Hm]-row, which only runs at B == Hm == 32;
    at B == 32 the semantics coincide).
    """
    s, a, r, s2, d, w = batch
    B, C, N, _ = s.shape
    H = P["Whh"].shape[2]
    Hm = M["gWhh"].shape[1]
    h = torch.zeros(B, N, H)
    ht = torch.zeros(B, N, H)
    hm = torch.zeros(B, Hm)
    hmt = torch.zeros(B, Hm)
    loss = 0.0
    for t in range(C):
        q, nh = agent_forward(P, s[:, t], h)
        qa = q.gather(2, a[:, t].unsqueeze(-1).long()).squeeze(-1)
        qtot, nhm = mixer_forward(M, qa, s[:, t], hm, hidden_dim)
        tq, nht = agent_forward(T, s2[:, t], ht.detach())
        tmax = tq.max(dim=2)[0]
        tqtot, nhmt = mixer_forward(TM, tmax, s2[:, t], hmt.detach(), hidden_dim)
        target = w * (r[:, t] + gamma * (1 - d[:, t]) * tqtot).sum(dim=1, keepdim=True)
        loss = loss + F.mse_loss(target.detach(), qtot)
        keep = (1.0 - d[:, t]).view(B, 1)
        h = nh * keep.view(B, 1, 1)
        ht = nht * keep.view(B, 1, 1)
        hm = nhm * keep
        hmt = nhmt * keep
    return loss, target.detach(), qtot


def qmix_qtot(P, M, batch, hidden_dim=32):
    """Behavior Q_tot of every (t, b) of a chunk batch, [C, B] (the forward half of qmix_loss,
    qmix/_train.py:55-75, hiddens reset where done)."""
    s, a, _, _, d, _ = batch
    B, C, N, _ = s.shape
    H = P["Whh"].shape[2]
    Hm = M["gWhh"].shape[1]
    h = torch.zeros(B, N, H)
    hm = torch.zeros(B, Hm)
    out = []
    with torch.no_grad():
        for t in range(C):
            q, nh = agent_forward(P, s[:, t], h)
            qa = q.gather(2, a[:, t].unsqueeze(-1).long()).squeeze(-1)
            qtot, nhm = mixer_forward(M, qa, s[:, t], hm, hidden_dim)
            out.append(qtot.view(B))
            keep = (1.0 - d[:, t]).view(B, 1)
            h = nh * keep.view(B, 1, 1)
            hm = nhm * keep
    return torch.stack(out)


def qmix_train_step(P, M, T, TM, batch, gamma, lr, grad_clip, adam_state=None, hidden_dim=32):
    """One Train_dqn update: backward, clip_grad_norm_ over AGENT params only
    (qmix/_train.py:111-115), Adam over agent + mixer (qmix/main.py:79-85)."""
    Pg = _requires(P)
    Mg = _requires(M)
    loss, target, qtot = qmix_loss(Pg, Mg, T, TM, batch, gamma, hidden_dim)
    allp = [Pg[k] for k in AGENT_KEYS] + [Mg[k] for k in MIXER_KEYS]
    grads = torch.autograd.grad(loss, allp)
    ga, _ = clip_grad_norm(list(grads[:len(AGENT_KEYS)]), grad_clip)
    gm = list(grads[len(AGENT_KEYS):])
    g = dict(zip(AGENT_KEYS, ga))
    g.update(dict(zip(["m." + k for k in MIXER_KEYS], gm)))
    state = {} if adam_state is None else adam_state
    params = {k: P[k] for k in AGENT_KEYS}
    params.update({"m." + k: M[k] for k in MIXER_KEYS})
    new = adam_step(params, g, state, lr)
    newP = {k: new[k] for k in AGENT_KEYS}
    newM = {k: new["m." + k] for k in MIXER_KEYS}
    new_td = (target - qtot.detach()).abs().view(-1)
    return newP, newM, g, loss.detach(), new_td


def qmix_min_loss(P, M, T, TM, batch, gamma, hidden_dim=32):
    """Minimal QMIX train inner loop, qmix/qmix.py:186-230 (recurrent, one iteration).

    Differs from Train_dqn: target = sum_i r_i + gamma*Q'_tot*(1-d) (no xN, no IS weight,
    :215-217) and smooth_l1 (:218). Hidden handling is the same: done rows reset to zero for the
    agents (:221-225) and both mixers (:226-232); the target paths are detached.
    """
    s, a, r, s2, d = batch[:5]
    B, C, N, _ = s.shape
    H = P["Whh"].shape[2]
    Hm = M["gWhh"].shape[1]
    h = torch.zeros(B, N, H)
    ht = torch.zeros(B, N, H)
    hm = torch.zeros(B, Hm)
    hmt = torch.zeros(B, Hm)
    loss = 0.0
    for t in range(C):
        q, nh = agent_forward(P, s[:, t], h)
        qa = q.gather(2, a[:, t].unsqueeze(-1).long()).squeeze(-1)
        qtot, nhm = mixer_forward(M, qa, s[:, t], hm, hidden_dim)
        tq, nht = agent_forward(T, s2[:, t], ht.detach())
        tmax = tq.max(dim=2)[0]
        tqtot, nhmt = mixer_forward(TM, tmax, s2[:, t], hmt.detach(), hidden_dim)
        target = r[:, t].sum(dim=1, keepdim=True) + gamma * tqtot * (1 - d[:, t])
        loss = loss + F.smooth_l1_loss(qtot, target.detach())
        keep = (1.0 - d[:, t]).view(B, 1)
        h = nh * keep.view(B, 1, 1)
        ht = nht * keep.view(B, 1, 1)
        hm = nhm * keep
        hmt = nhmt * keep
    return loss


def qmix_min_train_step(P, M, T, TM, batch, gamma, lr, grad_clip=5.0, adam_state=None, hidden_dim=32):
    """qmix/qmix.py:233-238: backward, clip_grad_norm_ on the agent net and on the mixer
    separately, one Adam step over both (lr, default betas / eps 1e-8)."""
    Pg = _requires(P)
    Mg = _requires(M)
    loss = qmix_min_loss(Pg, Mg, T, TM, batch, gamma, hidden_dim)
    allp = [Pg[k] for k in AGENT_KEYS] + [Mg[k] for k in MIXER_KEYS]
    grads = torch.autograd.grad(loss, allp)
    ga, _ = clip_grad_norm(list(grads[:len(AGENT_KEYS)]), grad_clip)
    gm, _ = clip_grad_norm(list(grads[len(AGENT_KEYS):]), grad_clip)
    g = dict(zip(AGENT_KEYS, ga))
    g.update(dict(zip(["m." + k for k in MIXER_KEYS], gm)))
    state = {} if adam_state is None else adam_state
    params = {k: P[k] for k in AGENT_KEYS}
    params.update({"m." + k: M[k] for k in MIXER_KEYS})
    new = adam_step(params, g, state, lr)
    return ({k: new[k] for k in AGENT_KEYS}, {k: new["m." + k] for k in MIXER_KEYS}, g, loss.detach())


def batch_from_fixture(fx):
    return (torch.tensor(fx["states"]), torch.tensor(fx["actions"]), torch.tensor(fx["rewards"]),
            torch.tensor(fx["next_states"]), torch.tensor(fx["dones"]), torch.tensor(fx["is_weight"]))
