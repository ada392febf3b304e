"""Oracle (test infrastructure only): MAPPO (rmappo, shared policy) restated in torch-CPU fp32.

Pinned against tests/golden/mappo_*.npz (tests/golden/make_golden_mappo.py imports the
reference). Autograd is used only for the PPO gradients. Parameters of one net (actor or
critic) are a dict over NET_KEYS; converters from the reference state_dict naming below.

  net_step          MLPBase + RNNLayer + head: mappo/utils/algorithm_utils/mlp.py:31-55 (LN(D),
                    [Linear, ReLU, LN] x 2 -- fc_h is built but unused, mlp.py:20-27),
                    rnn.py:24-29,79 (GRU on h*mask, LayerNorm on the output only),
                    r_actor_critic.py:82-93 (actor Categorical), :203-208 (critic v_out)
  evaluate_chunks   rnn.py:30-77 training path == per-step h <- h*mask_t (segments at zeros)
  ValueNorm         mappo/utils/valuenorm.py:8-78 (f32 running stats, beta 0.99999)
  compute_returns   mappo/runner/shared/shared_buffer.py:131-153 (delta in f32, gae in f64)
  ppo_train         mappo/algorithms/ramppo_network.py:56-287 + recurrent_generator
                    (shared_buffer.py:318-427) + clip_grad_norm_ + Adam(eps 1e-5)
  sample_actions    the build's own sampler (inverse CDF of the softmax over a uniform u);
                    torch.multinomial's stream is not reproducible on device, so the golden
                    test replays the reference's recorded samples instead (GATHER).
"""
import numpy as np
import torch

NET_KEYS = ["ln0_w", "ln0_b", "W1", "b1", "ln1_w", "ln1_b", "W2", "b2", "ln2_w", "ln2_b",
            "Wih", "Whh", "bih", "bhh", "lnr_w", "lnr_b", "Wo", "bo"]
_REF = {
    "ln0_w": "base.feature_norm.weight", "ln0_b": "base.feature_norm.bias",
    "W1": "base.mlp.fc1.0.weight", "b1": "base.mlp.fc1.0.bias",
    "ln1_w": "base.mlp.fc1.2.weight", "ln1_b": "base.mlp.fc1.2.bias",
    "W2": "base.mlp.fc2.0.0.weight", "b2": "base.mlp.fc2.0.0.bias",
    "ln2_w": "base.mlp.fc2.0.2.weight", "ln2_b": "base.mlp.fc2.0.2.bias",
    "Wih": "rnn.rnn.weight_ih_l0", "Whh": "rnn.rnn.weight_hh_l0",
    "bih": "rnn.rnn.bias_ih_l0", "bhh": "rnn.rnn.bias_hh_l0",
    "lnr_w": "rnn.norm.weight", "lnr_b": "rnn.norm.bias",
}
_HEAD = {"actor": ("act.action_out.linear.weight", "act.action_out.linear.bias"),
         "critic": ("v_out.weight", "v_out.bias")}
LN_EPS = 1e-5


def ref_name(key, kind):
    if key in ("Wo", "bo"):
        return _HEAD[kind][0 if key == "Wo" else 1]
    return _REF[key]


def net_from_state(sd, prefix, kind):
    """kind: 'actor' | 'critic'. sd: dict of arrays with reference names under prefix."""
    return {k: torch.tensor(np.asarray(sd[prefix + ref_name(k, kind)]), dtype=torch.float32) for k in NET_KEYS}


def layer_norm(x, w, b):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + LN_EPS) * w + b


def gru_cell(x, h, Wih, Whh, bih, bhh):
    gi = x @ Wih.t() + bih
    gh = h @ Whh.t() + bhh
    H = h.shape[-1]
    r = torch.sigmoid(gi[..., :H] + gh[..., :H])
    z = torch.sigmoid(gi[..., H:2 * H] + gh[..., H:2 * H])
    n = torch.tanh(gi[..., 2 * H:] + r * gh[..., 2 * H:])
    return (1 - z) * n + z * h


def net_step(P, obs, h, mask):
    """One step of an R_Actor / R_Critic trunk: returns (head output [R,O], new hidden [R,H])."""
    f = layer_norm(obs, P["ln0_w"], P["ln0_b"])
    f = layer_norm(torch.relu(f @ P["W1"].t() + P["b1"]), P["ln1_w"], P["ln1_b"])
    f = layer_norm(torch.relu(f @ P["W2"].t() + P["b2"]), P["ln2_w"], P["ln2_b"])
    h2 = gru_cell(f, h * mask, P["Wih"], P["Whh"], P["bih"], P["bhh"])
    y = layer_norm(h2, P["lnr_w"], P["lnr_b"])
    return y @ P["Wo"].t() + P["bo"], h2


def categorical(logits):
    logp = torch.log_softmax(logits, -1)
    return logp, -(logp.exp() * logp).sum(-1)


def sample_actions(logits, u):
    """The build's sampler: smallest a with u < cumsum(softmax)[a] (last action if none)."""
    p = torch.softmax(logits, -1)
    c = torch.cumsum(p, -1)
    a = (u.unsqueeze(-1) >= c).sum(-1).clamp(max=logits.shape[-1] - 1)
    return a


def get_actions(PA, PC, obs, ha, hc, masks, actions=None, u=None):
    """R_MAPPOPolicy.get_actions with the sample either given (actions) or drawn from u."""
    logits, ha2 = net_step(PA, obs, ha, masks)
    v, hc2 = net_step(PC, obs, hc, masks)
    logp_all, _ = categorical(logits)
    if actions is None:
        actions = sample_actions(logits, u)
    lp = logp_all.gather(-1, actions.long().view(-1, 1))
    return v, actions.view(-1, 1), lp, ha2, hc2


def evaluate_chunks(P, obs, h0, masks, L, head="actor", actions=None, active=None):
    """Training path on rows ordered (l, j) = l*n + j; h0 [n,H] is the chunk-start hidden."""
    n = h0.shape[0]
    h = h0
    outs = []
    for l in range(L):
        o, h = net_step(P, obs[l * n:(l + 1) * n], h, masks[l * n:(l + 1) * n])
        outs.append(o)
    out = torch.cat(outs, 0)
    if head == "critic":
        return out
    logp_all, ent = categorical(out)
    lp = logp_all.gather(-1, actions.long().view(-1, 1))
    ent_mean = (ent * active.view(-1)).sum() / active.sum()
    return lp, ent_mean


class ValueNorm:
    """mappo/utils/valuenorm.py: f32 running statistics."""

    def __init__(self, mean=0.0, mean_sq=0.0, debias=0.0, beta=0.99999, eps=1e-5):
        self.m = torch.tensor([mean], dtype=torch.float32).view(1)
        self.msq = torch.tensor([mean_sq], dtype=torch.float32).view(1)
        self.d = torch.tensor(debias, dtype=torch.float32)
        self.beta, self.eps = beta, eps

    def mean_var(self):
        dm = self.m / self.d.clamp(min=self.eps)
        dsq = self.msq / self.d.clamp(min=self.eps)
        return dm, (dsq - dm ** 2).clamp(min=1e-2)

    def update(self, x):
        x = torch.as_tensor(x, dtype=torch.float32)
        bm = x.reshape(-1, 1).mean(0)
        bsq = (x.reshape(-1, 1) ** 2).mean(0)
        w = self.beta
        self.m = self.m * w + bm * (1.0 - w)
        self.msq = self.msq * w + bsq * (1.0 - w)
        self.d = self.d * w + 1.0 * (1.0 - w)

    def normalize(self, x):
        mu, var = self.mean_var()
        return (torch.as_tensor(x) - mu) / torch.sqrt(var)

    def denormalize(self, x):
        mu, var = self.mean_var()
        return (torch.as_tensor(x) * torch.sqrt(var) + mu).numpy()


def compute_returns(rewards, value_preds, masks, next_value, vn, gamma, gae_lambda):
    """shared_buffer.py:139-148 with ValueNorm; arrays [T(+1),E,N,1] float32; returns [T+1,E,N,1]."""
    vp = value_preds.copy()
    vp[-1] = next_value
    T = rewards.shape[0]
    ret = np.zeros_like(vp)
    gae = np.zeros(rewards.shape[1:], np.float64)
    g32, gl = np.float32(gamma), gamma * gae_lambda
    for t in reversed(range(T)):
        dn1 = vn.denormalize(vp[t + 1])
        dn0 = vn.denormalize(vp[t])
        delta = rewards[t] + g32 * dn1 * masks[t + 1] - dn0
        gae = delta + (np.float32(gl) * masks[t + 1]) * gae
        ret[t] = gae + dn0
    return ret, vp


def huber(e, d):
    a = (e.abs() <= d).float()
    b = (e.abs() > d).float()
    return a * e ** 2 / 2 + b * d * (e.abs() - d / 2)


def _cast(x):
    """[T,E,N,...] -> [(E,N,T), ...] (shared_buffer.py:11-12)."""
    return np.ascontiguousarray(np.moveaxis(x, 0, 2)).reshape(-1, *x.shape[3:])


def chunk_batch(data, adv, L, order=None):
    """recurrent_generator (shared_buffer.py:318-427) for one minibatch holding every chunk.

    Returns row-(l, j)-ordered tensors plus chunk-start hiddens [n,H]; ``order`` = chunk order
    (the reference's randperm), identity when None.
    """
    T, E, N = data["rewards"].shape[:3]
    n_chunks = T * E * N // L
    order = np.arange(n_chunks) if order is None else np.asarray(order)
    cast = {k: _cast(data[k][:-1] if data[k].shape[0] == T + 1 else data[k])
            for k in ("obs", "actions", "action_log_probs", "value_preds", "returns", "masks", "active_masks")}
    cast["adv"] = _cast(adv)
    rs = np.moveaxis(data["rnn_states"][:-1], 0, 2).reshape(-1, *data["rnn_states"].shape[3:])
    rsc = np.moveaxis(data["rnn_states_critic"][:-1], 0, 2).reshape(-1, *data["rnn_states_critic"].shape[3:])
    idx = order[None, :] * L + np.arange(L)[:, None]          # [L, n]
    out = {k: torch.from_numpy(np.ascontiguousarray(v[idx.reshape(-1)])) for k, v in cast.items()}
    out["ha0"] = torch.from_numpy(np.ascontiguousarray(rs[order * L][:, 0]))
    out["hc0"] = torch.from_numpy(np.ascontiguousarray(rsc[order * L][:, 0]))
    return out


def normalized_advantages(data, vn):
    adv = data["returns"][:-1] - vn.denormalize(data["value_preds"][:-1])
    a = adv.copy()
    a[data["active_masks"][:-1] == 0.0] = np.nan
    return (adv - np.nanmean(a)) / (np.nanstd(a) + 1e-5)


def ppo_losses(PA, PC, b, L, vn, clip=0.2, huber_delta=10.0, entropy_coef=0.01):
    """ramppo_network.py:103-200 on one minibatch (rows (l, j)); vn already updated by the caller."""
    lp, ent = evaluate_chunks(PA, b["obs"], b["ha0"], b["masks"], L, "actor", b["actions"], b["active_masks"])
    v = evaluate_chunks(PC, b["obs"], b["hc0"], b["masks"], L, "critic")
    m = b["active_masks"]
    ratio = torch.exp(lp - b["action_log_probs"])
    s1 = ratio * b["adv"]
    s2 = torch.clamp(ratio, 1.0 - clip, 1.0 + clip) * b["adv"]
    pol = (-torch.sum(torch.min(s1, s2), dim=-1, keepdim=True) * m).sum() / m.sum()
    vpc = b["value_preds"] + (v - b["value_preds"]).clamp(-clip, clip)
    tgt = vn.normalize(b["returns"])
    vl = torch.max(huber(tgt - v, huber_delta), huber(tgt - vpc, huber_delta))
    vloss = (vl * m).sum() / m.sum()
    return pol, ent, vloss, ratio


def clip_grads(gs, max_norm):
    total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g, 2) for g in gs]), 2)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    return [g * coef for g in gs], total


def adam(P, G, state, lr, eps, betas=(0.9, 0.999)):
    out = {}
    for k in P:
        if k not in G:
            out[k] = P[k]
            continue
        m, v, t = state.get(k, (torch.zeros_like(P[k]), torch.zeros_like(P[k]), 0))
        t += 1
        m = m * betas[0] + G[k] * (1 - betas[0])
        v = v * betas[1] + G[k] * G[k] * (1 - betas[1])
        denom = v.sqrt() / ((1 - betas[1] ** t) ** 0.5) + eps
        out[k] = P[k] - (lr / (1 - betas[0] ** t)) * (m / denom)
        state[k] = (m, v, t)
    return out


def ppo_train(PA, PC, data, vn, epochs, L, perms=None, lr=1e-4, eps=1e-5, max_norm=0.5,
              value_loss_coef=0.5, entropy_coef=0.01, record=None):
    """R_MAPPO.train with one minibatch per epoch (train_batch_size 1). Returns new PA, PC, vn."""
    adv = normalized_advantages(data, vn)
    sa, sc = {}, {}
    for ep in range(epochs):
        b = chunk_batch(data, adv, L, None if perms is None else perms[ep])
        pa = {k: v.detach().clone().requires_grad_(True) for k, v in PA.items()}
        pc = {k: v.detach().clone().requires_grad_(True) for k, v in PC.items()}
        vn.update(b["returns"])
        pol, ent, vloss, ratio = ppo_losses(pa, pc, b, L, vn, entropy_coef=entropy_coef)
        ga = torch.autograd.grad(pol - ent * entropy_coef, [pa[k] for k in NET_KEYS])
        gc = torch.autograd.grad(vloss * value_loss_coef, [pc[k] for k in NET_KEYS])
        ga, na = clip_grads(list(ga), max_norm)
        gc, nc = clip_grads(list(gc), max_norm)
        if record is not None:
            record.append(dict(ga=dict(zip(NET_KEYS, ga)), gc=dict(zip(NET_KEYS, gc)), na=float(na), nc=float(nc),
                               pol=float(pol.detach()), ent=float(ent.detach()), vloss=float(vloss.detach())))
        PA = adam(PA, dict(zip(NET_KEYS, ga)), sa, lr, eps)
        PC = adam(PC, dict(zip(NET_KEYS, gc)), sc, lr, eps)
    return PA, PC, vn
