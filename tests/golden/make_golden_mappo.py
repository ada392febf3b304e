"""Generate golden vectors for the MAPPO hot path by importing the reference (rmappo, shared policy).

Runs ONLY in the build container (needs /root/reference, read-only); the GPU box only reads
the ``mappo_*.npz`` fixtures written next to this script. The reference imports ``gym`` (only
for the module name) and dispatches on space class names, so an in-memory ``gym`` stand-in with
``spaces.Box`` / ``spaces.Discrete`` is inserted. Every RNG draw the
reference makes (Categorical samples, torch.randperm) is recorded so the build can replay it.

  mappo_fwd.npz    R_MAPPOPolicy.get_actions (mappo/algorithms/rmappo_policy.py:57-90) and
                   evaluate_actions over data chunks with in-chunk mask zeros
                   (rmappo_policy.py:104-136, r_actor_critic.py:95-133,189-208, rnn.py:24-80)
  mappo_gae.npz    SharedReplayBuffer.compute_returns with ValueNorm
                   (mappo/runner/shared/shared_buffer.py:131-157, mappo/utils/valuenorm.py)
  mappo_train.npz  R_MAPPO.train (mappo/algorithms/ramppo_network.py:56-287) on a buffer filled
                   by a synthetic rollout (magym_runner.py:114-195 insert semantics)

Usage (from /root/repo):  python tests/golden/make_golden_mappo.py
"""
import importlib
import os
import random
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = "/root/reference/mappo"
OUT = os.path.dirname(os.path.abspath(__file__))


class Box:
    def __init__(self, low, high=None, shape=None, dtype=None):
        low = np.asarray(low, dtype=np.float32)
        self.low, self.high, self.shape = low, high, low.shape


class Discrete:
    def __init__(self, n):
        self.n = n


class Space:
    pass


def install_gym():
    gym = types.ModuleType("gym")
    sp = types.ModuleType("gym.spaces")
    sp.Box, sp.Discrete = Box, Discrete
    spc = types.ModuleType("gym.spaces.space")
    spc.Space = Space
    sp.space = spc
    gym.spaces = sp
    sys.modules.update({"gym": gym, "gym.spaces": sp, "gym.spaces.space": spc})


def load():
    install_gym()
    sys.path.insert(0, REF)
    try:
        m = types.SimpleNamespace()
        m.config = importlib.import_module("_config")
        m.policy = importlib.import_module("algorithms.rmappo_policy")
        m.trainer = importlib.import_module("algorithms.ramppo_network")
        m.buffer = importlib.import_module("runner.shared.shared_buffer")
        m.valuenorm = importlib.import_module("utils.valuenorm")
    finally:
        sys.path.pop(0)
    return m


def seed_all(s):
    random.seed(s)
    np.random.seed(s)
    torch.manual_seed(s)


def make_args(m, **kw):
    args = m.config.get_config().parse_known_args([])[0]
    for k, v in kw.items():
        setattr(args, k, v)
    return args


def sd(prefix, module):
    return {f"{prefix}{k}": v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


def gen_obs(rng, shape):
    """Checkers-like observations: 2 coords in [0,1], then {0,1} bits (p=0.2)."""
    o = (rng.random(shape) < 0.2).astype(np.float32)
    o[..., :2] = rng.random(shape[:-1] + (2,)).astype(np.float32)
    return o


class SampleRecorder:
    """Wraps torch.multinomial (Categorical.sample) to record the drawn actions."""

    def __init__(self):
        self.draws = []
        self._orig = torch.multinomial

    def __enter__(self):
        def rec(*a, **k):
            out = self._orig(*a, **k)
            self.draws.append(out.detach().cpu().numpy().copy())
            return out
        torch.multinomial = rec
        return self

    def __exit__(self, *exc):
        torch.multinomial = self._orig


def fwd_fixture(m):
    seed_all(42)
    D, A, H, N, E = 47, 5, 32, 2, 6
    args = make_args(m)
    pol = m.policy.R_MAPPOPolicy(args, Box(np.zeros(D)), Box(np.zeros(D)), Discrete(A), torch.device("cpu"))
    rng = np.random.default_rng(1)
    R = E * N
    obs = gen_obs(rng, (R, D))
    ha = (rng.standard_normal((R, 1, H)) * 0.5).astype(np.float32)
    hc = (rng.standard_normal((R, 1, H)) * 0.5).astype(np.float32)
    masks = np.ones((R, 1), np.float32)
    masks[[1, 4, 7]] = 0.0
    with torch.no_grad(), SampleRecorder() as rec:
        v, a, lp, ha2, hc2 = pol.get_actions(obs, obs, ha, hc, masks)
    out = dict(obs=obs, ha=ha, hc=hc, masks=masks, values=v.numpy(), actions=a.numpy(), logp=lp.numpy(),
               ha_out=ha2.numpy(), hc_out=hc2.numpy(), draws=np.stack(rec.draws))
    # training path: chunks of L steps for n sequences, masks with zeros inside the chunk
    L, n = 5, 7
    sobs = gen_obs(rng, (L * n, D))
    sh = (rng.standard_normal((n, 1, H)) * 0.5).astype(np.float32)
    shc = (rng.standard_normal((n, 1, H)) * 0.5).astype(np.float32)
    smask = np.ones((L * n, 1), np.float32)
    smask[[0 * n + 2, 2 * n + 1, 2 * n + 5, 3 * n + 1]] = 0.0   # (step l, seq j) at row l*n + j
    sact = rng.integers(0, A, (L * n, 1)).astype(np.float32)
    sactive = np.ones((L * n, 1), np.float32)
    sactive[[4, 11]] = 0.0
    with torch.no_grad():
        sv, slp, sent = pol.evaluate_actions(sobs, sobs, sh, shc, sact, smask, None, sactive)
    out.update(seq_obs=sobs, seq_ha=sh, seq_hc=shc, seq_masks=smask, seq_actions=sact, seq_active=sactive,
               seq_values=sv.numpy(), seq_logp=slp.numpy(), seq_entropy=np.float32(sent.item()),
               seq_L=np.int64(L), seq_n=np.int64(n))
    out.update(sd("actor.", pol.actor))
    out.update(sd("critic.", pol.critic))
    np.savez(os.path.join(OUT, "mappo_fwd.npz"), **out)


def gae_fixture(m):
    seed_all(7)
    E, N, T = 3, 2, 8
    args = make_args(m, batch_size=E, max_step=T)
    buf = m.buffer.SharedReplayBuffer(args, N, Box(np.zeros(47)), Box(np.zeros(47)), Discrete(5))
    rng = np.random.default_rng(2)
    buf.rewards[:] = rng.choice([-0.01, 0.99, -1.01, 9.99, -10.01], size=buf.rewards.shape).astype(np.float32)
    buf.value_preds[:] = rng.standard_normal(buf.value_preds.shape).astype(np.float32)
    buf.masks[:] = 1.0
    buf.masks[3, 1] = 0.0
    buf.masks[6, :, 0] = 0.0
    buf.masks[T, 2] = 0.0
    vn = m.valuenorm.ValueNorm(1)
    for _ in range(3):
        vn.update(torch.from_numpy(rng.standard_normal((50, 1)).astype(np.float32) * 3 + 1))
    nv = rng.standard_normal((E, N, 1)).astype(np.float32)
    pre = dict(rewards=buf.rewards.copy(), value_preds=buf.value_preds.copy(), masks=buf.masks.copy(), next_value=nv)
    buf.compute_returns(nv, vn)
    pre.update(returns=buf.returns.copy(), vn_mean=vn.running_mean.detach().numpy().copy(),
               vn_mean_sq=vn.running_mean_sq.detach().numpy().copy(),
               vn_debias=vn.debiasing_term.detach().numpy().copy(), gamma=np.float32(args.gamma),
               gae_lambda=np.float32(args.gae_lambda))
    np.savez(os.path.join(OUT, "mappo_gae.npz"), **pre)


def train_fixture(m):
    seed_all(42)
    D, A, H, N, E, T, L, EPOCHS = 47, 5, 32, 2, 4, 10, 5, 3
    args = make_args(m, batch_size=E, max_step=T, ppo_epoch=EPOCHS, data_chunk_length=L)
    pol = m.policy.R_MAPPOPolicy(args, Box(np.zeros(D)), Box(np.zeros(D)), Discrete(A), torch.device("cpu"))
    tr = m.trainer.R_MAPPO(args, pol, torch.device("cpu"))
    buf = m.buffer.SharedReplayBuffer(args, N, Box(np.zeros(D)), Box(np.zeros(D)), Discrete(A))
    rng = np.random.default_rng(3)
    buf.obs[0] = gen_obs(rng, (E, N, D))
    buf.share_obs[0] = buf.obs[0]
    done_at = {3: [1], 7: [0, 2]}          # step -> envs whose episode ends (all agents done)
    agent_done = {5: [(3, 1)]}             # step -> (env, agent) done while the env goes on
    for t in range(T):
        with torch.no_grad():
            v, a, lp, ha, hc = pol.get_actions(np.concatenate(buf.obs[t]), np.concatenate(buf.share_obs[t]),
                                               np.concatenate(buf.rnn_states[t]),
                                               np.concatenate(buf.rnn_states_critic[t]),
                                               np.concatenate(buf.masks[t]))
        sp = lambda x: np.array(np.split(x.numpy(), E))
        v, a, lp, ha, hc = sp(v), sp(a), sp(lp), sp(ha), sp(hc)
        nobs = gen_obs(rng, (E, N, D))
        rew = rng.choice([-0.01, 0.99, -1.01, 9.99], size=(E, N, 1)).astype(np.float32)
        dones = np.zeros((E, N), bool)
        for e in done_at.get(t, []):
            dones[e] = True
        for e, k in agent_done.get(t, []):
            dones[e, k] = True
        dones_env = dones.all(axis=1)
        ha[dones_env] = 0.0
        hc[dones_env] = 0.0
        masks = np.ones((E, N, 1), np.float32)
        masks[dones_env] = 0.0
        active = np.ones((E, N, 1), np.float32)
        active[dones] = 0.0
        active[dones_env] = 1.0
        buf.insert(nobs, nobs, ha, hc, a, lp, v, rew, masks, active_masks=active)
    with torch.no_grad():
        nv = pol.get_values(np.concatenate(buf.share_obs[-1]), np.concatenate(buf.rnn_states_critic[-1]),
                            np.concatenate(buf.masks[-1]))
    buf.compute_returns(np.array(np.split(nv.numpy(), E)), tr.value_normalizer)
    before = {}
    before.update(sd("actor.", pol.actor))
    before.update(sd("critic.", pol.critic))
    vn0 = {k: v.detach().numpy().copy() for k, v in tr.value_normalizer.state_dict().items()}
    data = dict(obs=buf.obs.copy(), rnn_states=buf.rnn_states.copy(), rnn_states_critic=buf.rnn_states_critic.copy(),
                actions=buf.actions.copy(), action_log_probs=buf.action_log_probs.copy(),
                value_preds=buf.value_preds.copy(), returns=buf.returns.copy(), masks=buf.masks.copy(),
                active_masks=buf.active_masks.copy(), rewards=buf.rewards.copy())
    # record randperm draws, the clipped grads fed to each Adam step, and the pre-clip norms
    perms, grads, norms = [], [], []
    orig_perm, orig_clip = torch.randperm, torch.nn.utils.clip_grad_norm_

    def perm(*a, **k):
        p = orig_perm(*a, **k)
        perms.append(p.numpy().copy())
        return p

    def clip(params, *a, **k):
        params = list(params)
        n = orig_clip(params, *a, **k)
        norms.append(float(n))
        return n

    for opt, tag in ((pol.actor_optimizer, "a"), (pol.critic_optimizer, "c")):
        step0 = opt.step

        def wrapped(*a, _s=step0, _o=opt, _t=tag, **k):
            grads.append((_t, [p.grad.detach().numpy().copy() if p.grad is not None else None
                               for g in _o.param_groups for p in g["params"]]))
            return _s(*a, **k)
        opt.step = wrapped
    torch.randperm, torch.nn.utils.clip_grad_norm_ = perm, clip
    try:
        info = tr.train(buf)
    finally:
        torch.randperm, torch.nn.utils.clip_grad_norm_ = orig_perm, orig_clip
    after = {}
    after.update(sd("actor.", pol.actor))
    after.update(sd("critic.", pol.critic))
    vn1 = {k: v.detach().numpy().copy() for k, v in tr.value_normalizer.state_dict().items()}
    out = {f"data.{k}": v for k, v in data.items()}
    out.update({f"before.{k}": v for k, v in before.items()})
    out.update({f"after.{k}": v for k, v in after.items()})
    out.update({f"vn0.{k}": v for k, v in vn0.items()})
    out.update({f"vn1.{k}": v for k, v in vn1.items()})
    out["perms"] = np.stack(perms)
    out["norms"] = np.array(norms, np.float64)
    names_a = [n for n, _ in pol.actor.named_parameters()]
    names_c = [n for n, _ in pol.critic.named_parameters()]
    ia = ic = 0
    for tag, gl in grads:
        names = names_a if tag == "a" else names_c
        idx = ia if tag == "a" else ic
        for n, g in zip(names, gl):
            if g is not None:
                out[f"grad{tag}{idx}.{n}"] = g
        if tag == "a":
            ia += 1
        else:
            ic += 1
    for k in ("value_loss", "policy_loss", "dist_entropy", "actor_grad_norm", "critic_grad_norm"):
        out[f"info.{k}"] = np.float64(info[k])
    out["info.ratio"] = np.float64(float(info["ratio"]))
    out.update(dict(E=np.int64(E), N=np.int64(N), T=np.int64(T), L=np.int64(L), epochs=np.int64(EPOCHS),
                    gamma=np.float32(args.gamma), gae_lambda=np.float32(args.gae_lambda)))
    np.savez(os.path.join(OUT, "mappo_train.npz"), **out)


if __name__ == "__main__":
    m = load()
    fwd_fixture(m)
    gae_fixture(m)
    train_fixture(m)
    print("wrote mappo_fwd.npz, mappo_gae.npz, mappo_train.npz")
