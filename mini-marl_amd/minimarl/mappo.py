"""MAPPO (rmappo, shared policy) on the MI355X: policy, device rollout buffer, trainer, runner.

Mirrors the reference's MAPPO interface (mappo/algorithms/rmappo_policy.py R_MAPPOPolicy,
mappo/runner/shared/shared_buffer.py SharedReplayBuffer, mappo/algorithms/ramppo_network.py
R_MAPPO, mappo/runner/shared/magym_runner.py MAGYM_Runner) over the C ABI in
include/minimarl.h (csrc/mappo.hip). Everything runs on the GPU; there is no CPU path.

Deviations: E independent envs instead of one env stepped E times per timestep
(magym_runner.py:53-54); the rollout's Categorical sample uses the device counter RNG
(inverse CDF); the one PPO minibatch per epoch (train_batch_size 1) is processed in chunk
order instead of a torch.randperm order (a full-batch gradient: same value up to float
summation order, pinned by tests/test_mappo_oracle.py::test_ppo_train_golden[False]).
"""
import ctypes

import numpy as np
import torch

from ._lib import (MM_MAPPO_ROLLOUT, MM_MAPPO_TRAIN, MM_MAPPO_VALUES, MM_MLOSS_ENTROPY, MM_MLOSS_POLICY,
                   MM_MLOSS_RATIO, MM_MLOSS_VALUE, MappoBwdArgs, MappoDims, MappoFwdArgs, c_i64, check, lib)
from .qnet import ptr, stream_handle

KEYS = ["ln0_w", "ln0_b", "W1", "b1", "ln1_w", "ln1_b", "W2", "b2", "ln2_w", "ln2_b",
        "Wih", "Whh", "bih", "bhh", "lnr_w", "lnr_b", "Wo", "bo"]
# reference parameter names (mappo/algorithms/r_actor_critic.py, utils/algorithm_utils/*)
REF_NAMES = {
    "ln0_w": "base.feature_norm.weight", "ln0_b": "base.feature_norm.bias",
    "W1": "base.mlp.fc1.0.weight", "b1": "base.mlp.fc1.0.bias",
    "ln1_w": "base.mlp.fc1.2.weight", "ln1_b": "base.mlp.fc1.2.bias",
    "W2": "base.mlp.fc2.0.0.weight", "b2": "base.mlp.fc2.0.0.bias",
    "ln2_w": "base.mlp.fc2.0.2.weight", "ln2_b": "base.mlp.fc2.0.2.bias",
    "Wih": "rnn.rnn.weight_ih_l0", "Whh": "rnn.rnn.weight_hh_l0",
    "bih": "rnn.rnn.bias_ih_l0", "bhh": "rnn.rnn.bias_hh_l0",
    "lnr_w": "rnn.norm.weight", "lnr_b": "rnn.norm.bias",
}
HEAD_NAMES = {0: ("act.action_out.linear.weight", "act.action_out.linear.bias"), 1: ("v_out.weight", "v_out.bias")}


def ref_name(key, net):
    if key in ("Wo", "bo"):
        return HEAD_NAMES[net][0 if key == "Wo" else 1]
    return REF_NAMES[key]


class MappoNet:
    """One net's parameters (net 0 = R_Actor, net 1 = R_Critic) in the kernel's flat layout."""

    def __init__(self, net, obs_dim, n_actions=5, hidden=32, device="cuda", seed=None):
        self.net, self.D, self.A, self.H = int(net), int(obs_dim), int(n_actions), int(hidden)
        self.O = self.A if self.net == 0 else 1
        self.device = torch.device(device)
        self.dims = MappoDims(self.D, self.H, self.A)
        offs = (c_i64 * 19)()
        check(lib().mm_mappo_param_offsets(ctypes.byref(self.dims), self.net, offs), "mappo_param_offsets")
        self.offs = list(offs)
        self.total = self.offs[18]
        self.flat = torch.zeros(self.total, device=self.device)
        self.Dp, self.Op = (self.D + 3) // 4 * 4, (self.O + 3) // 4 * 4
        if seed is not None:
            self.init_default(seed)

    def shape(self, key):
        D, H, O = self.D, self.H, self.O
        return {"ln0_w": (D,), "ln0_b": (D,), "W1": (H, D), "b1": (H,), "ln1_w": (H,), "ln1_b": (H,),
                "W2": (H, H), "b2": (H,), "ln2_w": (H,), "ln2_b": (H,), "Wih": (3 * H, H), "Whh": (3 * H, H),
                "bih": (3 * H,), "bhh": (3 * H,), "lnr_w": (H,), "lnr_b": (H,), "Wo": (O, H), "bo": (O,)}[key]

    def view(self, key, t=None):
        """Logical view of one tensor inside ``t`` (default: the parameters); pads are excluded."""
        t = self.flat if t is None else t
        i = KEYS.index(key)
        o = self.offs[i]
        if key == "W1":
            return t[o:o + self.H * self.Dp].view(self.H, self.Dp)[:, :self.D]
        if key == "Wo":
            return t[o:o + self.Op * self.H].view(self.Op, self.H)[:self.O]
        n = int(np.prod(self.shape(key)))
        return t[o:o + n].view(self.shape(key))

    def init_default(self, seed):
        """The reference init (orthogonal weights, zero biases, unit LayerNorms; gain sqrt(2) for the
        ReLU MLP, 1 for the GRU and the value head, 0.01 for the policy head)."""
        g = torch.Generator().manual_seed(int(seed))
        self.flat.zero_()
        relu_gain = float(np.sqrt(2.0))
        for key in KEYS:
            shp = self.shape(key)
            if key.startswith("ln") and key.endswith("_w"):
                self.view(key).fill_(1.0)
            elif len(shp) == 2:
                w = torch.empty(shp)
                gain = relu_gain if key in ("W1", "W2") else (0.01 if (key == "Wo" and self.net == 0) else 1.0)
                torch.nn.init.orthogonal_(w, gain=gain, generator=g)
                self.view(key).copy_(w.to(self.device))

    def load_reference_state(self, sd, prefix=""):
        for k in KEYS:
            v = torch.as_tensor(np.asarray(sd[prefix + ref_name(k, self.net)]), dtype=torch.float32)
            self.view(k).copy_(v.to(self.device))

    def state_dict(self):
        return {ref_name(k, self.net): self.view(k).detach().cpu().clone() for k in KEYS}


def _ptrs(*ts):
    return [ptr(t) if t is not None else None for t in ts]


class MappoPolicy:
    """R_MAPPOPolicy (rmappo_policy.py:7-153): shared actor + critic for all agents."""

    def __init__(self, obs_dim, n_actions=5, hidden=32, device="cuda", seed=None):
        self.actor = MappoNet(0, obs_dim, n_actions, hidden, device, None if seed is None else seed)
        self.critic = MappoNet(1, obs_dim, n_actions, hidden, device, None if seed is None else seed + 1)
        self.dims = self.actor.dims
        self.D, self.A, self.H = int(obs_dim), int(n_actions), int(hidden)
        self.device = self.actor.device

    def _fwd(self, args):
        check(lib().mm_mappo_fwd(ctypes.byref(self.dims), ctypes.byref(args), stream_handle(self.device)),
              "mappo_fwd")

    def rollout_args(self, obs, ha, hc, masks, ha_out, hc_out, logp_out, value_out, act_out=None, act_in=None,
                     u=None, seed=0, counter=0, counter_ptr=None):
        a = MappoFwdArgs()
        a.net[0].P, a.net[0].h_in, a.net[0].h_out, a.net[0].out = _ptrs(self.actor.flat, ha, ha_out, logp_out)
        a.net[1].P, a.net[1].h_in, a.net[1].h_out, a.net[1].out = _ptrs(self.critic.flat, hc, hc_out, value_out)
        a.obs, a.mask, a.act_in, a.act_out, a.u = _ptrs(obs, masks, act_in, act_out, u)
        a.seed, a.counter, a.counter_ptr = int(seed), int(counter), counter_ptr
        a.rows = int(obs.shape[0])
        a.mode = MM_MAPPO_ROLLOUT
        return a

    def get_actions(self, obs, ha, hc, masks=None, actions=None, u=None, seed=0, counter=0):
        """obs [R,D], ha/hc [R,H], masks [R] -> values [R,1], actions [R,1], logp [R,1], ha', hc'.

        The sample is drawn by the device RNG (or from injected uniforms u [R]); pass ``actions``
        to evaluate given actions (the reference's get_actions always samples, rmappo_policy.py:86)."""
        R = obs.shape[0]
        dev = self.device
        ha2, hc2 = torch.empty(R, self.H, device=dev), torch.empty(R, self.H, device=dev)
        lp, v = torch.empty(R, device=dev), torch.empty(R, device=dev)
        act_in = None if actions is None else actions.reshape(-1).to(torch.int32).contiguous()
        act = torch.empty(R, dtype=torch.int32, device=dev) if actions is None else act_in
        self._fwd(self.rollout_args(obs.contiguous(), ha.contiguous(), hc.contiguous(),
                                    None if masks is None else masks.reshape(-1).contiguous(), ha2, hc2, lp, v,
                                    None if actions is not None else act, act_in, u, seed, counter))
        return v.view(R, 1), act.view(R, 1), lp.view(R, 1), ha2, hc2

    def get_values(self, obs, hc, masks=None):
        R = obs.shape[0]
        v = torch.empty(R, device=self.device)
        a = MappoFwdArgs()
        a.net[1].P, a.net[1].h_in, a.net[1].out = _ptrs(self.critic.flat, hc.contiguous(), v)
        a.obs, a.mask = _ptrs(obs.contiguous(), None if masks is None else masks.reshape(-1).contiguous())
        a.rows, a.mode = R, MM_MAPPO_VALUES
        self._fwd(a)
        return v.view(R, 1)


def _rs(rows):
    return (rows + 63) // 64 * 64


class MappoBuffer:
    """SharedReplayBuffer (shared_buffer.py:15-129) in HBM: [T(+1), EN, ...] with EN = envs*agents."""

    def __init__(self, T, n_envs, n_agents, obs_dim, hidden=32, device="cuda"):
        self.T, self.E, self.N, self.D, self.H = int(T), int(n_envs), int(n_agents), int(obs_dim), int(hidden)
        self.EN = self.E * self.N
        dev = self.device = torch.device(device)
        T, EN = self.T, self.EN
        self.obs = torch.zeros(T + 1, EN, self.D, device=dev)
        self.rnn_states = torch.zeros(T + 1, EN, self.H, device=dev)
        self.rnn_states_critic = torch.zeros(T + 1, EN, self.H, device=dev)
        self.value_preds = torch.zeros(T + 1, EN, device=dev)
        self.returns = torch.zeros(T + 1, EN, device=dev)
        self.actions = torch.zeros(T, EN, dtype=torch.int32, device=dev)
        self.action_log_probs = torch.zeros(T, EN, device=dev)
        self.rewards = torch.zeros(T, EN, device=dev)
        self.masks = torch.ones(T + 1, EN, device=dev)
        self.active_masks = torch.ones(T + 1, EN, device=dev)

    def load_reference(self, data):
        """Fill from reference-shaped numpy arrays ([T(+1), E, N, ...], see make_golden_mappo.py)."""
        def put(dst, src, dtype=torch.float32):
            dst.copy_(torch.as_tensor(np.ascontiguousarray(src)).reshape(dst.shape).to(dtype))
        put(self.obs, data["obs"])
        put(self.rnn_states, data["rnn_states"])
        put(self.rnn_states_critic, data["rnn_states_critic"])
        put(self.value_preds, data["value_preds"])
        put(self.returns, data["returns"])
        put(self.actions, data["actions"], torch.int32)
        put(self.action_log_probs, data["action_log_probs"])
        put(self.rewards, data["rewards"])
        put(self.masks, data["masks"])
        put(self.active_masks, data["active_masks"])

    def after_update(self):
        """shared_buffer.py:119-129: last slot becomes the first."""
        for t in (self.obs, self.rnn_states, self.rnn_states_critic, self.masks, self.active_masks):
            t[0].copy_(t[-1])

    def compute_returns(self, vn, gamma=0.99, gae_lambda=0.95):
        """shared_buffer.py:131-153 with ValueNorm (value_preds[T] must hold the next value)."""
        check(lib().mm_mappo_gae(ptr(self.rewards), ptr(self.value_preds), ptr(self.masks), ptr(self.returns),
                                 ptr(vn), self.T, self.EN, float(gamma), float(gae_lambda),
                                 stream_handle(self.device)), "mappo_gae")


class MappoTrainer:
    """R_MAPPO (ramppo_network.py:9-287) with train_batch_size 1, recurrent chunks of L steps."""

    def __init__(self, policy, T, EN, L=5, ppo_epoch=15, clip_param=0.2, huber_delta=10.0, entropy_coef=0.01,
                 value_loss_coef=0.5, max_grad_norm=0.5, actor_lr=1e-4, critic_lr=1e-4, opti_eps=1e-5,
                 grad_allreduce=None, fused=True):
        """fused: one mm_mappo_grad pass per epoch (forward recomputed in the backward, weight gradients
        reduced on MFMA in the same kernel); False: the TRAIN forward with saved activations, the BPTT
        kernel writing per-row operands and the separate weight-gradient reduction."""
        assert T % L == 0, "episode length must be a multiple of data_chunk_length"
        self.fused = bool(fused)
        self.p = policy
        self.T, self.EN, self.L, self.epochs = int(T), int(EN), int(L), int(ppo_epoch)
        self.clip, self.huber, self.ent, self.vcoef = clip_param, huber_delta, entropy_coef, value_loss_coef
        self.max_norm, self.lrs, self.eps = max_grad_norm, (actor_lr, critic_lr), opti_eps
        self.allreduce = grad_allreduce
        dev = self.device = policy.device
        L_ = lib()
        d = ctypes.byref(policy.dims)
        self.rows = self.T * self.EN
        self.rs = _rs(self.rows)
        if self.fused:
            n_scr = int(L_.mm_mappo_grad_scratch_count(d, self.L, self.T, self.EN))
            if n_scr <= 0:
                raise RuntimeError("mappo_grad: unsupported dims for the fused gradient pass")
            self.gscr = torch.zeros(n_scr, device=dev)
        else:
            ns = [L_.mm_mappo_save_fields(d, n) for n in (0, 1)]
            ng = [L_.mm_mappo_grad_fields(d, n) for n in (0, 1)]
            self.save = [torch.zeros(self.rs * ns[n], device=dev) for n in (0, 1)]
            self.gsoa = [torch.zeros(self.rs * ng[n], device=dev) for n in (0, 1)]
            self.partial = torch.zeros(int(L_.mm_mappo_wgrad_partial_count(d, self.rs)), device=dev)
        nets = (policy.actor, policy.critic)
        self.grad = [torch.zeros_like(n.flat) for n in nets]
        self.m = [torch.zeros_like(n.flat) for n in nets]
        self.v = [torch.zeros_like(n.flat) for n in nets]
        self.step = [torch.zeros(1, device=dev) for _ in nets]
        self.norm_part = [torch.zeros(256, device=dev) for _ in nets]
        self.norms = torch.zeros(2, max(1, self.epochs), device=dev)
        self.vn = torch.zeros(3, device=dev)          # ValueNorm running mean, mean sq, debias (f32)
        self.stats = torch.zeros(8, device=dev)
        self.adv = torch.zeros(self.rows, device=dev)
        self.adv_part = torch.zeros(7 * 256 + 5, dtype=torch.float64, device=dev)
        self.loss_acc = torch.zeros(4, device=dev)

    # -- checkpoint (minimarl.checkpoint) ------------------------------------------------------
    def checkpoint_tensors(self):
        ts = {"actor": self.p.actor.flat, "critic": self.p.critic.flat, "vn": self.vn}
        for n in (0, 1):
            ts[f"m{n}"], ts[f"v{n}"], ts[f"step{n}"] = self.m[n], self.v[n], self.step[n]
        return ts, {}

    def restore_tensors(self, ts, scalars):
        from .checkpoint import copy_into
        copy_into(self.p.actor.flat, ts["actor"], "actor")
        copy_into(self.p.critic.flat, ts["critic"], "critic")
        copy_into(self.vn, ts["vn"], "vn")
        for n in (0, 1):
            copy_into(self.m[n], ts[f"m{n}"], f"m{n}")
            copy_into(self.v[n], ts[f"v{n}"], f"v{n}")
            copy_into(self.step[n], ts[f"step{n}"], f"step{n}")

    # -- ValueNorm (utils/valuenorm.py) ------------------------------------------------------
    def value_normalizer_state(self):
        v = self.vn.detach().cpu().numpy()
        return {"running_mean": v[0:1], "running_mean_sq": v[1:2], "debiasing_term": np.float32(v[2])}

    def load_value_normalizer(self, mean, mean_sq, debias):
        self.vn.copy_(torch.tensor([mean, mean_sq, debias], dtype=torch.float32))

    def denormalize(self, x):
        v = self.vn.detach().cpu().double()
        d = max(float(v[2]), 1e-5)
        mean, msq = float(np.float32(v[0] / d)), float(np.float32(v[1] / d))
        var = max(msq - mean * mean, 1e-2)
        return x * float(np.sqrt(var)) + mean

    # -- one train() ------------------------------------------------------------------------
    def fwd_args(self, buf):
        if self.fused:
            return None
        a = MappoFwdArgs()
        a.net[0].P, a.net[0].h_in, a.net[0].save = _ptrs(self.p.actor.flat, buf.rnn_states, self.save[0])
        a.net[1].P, a.net[1].h_in, a.net[1].save = _ptrs(self.p.critic.flat, buf.rnn_states_critic, self.save[1])
        a.obs, a.mask = _ptrs(buf.obs, buf.masks)
        a.en, a.T, a.L, a.rs, a.mode = self.EN, self.T, self.L, self.rs, MM_MAPPO_TRAIN
        return a

    def bwd_args(self, buf):
        b = MappoBwdArgs()
        b.P[0], b.P[1] = ptr(self.p.actor.flat), ptr(self.p.critic.flat)
        if not self.fused:
            b.save[0], b.save[1] = ptr(self.save[0]), ptr(self.save[1])
            b.gsoa[0], b.gsoa[1] = ptr(self.gsoa[0]), ptr(self.gsoa[1])
        (b.obs, b.mask, b.active, b.act, b.adv, b.old_logp, b.old_value, b.returns, b.stats,
         b.loss_acc) = _ptrs(buf.obs, buf.masks, buf.active_masks, buf.actions, self.adv, buf.action_log_probs,
                             buf.value_preds, buf.returns, self.stats, self.loss_acc)
        b.clip, b.huber_delta, b.entropy_coef, b.value_coef = self.clip, self.huber, self.ent, self.vcoef
        b.en, b.T, b.L, b.rs = self.EN, self.T, self.L, self.rs
        return b

    def prepare(self, buf):
        """Advantages (returns - denorm(V)), their masked mean/std and the return moments. Data
        parallel: the raw sums are all-reduced so every replica normalises with the global
        statistics and applies the same ValueNorm updates."""
        s = stream_handle(self.device)
        check(lib().mm_mappo_adv_stats(ptr(buf.returns), ptr(buf.value_preds), ptr(buf.active_masks), ptr(self.vn),
                                       ptr(self.adv), self.rows, ptr(self.adv_part), ptr(self.stats), s),
              "mappo_adv_stats")
        if self.allreduce is not None:
            sums = self.adv_part[7 * 256:7 * 256 + 5]
            world = self.allreduce(sums)
            check(lib().mm_mappo_stats_from_sums(ptr(sums), self.rows * world, ptr(self.stats), s),
                  "mappo_stats_from_sums")
        self.loss_acc.zero_()

    def gradients(self, buf, fa=None, ba=None):
        """This epoch's unclipped gradients of both nets into self.grad (loss seeds + chunked BPTT +
        weight-gradient reduction, ramppo_network.py:56-209)."""
        L_, s, d = lib(), stream_handle(self.device), ctypes.byref(self.p.dims)
        ba = ba or self.bwd_args(buf)
        if self.fused:
            check(L_.mm_mappo_grad(d, ctypes.byref(ba), ptr(buf.rnn_states), ptr(buf.rnn_states_critic),
                                   ptr(self.grad[0]), ptr(self.grad[1]), ptr(self.gscr), s), "mappo_grad")
            return
        fa = fa or self.fwd_args(buf)
        check(L_.mm_mappo_fwd(d, ctypes.byref(fa), s), "mappo_fwd(train)")
        check(L_.mm_mappo_bwd(d, ctypes.byref(ba), s), "mappo_bwd")
        for n in (0, 1):
            check(L_.mm_mappo_wgrad(d, n, ptr(self.gsoa[n]), self.rs, ptr(self.grad[n]), ptr(self.partial), s),
                  "mappo_wgrad")

    def epoch(self, buf, ep, fa=None, ba=None):
        L_, s, d = lib(), stream_handle(self.device), ctypes.byref(self.p.dims)
        check(L_.mm_mappo_vn_update(ptr(self.vn), ptr(self.stats), 0.99999, s), "mappo_vn_update")
        self.gradients(buf, fa, ba)
        # data parallel: the loss seeds already divide by the GLOBAL active count (stats from the
        # all-reduced sums in prepare()), so the SUM over replicas is the global-batch gradient: no
        # further 1/world
        scale = 1.0
        if self.allreduce is not None:
            for n in (0, 1):
                self.allreduce(self.grad[n])
        nets = (self.p.actor, self.p.critic)
        for n in (0, 1):
            check(L_.mm_clip_adam(ptr(nets[n].flat), ptr(self.grad[n]), ptr(self.m[n]), ptr(self.v[n]),
                                  nets[n].total, nets[n].total, self.max_norm, self.lrs[n], 0.9, 0.999, self.eps,
                                  ptr(self.step[n]), ptr(self.norm_part[n]), ptr(self.norms[n, ep % self.norms.shape[1]]),
                                  scale, s), "clip_adam")

    def train(self, buf):
        self.prepare(buf)
        fa, ba = self.fwd_args(buf), self.bwd_args(buf)
        for ep in range(self.epochs):
            self.epoch(buf, ep, fa, ba)
        return self.train_info()

    def train_info(self):
        la = self.loss_acc.detach().cpu().numpy().astype(np.float64)
        nrm = self.norms.detach().cpu().numpy().astype(np.float64)
        e = max(1, self.epochs)
        return {"value_loss": la[MM_MLOSS_VALUE] / e, "policy_loss": la[MM_MLOSS_POLICY] / e,
                "dist_entropy": la[MM_MLOSS_ENTROPY] / e, "actor_grad_norm": nrm[0].mean(),
                "critic_grad_norm": nrm[1].mean(), "ratio": la[MM_MLOSS_RATIO] / (e * self.rows)}


class MappoRunner:
    """MAGYM_Runner (magym_runner.py:30-195) on lockstep device envs: collect -> insert -> compute -> train."""

    def __init__(self, env, policy, T=100, L=5, ppo_epoch=15, gamma=0.99, gae_lambda=0.95, seed=0,
                 grad_allreduce=None):
        self.env, self.p = env, policy
        self.E, self.N, self.D = env.E, env.N, env.obs_dim
        self.T, self.gamma, self.gl = int(T), gamma, gae_lambda
        dev = self.device = policy.device
        self.buf = MappoBuffer(T, self.E, self.N, self.D, policy.H, dev)
        self.trainer = MappoTrainer(policy, T, self.E * self.N, L, ppo_epoch, grad_allreduce=grad_allreduce)
        self.seed = int(seed)
        self.counter = torch.zeros(1, dtype=torch.int64, device=dev)
        self.done = torch.zeros(self.E, dtype=torch.uint8, device=dev)
        self.args = []
        b = self.buf
        for t in range(self.T):
            a = policy.rollout_args(b.obs[t], b.rnn_states[t], b.rnn_states_critic[t], b.masks[t],
                                    b.rnn_states[t + 1], b.rnn_states_critic[t + 1], b.action_log_probs[t],
                                    b.value_preds[t], act_out=b.actions[t], seed=self.seed,
                                    counter_ptr=ptr(self.counter))
            self.args.append(a)

    def warmup(self):
        self.env.reset(out=self.buf.obs[0].view(self.E, self.N, self.D))

    def collect_step(self, t):
        L_, s, b = lib(), stream_handle(self.device), self.buf
        check(L_.mm_mappo_fwd(ctypes.byref(self.p.dims), ctypes.byref(self.args[t]), s), "mappo_fwd")
        # no terminal obs needed (MAPPO bootstraps through masks): only the auto-reset current obs
        check(L_.mm_env_step(self.env.handle(), ptr(b.actions[t]), None, ptr(b.obs[t + 1]),
                             ptr(b.rewards[t]), ptr(self.done), s), "env_step")
        check(L_.mm_mappo_insert(ptr(self.done), self.N, self.p.H, self.E, ptr(b.masks[t + 1]),
                                 ptr(b.active_masks[t + 1]), ptr(b.rnn_states[t + 1]), ptr(b.rnn_states_critic[t + 1]),
                                 ptr(self.counter), s), "mappo_insert")

    def rollout(self):
        for t in range(self.T):
            self.collect_step(t)

    def compute(self):
        b = self.buf
        a = MappoFwdArgs()
        a.net[1].P, a.net[1].h_in, a.net[1].out = _ptrs(self.p.critic.flat, b.rnn_states_critic[self.T],
                                                        b.value_preds[self.T])
        a.obs, a.mask = _ptrs(b.obs[self.T], b.masks[self.T])
        a.rows, a.mode = b.EN, MM_MAPPO_VALUES
        self.p._fwd(a)
        b.compute_returns(self.trainer.vn, self.gamma, self.gl)

    def train(self):
        info = self.trainer.train(self.buf)
        self.buf.after_update()
        return info

    def run_episode(self):
        self.rollout()
        self.compute()
        return self.train()
