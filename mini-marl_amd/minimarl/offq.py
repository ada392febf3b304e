"""Episode-level recurrent QMix / VDN (the reference's ``offpolicy/`` fork) on the MI355X.

Mirrors ``QMix`` (offpolicy/algorithms/qmix/qmix.py:13-242: train_policy_on_batch,
hard_target_updates, soft_target_updates) together with its shared ``QMixPolicy``
(algorithm/QMixPolicy.py:10-226: get_q_values, actions_from_q, init_hidden) over the C ABI in
include/minimarl.h (csrc/offq.hip). Everything runs on the GPU; there is no CPU path.

Parameters live in one flat device vector per net set, [agent | mixer]: the agent net in the trunk
layout shared with MAPPO (MGeo: W1 rows padded to ceil4(D), the Q head to ceil4(A) rows) and the
QMixer's 14 tensors in named_parameters() order. Gradients, Adam moments and the target copy use
the same layout, so clip_grad_norm_ over ``self.parameters`` (agent + mixer, qmix.py:69-74,202)
and Adam(eps = opti_eps) are one mm_clip_adam call.
"""
import ctypes

import numpy as np
import torch

from ._lib import MM_OFFQ_QMIX, MM_OFFQ_VDN, OffqBatch, OffqDims, c_i64, check, lib
from .qnet import ptr, stream_handle

AGENT_KEYS = ["ln0_w", "ln0_b", "W1", "b1", "ln1_w", "ln1_b", "W2", "b2", "ln2_w", "ln2_b",
              "Wih", "Whh", "bih", "bhh", "lnr_w", "lnr_b", "Wo", "bo"]
# AgentQFunction state_dict names (agent_q_function.py:10-21; RNNBase = MLPBase + RNNLayer)
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
MIXER_KEYS = ["hyper_w1.0.weight", "hyper_w1.0.bias", "hyper_w1.2.weight", "hyper_w1.2.bias",
              "hyper_w2.0.weight", "hyper_w2.0.bias", "hyper_w2.2.weight", "hyper_w2.2.bias",
              "hyper_b1.weight", "hyper_b1.bias",
              "hyper_b2.0.weight", "hyper_b2.0.bias", "hyper_b2.2.weight", "hyper_b2.2.bias"]


class OffQMix:
    """QMix / VDN trainer + shared recurrent Q policy (one policy, ``policy_0``)."""

    def __init__(self, n_agents, obs_dim, n_actions, episode_length, batch_size, mixer="qmix", hidden=64,
                 mixer_hidden=32, hyper_hidden=64, gamma=0.99, lr=5e-4, opti_eps=1e-5, max_grad_norm=10.0,
                 use_double_q=True, use_per=True, use_huber_loss=False, huber_delta=10.0, per_nu=0.9,
                 per_eps=1e-6, tau=0.005, device="cuda", seed=None, grad_allreduce=None):
        assert mixer in ("qmix", "vdn")
        self.N, self.D, self.A, self.H = int(n_agents), int(obs_dim), int(n_actions), int(hidden)
        self.T, self.B = int(episode_length), int(batch_size)
        self.mixer_kind = mixer
        self.S = self.N * self.D                  # share_obs = concat of the agents' obs (base_runner.py:337-340)
        self.K, self.Hh = int(mixer_hidden), int(hyper_hidden)
        self.gamma, self.lr, self.eps, self.max_norm = gamma, lr, opti_eps, max_grad_norm
        self.double_q, self.use_per, self.huber, self.delta = use_double_q, use_per, use_huber_loss, huber_delta
        self.per_nu, self.per_eps, self.tau = per_nu, per_eps, tau
        # data-parallel replicas (minimarl.dist.make_allreduce): the flat [agent | mixer] gradient is
        # summed over ranks (one RCCL all-reduce per update) and averaged inside clip/Adam; every rank
        # samples its own episode shard, so each rank's loss keeps its own mask-count denominator
        self.allreduce = grad_allreduce
        self.device = torch.device(device)
        self.dims = OffqDims(self.N, self.D, self.H, self.A, MM_OFFQ_QMIX if mixer == "qmix" else MM_OFFQ_VDN,
                             self.S, self.K, self.Hh)
        L = lib()
        na, nm = c_i64(), c_i64()
        check(L.mm_offq_param_counts(ctypes.byref(self.dims), ctypes.byref(na), ctypes.byref(nm)), "offq_param_counts")
        self.n_agent, self.n_mixer = int(na.value), int(nm.value)
        self.total = self.n_agent + self.n_mixer
        mo = (c_i64 * 15)()
        check(L.mm_offq_mixer_offsets(ctypes.byref(self.dims), mo), "offq_mixer_offsets")
        self.moffs = list(mo)
        self.Dp, self.Ap = (self.D + 3) // 4 * 4, (self.A + 3) // 4 * 4
        H, Dp, Ap = self.H, self.Dp, self.Ap
        sz = [Dp, Dp, H * Dp, H, H, H, H * H, H, H, H, 3 * H * H, 3 * H * H, 3 * H, 3 * H, H, H, Ap * H, Ap]
        self.aoffs = list(np.concatenate([[0], np.cumsum(sz)]).astype(np.int64))
        assert self.aoffs[-1] == self.n_agent, (self.aoffs[-1], self.n_agent)
        dev = self.device
        self.P = torch.zeros(self.total, device=dev)
        self.PT = torch.zeros(self.total, device=dev)
        self.grad = torch.zeros(self.total, device=dev)
        self.m = torch.zeros(self.total, device=dev)
        self.v = torch.zeros(self.total, device=dev)
        self.step = torch.zeros(1, device=dev)
        self.partials = torch.zeros(512, device=dev)
        self.norm = torch.zeros(1, device=dev)
        self.stats = torch.zeros(2, device=dev)
        self.prio = torch.zeros(self.B, device=dev)
        nbytes = int(L.mm_offq_workspace_bytes(ctypes.byref(self.dims), self.T, self.B))
        check(0 if nbytes > 0 else -22, "offq_workspace_bytes")
        self.ws = torch.zeros((nbytes + 3) // 4, device=dev)
        self.ws_bytes = nbytes
        self._qws = {}
        if seed is not None:
            self.init_default(seed)
            self.hard_target_updates()

    # -- parameter views ---------------------------------------------------------------------
    def agent_shape(self, key):
        D, H, A = self.D, self.H, self.A
        return {"ln0_w": (D,), "ln0_b": (D,), "W1": (H, D), "b1": (H,), "ln1_w": (H,), "ln1_b": (H,),
                "W2": (H, H), "b2": (H,), "ln2_w": (H,), "ln2_b": (H,), "Wih": (3 * H, H), "Whh": (3 * H, H),
                "bih": (3 * H,), "bhh": (3 * H,), "lnr_w": (H,), "lnr_b": (H,), "Wo": (A, H), "bo": (A,)}[key]

    def agent_view(self, key, t=None):
        t = self.P if t is None else t
        o = self.aoffs[AGENT_KEYS.index(key)]
        if key == "W1":
            return t[o:o + self.H * self.Dp].view(self.H, self.Dp)[:, :self.D]
        if key == "Wo":
            return t[o:o + self.Ap * self.H].view(self.Ap, self.H)[:self.A]
        n = int(np.prod(self.agent_shape(key)))
        return t[o:o + n].view(self.agent_shape(key))

    def mixer_shape(self, key):
        S, K, Hh, NK = self.S, self.K, self.Hh, self.N * self.K
        return {"hyper_w1.0.weight": (Hh, S), "hyper_w1.0.bias": (Hh,), "hyper_w1.2.weight": (NK, Hh),
                "hyper_w1.2.bias": (NK,), "hyper_w2.0.weight": (Hh, S), "hyper_w2.0.bias": (Hh,),
                "hyper_w2.2.weight": (K, Hh), "hyper_w2.2.bias": (K,), "hyper_b1.weight": (K, S),
                "hyper_b1.bias": (K,), "hyper_b2.0.weight": (Hh, S), "hyper_b2.0.bias": (Hh,),
                "hyper_b2.2.weight": (1, Hh), "hyper_b2.2.bias": (1,)}[key]

    def mixer_view(self, key, t=None):
        t = self.P if t is None else t
        i = MIXER_KEYS.index(key)
        o = self.n_agent + self.moffs[i]
        n = self.moffs[i + 1] - self.moffs[i]
        return t[o:o + n].view(self.mixer_shape(key))

    def init_default(self, seed):
        """The reference init: orthogonal weights (gain sqrt(2) for the ReLU MLP, 1 for the GRU and
        the hypernets, ``gain`` = 0.01 for the Q head), zero biases, unit LayerNorms."""
        g = torch.Generator().manual_seed(int(seed))
        self.P.zero_()
        for key in AGENT_KEYS:
            shp = self.agent_shape(key)
            if key.startswith("ln") and key.endswith("_w"):
                self.agent_view(key).fill_(1.0)
            elif len(shp) == 2:
                w = torch.empty(shp)
                gain = float(np.sqrt(2.0)) if key in ("W1", "W2") else (0.01 if key == "Wo" else 1.0)
                torch.nn.init.orthogonal_(w, gain=gain, generator=g)
                self.agent_view(key).copy_(w.to(self.device))
        if self.mixer_kind == "qmix":
            for key in MIXER_KEYS:
                if key.endswith("weight"):
                    w = torch.empty(self.mixer_shape(key))
                    torch.nn.init.orthogonal_(w, gain=1.0, generator=g)
                    self.mixer_view(key).copy_(w.to(self.device))

    def load_reference_state(self, q_sd, m_sd=None, target_q_sd=None, target_m_sd=None):
        """q_sd: AgentQFunction.state_dict(); m_sd: QMixer.state_dict(); targets default to copies."""
        for t, qs, ms in ((self.P, q_sd, m_sd), (self.PT, target_q_sd or q_sd, target_m_sd or m_sd)):
            for k in AGENT_KEYS:
                self.agent_view(k, t).copy_(torch.as_tensor(np.asarray(qs[AGENT_REF[k]]), dtype=torch.float32))
            if self.mixer_kind == "qmix":
                for k in MIXER_KEYS:
                    self.mixer_view(k, t).copy_(torch.as_tensor(np.asarray(ms[k]), dtype=torch.float32))

    def state_dict(self, target=False):
        t = self.PT if target else self.P
        q = {AGENT_REF[k]: self.agent_view(k, t).detach().cpu().clone() for k in AGENT_KEYS}
        m = ({k: self.mixer_view(k, t).detach().cpu().clone() for k in MIXER_KEYS}
             if self.mixer_kind == "qmix" else {})
        return q, m

    # -- training ----------------------------------------------------------------------------
    def _dev(self, x):
        t = x if torch.is_tensor(x) else torch.as_tensor(np.asarray(x))
        return t.to(device=self.device, dtype=torch.float32).contiguous()

    def train_policy_on_batch(self, batch, update_policy_id=None):
        """QMix.train_policy_on_batch (qmix.py:80-210). batch = the PrioritizedRecReplayBuffer.sample
        tuple (obs, share_obs, acts, rewards, dones, dones_env, avail_acts, importance_weights, idxes),
        each of the first six a {policy_id: array} dict (numpy or device tensors). Returns
        (train_info {loss, grad_norm, Q_tot} as device scalars, new priorities [B] device tensor or
        None, idxes)."""
        obs, share, acts, rew, _dones, dones_env, _avail, isw, idxes = batch
        pid = "policy_0" if isinstance(obs, dict) else None
        pick = (lambda d: d[pid]) if pid else (lambda d: d)
        o = self._dev(pick(obs))
        assert tuple(o.shape) == (self.N, self.T + 1, self.B, self.D), o.shape
        a = self._dev(pick(acts))
        r = self._dev(pick(rew))
        de = self._dev(pick(dones_env))
        s = self._dev(pick(share)) if self.mixer_kind == "qmix" else None
        w = self._dev(isw) if (self.use_per and isw is not None) else None
        self._keep = (o, a, r, de, s, w)                # alive until the kernels ran
        bt = OffqBatch()
        bt.obs, bt.share_obs, bt.acts, bt.rewards, bt.dones_env = ptr(o), ptr(s), ptr(a), ptr(r), ptr(de)
        bt.is_weight = ptr(w)
        bt.T, bt.B, bt.double_q, bt.huber = self.T, self.B, int(self.double_q), int(self.huber)
        bt.gamma, bt.huber_delta, bt.per_nu, bt.per_eps = self.gamma, self.delta, self.per_nu, self.per_eps
        L, st = lib(), stream_handle(self.device)
        check(L.mm_offq_loss_grad(ctypes.byref(self.dims), ctypes.byref(bt), ptr(self.P), ptr(self.PT), ptr(self.grad),
                                  ptr(self.ws), self.ws_bytes, ptr(self.stats), ptr(self.prio), st), "offq_loss_grad")
        scale = 1.0
        if self.allreduce is not None:
            scale = 1.0 / self.allreduce(self.grad)
        check(L.mm_clip_adam(ptr(self.P), ptr(self.grad), ptr(self.m), ptr(self.v), self.total, self.total,
                             self.max_norm, self.lr, 0.9, 0.999, self.eps, ptr(self.step), ptr(self.partials),
                             ptr(self.norm), scale, st), "clip_adam")
        info = {"loss": self.stats[0], "grad_norm": self.norm[0], "Q_tot": self.stats[1]}
        return info, (self.prio if w is not None else None), idxes

    def hard_target_updates(self):
        """qmix.py:213-219: target agent net and target mixer <- behavior."""
        self.PT.copy_(self.P)

    def soft_target_updates(self):
        """qmix.py:221-226 / utils/util.py:123-134 (tau)."""
        check(lib().mm_offq_soft_update(ptr(self.PT), ptr(self.P), self.total, float(self.tau),
                                        stream_handle(self.device)), "offq_soft_update")

    # -- checkpoint (minimarl.checkpoint) ------------------------------------------------------
    def checkpoint_tensors(self):
        return ({"P": self.P, "PT": self.PT, "m": self.m, "v": self.v, "step": self.step},
                {"mixer": self.mixer_kind})

    def restore_tensors(self, ts, scalars):
        from .checkpoint import copy_into
        for k in ("P", "PT", "m", "v", "step"):
            copy_into(getattr(self, k), ts[k], k)

    # -- acting ------------------------------------------------------------------------------
    def init_hidden(self, num_agents, batch_size):
        """QMixPolicy.init_hidden (QMixPolicy.py:213-218)."""
        if num_agents == -1:
            return torch.zeros(batch_size, self.H, device=self.device)
        return torch.zeros(num_agents, batch_size, self.H, device=self.device)

    def get_q_values(self, obs, rnn_states=None, target=False):
        """QMixPolicy.get_q_values (prev_act_inp off): obs [R, D] or [L, R, D], hidden [R, H] ->
        (q [R, A] or [L, R, A], new hidden [R, H])."""
        x = self._dev(obs)
        seq = x.dim() == 3
        if not seq:
            x = x.unsqueeze(0)
        Ls, R = int(x.shape[0]), int(x.shape[1])
        key = (Ls, R)
        if key not in self._qws:
            nb = int(lib().mm_offq_qvals_workspace_bytes(ctypes.byref(self.dims), Ls, R))
            check(0 if nb > 0 else -22, "offq_qvals_workspace_bytes")
            self._qws[key] = (torch.empty((nb + 3) // 4, device=self.device), nb)
        ws, nb = self._qws[key]
        q = torch.empty(Ls, R, self.A, device=self.device)
        h2 = torch.empty(R, self.H, device=self.device)
        h0 = None if rnn_states is None else self._dev(rnn_states).reshape(R, self.H)
        check(lib().mm_offq_q_values(ctypes.byref(self.dims), ptr(self.PT if target else self.P), ptr(x), ptr(h0),
                                     ptr(q), ptr(h2), Ls, R, ptr(ws), nb, stream_handle(self.device)),
              "offq_q_values")
        return (q if seq else q[0]), h2

    def get_actions(self, obs, rnn_states=None):
        """Greedy get_actions (explore=False, QMixPolicy.py:117-195): one-hot actions [R, A], new
        hidden, greedy Q [R, 1]."""
        q, h2 = self.get_q_values(obs, rnn_states)
        gq, ga = q.max(-1)
        return torch.nn.functional.one_hot(ga, self.A).float(), h2, gq.unsqueeze(-1)
