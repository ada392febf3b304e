"""Reference-signature adapters: drop-ins for the reference's duck-typed classes,
backed by the device kernels, so a reference-shaped harness (its runners, its tests) can drive the
engine unchanged.

  Q_Net                        qmix/_network.py:5-77, vdn/_network.py:61-91   (minimarl.qnet.Q_Net)
  Mix_Net                      qmix/_network.py:172-220
  Train_dqn                    qmix/_train.py:7-121        .train(Replay_buffer, bq, bm, tq, tm, optimizer, eps)
  Target_Dqn                   vdn/_train.py:8-101         .train(target_network, optimizer, eps) -> loss
  Target_Double_Dqn            vdn/_train.py:104-158
  Prioritized_Experience_Replay vdn/replay_buffer/buffer.py:10-90, qmix/replay_buffer/per.py:10-81
  R_MAPPOPolicy                mappo/algorithms/rmappo_policy.py:7-153

Deliberate differences: tensors stay on the GPU; the optimizer argument supplies only
its hyper-parameters (lr, betas, eps of param_groups[0]) — the Adam moments live in the device
learner bound to the nets on the first call; ``R_MAPPOPolicy.get_actions`` samples with the device
counter RNG (the reference's torch.multinomial stream cannot be reproduced on the device) and, like
the reference (rmappo_policy.py:86), ignores ``deterministic``; PER sampling consumes Python's
``random`` exactly like the reference (one ``random.random()`` per stratum, ``random.uniform`` =
a + (b - a) * random()), so equal seeds give equal strata.
"""
import ctypes
import random

import numpy as np
import torch

from ._lib import MixNetIO, check, lib
from .learner import Mixer, QLearner
from .qnet import Q_Net, ptr, stream_handle  # noqa: F401  (re-exported: the agent-net adapter)
from .replay import DevicePER


def _dev(x, device, dtype=torch.float32):
    return torch.as_tensor(x, dtype=dtype).to(device)


def _hyper(optimizer):
    """(lr, betas, eps) of a torch optimizer's first param group (defaults: the reference's Adam)."""
    g = getattr(optimizer, "param_groups", None)
    if g:
        return float(g[0].get("lr", 1e-3)), tuple(g[0].get("betas", (0.9, 0.999))), float(g[0].get("eps", 1e-8))
    return 1e-3, (0.9, 0.999), 1e-8


class Mix_Net:
    """qmix/_network.py:172-220: GRUCell(state, hx) + abs-monotone hypernetworks, one fused launch."""

    def __init__(self, observation_space, args=None, hidden_dim=32, hx_size=32, device="cuda", seed=None):
        if args is not None and not getattr(args, "use_recurrent", True):
            raise NotImplementedError("Mix_Net without the GRU (use_recurrent=False) is not on the hot path")
        self.n_agents = len(observation_space)
        self.state_size = sum(int(sp.shape[0]) for sp in observation_space)
        self.hidden_dim, self.hx_size = int(hidden_dim), int(hx_size)
        self.device = torch.device(device)
        self.mixer = Mixer(self.n_agents, self.state_size, self.hx_size, self.hidden_dim, self.device, seed=seed)

    def load_state_dict(self, state_dict):
        if isinstance(state_dict, Mix_Net):
            self.mixer.flat.copy_(state_dict.mixer.flat)
            return
        self.mixer.load_reference_state({k: v.cpu().numpy() if torch.is_tensor(v) else v
                                         for k, v in state_dict.items()})

    def state_dict(self):
        return self.mixer.state_dict()

    def parameters(self):
        return [self.mixer.flat]

    def __call__(self, q_values, observations, hidden):
        return self.forward(q_values, observations, hidden)

    @torch.no_grad()
    def forward(self, q_values, observations, hidden):
        """q [B,N], obs [B,N,D], hidden [B,hx] -> (Q_tot [B,1], next hidden [B,hx])."""
        obs = _dev(observations, self.device).contiguous()
        B, N, D = obs.shape
        assert N == self.n_agents and N * D == self.state_size, f"obs {tuple(obs.shape)} vs state {self.state_size}"
        q = _dev(q_values, self.device).reshape(B, N).contiguous()
        h = _dev(hidden, self.device).reshape(B, self.hx_size).contiguous()
        h2 = torch.empty(B, self.hx_size, device=self.device)
        qtot = torch.empty(B, device=self.device)
        s_off = torch.arange(B, dtype=torch.int64, device=self.device) * (N * D)
        nets = (MixNetIO * 1)()
        n = nets[0]
        n.P, n.q, n.s_off, n.h_in, n.h_out, n.qtot = (t.data_ptr() for t in (self.mixer.flat, q, s_off, h, h2, qtot))
        check(lib().mm_mixer_fwd(B, N, self.state_size, self.hx_size, self.hidden_dim, ptr(obs), ptr(obs), nets, 1,
                                 stream_handle(self.device)), "mixer_fwd")
        return qtot.view(B, 1), h2

    def init_hidden(self, batch_size=1):
        return torch.zeros((batch_size, self.hx_size), device=self.device)


class Prioritized_Experience_Replay:
    """Chunk-level prioritized replay with the sum tree and the chunk payloads in HBM."""

    def __init__(self, args, flavor="vdn", device="cuda"):
        self.device = torch.device(device)
        self.capacity = int(args.buffer_limit)
        # qmix/replay_buffer/per.py has no step decay: use_step_weight defaults to flavor == "vdn"
        self.per = DevicePER.from_args(args, flavor, device=self.device)
        self._store = None

    @property
    def alpha(self):
        return self.per.alpha

    @property
    def beta(self):
        return self.per.beta

    def __len__(self):
        return len(self.per)

    def _alloc(self, C, N, D):
        cap, dev = self.capacity, self.device
        self._store = {"s": torch.zeros(cap, C, N, D, device=dev), "a": torch.zeros(cap, C, N, device=dev),
                       "r": torch.zeros(cap, C, N, device=dev), "s2": torch.zeros(cap, C, N, D, device=dev),
                       "d": torch.zeros(cap, C, device=dev)}

    def collect_sample(self, sample, td_error, warm_up):
        """buffer.py:37-40: sample = [states (C x N x D), actions (C x 1 x N), rewards (C x N),
        next states, dones (C)]; priority (td + eps)^alpha; returns the fill count during warm-up."""
        s, a, r, s2, d = sample
        s = _dev(np.asarray(s, np.float32), self.device)
        C, N, D = s.shape
        if self._store is None:
            self._alloc(C, N, D)
        slot = self.per.add(torch.tensor([float(td_error)], dtype=torch.float32))
        st = self._store
        st["s"].index_copy_(0, slot, s.unsqueeze(0))
        st["a"].index_copy_(0, slot, _dev(np.asarray(a, np.float32), self.device).reshape(1, C, N))
        st["r"].index_copy_(0, slot, _dev(np.asarray(r, np.float32), self.device).reshape(1, C, N))
        st["s2"].index_copy_(0, slot, _dev(np.asarray(s2, np.float32), self.device).reshape(1, C, N, D))
        st["d"].index_copy_(0, slot, _dev(np.asarray(d, np.float32), self.device).reshape(1, C))
        return len(self.per) if warm_up else None

    def sample(self, batch_size, _chunk_size):
        """buffer.py:42-86 -> (states [B,C,N,D], actions [B,C,N], rewards [B,C,N], next_states, dones [B,C,1],
        priority_idx (tree nodes, device int64 [B]), is_weight [B,1])."""
        B = int(batch_size)
        fracs = [random.random() for _ in range(B)]       # random.uniform(left, right) draws, in order
        nodes, slots, w = self.per.sample(B, fracs=fracs)
        st = self._store
        C = st["d"].shape[1]
        return (st["s"][slots], st["a"][slots], st["r"][slots], st["s2"][slots], st["d"][slots].view(B, C, 1),
                nodes, w.view(B, 1))

    def update(self, priority_idx, new_td_error):
        """buffer.py:88-90 (one index) or a whole batch at once (last duplicate wins, like the loop)."""
        nodes = torch.as_tensor(priority_idx, dtype=torch.int64).to(self.device).reshape(-1)
        td = torch.as_tensor(new_td_error, dtype=torch.float32).to(self.device).reshape(-1)
        self.per.update(nodes, td)

    update_batch = update


def _update_priorities(Replay_buffer, priority_idx, new_td):
    if hasattr(Replay_buffer, "update_batch"):
        Replay_buffer.update_batch(priority_idx, new_td)
        return
    for index in range(len(priority_idx)):               # the reference's per-index loop
        Replay_buffer.update(priority_idx[index], new_td[index])


class _LearnerAdapter:
    mode = None

    def __init__(self, args, device="cuda"):
        self.device = torch.device(device)
        self.batch_size = int(args.batch_size)
        self.update_iter = int(args.update_iter)
        self.chunk_size = int(args.chunk_size) if getattr(args, "use_recurrent", True) else 1
        self.gamma = float(args.gamma)
        self.grad_clip_norm = float(args.grad_clip_norm)
        self._learner, self._key = None, None

    def _bind(self, beh, tgt, mix, tmix, optimizer):
        """The QLearner for these nets and this optimizer. A change of any net, of the optimizer object or of its
        lr / betas / eps rebuilds it: the old learner releases its nets first. The Adam moments carry over only
        when the SAME optimizer object trains the same nets with changed hyper-parameters (the reference's
        torch optimizer keeps its state across calls; a new optimizer object starts empty)."""
        lr, betas, eps = _hyper(optimizer)
        key = tuple(id(x) for x in (beh, tgt, mix, tmix, optimizer)) + (lr, tuple(betas), eps)
        if self._learner is None or key != self._key:
            adam = None
            if self._learner is not None:
                state = self._learner.release()
                if self._key[0] == key[0] and self._key[2] == key[2] and self._key[4] == key[4]:
                    adam = state
            self._learner = QLearner(beh.net, tgt.net, mix.mixer if mix is not None else None,
                                     tmix.mixer if tmix is not None else None, batch=self.batch_size,
                                     chunk=self.chunk_size, gamma=self.gamma, lr=lr, grad_clip=self.grad_clip_norm,
                                     betas=betas, adam_eps=eps, mode=self.mode, device=self.device)
            if adam is not None:
                self._learner.adopt_adam(adam)
            self._key = key
        return self._learner

    def _iterate(self, Replay_buffer, L):
        loss = torch.zeros(1, device=self.device)
        for _ in range(self.update_iter):
            states, actions, rewards, next_states, dones, priority_idx, w = Replay_buffer.sample(self.batch_size,
                                                                                                self.chunk_size)
            L.load_batch(states, actions, rewards, next_states, dones, w)
            L.train_step(L._obs_buf, L._obs_buf)
            loss += L.loss
            _update_priorities(Replay_buffer, priority_idx, L.td_last.clone().view(-1, 1))
        return loss


class Train_dqn(_LearnerAdapter):
    """qmix/_train.py:7-121 (works for any batch size; the reference needs B == 32, App. A 6)."""
    mode = "qmix"

    def train(self, Replay_buffer, behavior_q_net, behavior_mix_net, target_q_net, target_mix_net, optimizer,
              epsilon):
        L = self._bind(behavior_q_net, target_q_net, behavior_mix_net, target_mix_net, optimizer)
        self._iterate(Replay_buffer, L)
        return None


class Target_Dqn(_LearnerAdapter):
    """vdn/_train.py:56-101: returns the loss averaged over the update_iter updates (a device tensor)."""
    mode = "vdn"

    def __init__(self, Replay_buffer, behavior_network, target_network, args, device="cuda"):
        super().__init__(args, device)
        self.replay_buffer = Replay_buffer
        self.behavior_network = behavior_network
        self.target_network = target_network

    def train(self, target_network, optimizer, epsilon):
        L = self._bind(self.behavior_network, target_network, None, None, optimizer)
        if self.mode == "vdn_double":
            L.double_eps = float(epsilon)
        return (self._iterate(self.replay_buffer, L) / self.update_iter).view(())


class Target_Double_Dqn(Target_Dqn):
    """vdn/_train.py:104-158: the double net (behavior weights) picks s' actions epsilon-greedily
    (device counter RNG), the target net evaluates them."""
    mode = "vdn_double"


class R_MAPPOPolicy:
    """rmappo_policy.py:7-153 over the fused actor / critic kernels (shared policy, recurrent, Discrete)."""

    def __init__(self, args, obs_space, cent_obs_space, act_space, device="cuda", seed=None):
        from .mappo import MappoPolicy
        self.device = torch.device(device)
        D = int(obs_space.shape[0])
        if tuple(cent_obs_space.shape) != tuple(obs_space.shape):
            raise NotImplementedError("use_centralized_V=True (critic input != actor input) is not on the hot "
                                      "path (mappo/_config.py:146-150 default False)")
        self.hidden = int(getattr(args, "hidden_size", 32))
        self.actor_lr = float(getattr(args, "actor_lr", getattr(args, "lr", 1e-4)))
        self.critic_lr = float(getattr(args, "critic_lr", 1e-4))
        self.opti_eps = float(getattr(args, "opti_eps", 1e-5))
        self.policy = MappoPolicy(D, int(act_space.n), self.hidden, self.device, seed=seed)
        self.actor, self.critic = self.policy.actor, self.policy.critic
        self.seed = int(getattr(args, "seed", 1))
        self._counter = 0
        self._eval = {}

    def _t(self, x):
        return _dev(x, self.device).contiguous()

    def _same_input(self, obs, cent_obs):
        if cent_obs is obs:
            return
        co = self._t(cent_obs)
        if co.data_ptr() != obs.data_ptr() and not torch.equal(co, obs):
            raise NotImplementedError("cent_obs differs from obs: a centralized critic input is not supported")

    def get_actions(self, obs, cent_obs, rnn_states_actor, rnn_states_critic, masks, available_actions=None,
                    deterministic=False):
        obs_t = self._t(obs)
        self._same_input(obs_t, cent_obs)
        R = obs_t.shape[0]
        ha = self._t(rnn_states_actor).reshape(R, self.hidden)
        hc = self._t(rnn_states_critic).reshape(R, self.hidden)
        m = self._t(masks).reshape(R)
        v, a, lp, ha2, hc2 = self.policy.get_actions(obs_t, ha, hc, m, seed=self.seed, counter=self._counter)
        self._counter += 1
        return v, a.long(), lp, ha2.view(R, 1, self.hidden), hc2.view(R, 1, self.hidden)

    def get_values(self, cent_obs, rnn_states_critic, masks):
        co = self._t(cent_obs)
        R = co.shape[0]
        return self.policy.get_values(co, self._t(rnn_states_critic).reshape(R, self.hidden), self._t(masks).reshape(R))

    def act(self, obs, rnn_states_actor, masks, available_actions=None, deterministic=False):
        from ._lib import MM_MAPPO_ROLLOUT, MappoFwdArgs
        obs_t = self._t(obs)
        R = obs_t.shape[0]
        ha = self._t(rnn_states_actor).reshape(R, self.hidden)
        hc = torch.zeros_like(ha)
        ha2, hc2 = torch.empty_like(ha), torch.empty_like(ha)
        lp, v = torch.empty(R, device=self.device), torch.empty(R, device=self.device)
        act = torch.empty(R, dtype=torch.int32, device=self.device)
        a = self.policy.rollout_args(obs_t, ha, hc, self._t(masks).reshape(R), ha2, hc2, lp, v, act_out=act,
                                     seed=self.seed, counter=self._counter)
        a.mode = MM_MAPPO_ROLLOUT
        a.deterministic = 1 if deterministic else 0
        self._counter += 1
        self.policy._fwd(a)
        return act.long().view(R, 1), ha2.view(R, 1, self.hidden)

    def evaluate_actions(self, cent_obs, obs, rnn_states_actor, rnn_states_critic, action, masks,
                         available_actions=None, active_masks=None):
        """A minibatch of n recurrent chunks of length L (rows ordered (l, j), chunk-start hiddens [n, 1, H],
        shared_buffer.py:318-427) through the TRAIN-mode fused forward: values [L*n, 1], log-probs of
        ``action`` [L*n, 1], entropy (masked mean over active_masks, r_actor_critic.py:95-140)."""
        from .mappo import MappoBuffer, MappoTrainer
        obs_t = self._t(obs)
        self._same_input(obs_t, cent_obs)
        rows = obs_t.shape[0]
        ha0 = self._t(rnn_states_actor)
        n = ha0.shape[0]
        L = rows // n
        assert L * n == rows, "rows must be a whole number of chunks"
        key = (L, n)
        if key not in self._eval:
            buf = MappoBuffer(L, n, 1, self.policy.D, self.hidden, self.device)
            self._eval[key] = (buf, MappoTrainer(self.policy, L, n, L=L, ppo_epoch=1, fused=False))
        buf, tr = self._eval[key]
        buf.obs[:L].copy_(obs_t.view(L, n, -1))
        buf.masks[:L].copy_(self._t(masks).view(L, n))
        buf.rnn_states[0].copy_(ha0.reshape(n, self.hidden))
        buf.rnn_states_critic[0].copy_(self._t(rnn_states_critic).reshape(n, self.hidden))
        d = ctypes.byref(self.policy.dims)
        check(lib().mm_mappo_fwd(d, ctypes.byref(tr.fwd_args(buf)), stream_handle(self.device)), "mappo_fwd(train)")
        A = self.policy.A
        ns0 = lib().mm_mappo_save_fields(d, 0)
        ns1 = lib().mm_mappo_save_fields(d, 1)
        s0 = tr.save[0].view(-1, ns0, 64)
        logp_all = s0[:, ns0 - A:, :].permute(0, 2, 1).reshape(-1, A)[:rows]
        values = tr.save[1].view(-1, ns1, 64)[:, ns1 - 1, :].reshape(-1)[:rows]
        act = self._t(action).reshape(rows, 1).long()
        lp = logp_all.gather(1, act)
        ent = -(logp_all.exp() * logp_all).sum(-1, keepdim=True)
        if active_masks is not None:
            am = self._t(active_masks).reshape(rows, 1)
            dist_entropy = (ent * am).sum() / am.sum()
        else:
            dist_entropy = ent.mean()
        return values.view(rows, 1), lp, dist_entropy
