"""Device learner for chunked-BPTT QMIX / VDN (csrc/learner.hip + the fused agent forward).

Mirrors ``Train_dqn`` (qmix/_train.py:7-121) and ``Target_Dqn`` (vdn/_train.py:184-235):
one ``update()`` = PER sample of B chunks x C steps, behavior + target agent nets and
mixers forward over the C steps, loss, backward through time, clip_grad_norm_ (QMIX:
agent params only, qmix/_train.py:111-115; VDN: all), Adam, priority update with the
last step's |y - Q_tot|. Everything is enqueued on the current HIP stream with no host
sync, so an update can be captured as one HIP graph and replayed.

Mode "vdn_double" is ``Target_Double_Dqn`` (vdn/_train.py:104-158): the bootstrap is the target
net's Q at the actions an epsilon-greedy copy of the behavior net picks on s' (its own hidden
chain), Σ_i Q_tgt(s', a*_i); everything else as "vdn". The draws are injected
(``set_double_draws``) or come from the device counter RNG.

Mode "qmix_min" is the minimal QMIX of ``qmix/qmix.py`` (``train``
qmix/qmix.py:174-238): target Σ_i r_i + γ(1-d)Q'_tot (no xN, no IS weight), smooth-L1 loss,
clip_grad_norm_ on the agent net and on the mixer separately, uniform chunk replay
(``sample_uniform_and_grads``); its nets are QNet(D->128->32, GRUCell 32) and MixNet(hx 64).

Parameters live in ONE flat fp32 buffer ``P = [agent theta | mixer phi]`` (grads,
Adam moments alike), the layout the RCCL gradient all-reduce works on.
"""
import ctypes
import math

import numpy as np
import torch

from ._lib import (MM_LOSS_HUBER, MM_LOSS_MIX_SUM, MM_LOSS_TARGET_SUM, MM_Q_ACT, MM_Q_GATHER, MM_Q_MAX, MixNetIO,
                   OuterArgs, QFwdIO, TmvArgs, c_i64, check, lib)
from .qnet import KEYS as AGENT_KEYS
from .qnet import AgentQNet, graph_capture, ptr, stream_handle

MIX_KEYS = ["gWih", "gWhh", "gbih", "gbhh", "w1W", "w1b", "w2W", "w2b", "b1W", "b1b", "b2aW", "b2ab", "b2bW",
            "b2bb"]
_MIX_FMT = {
    "gWih": "gru.weight_ih", "gWhh": "gru.weight_hh", "gbih": "gru.bias_ih", "gbhh": "gru.bias_hh",
    "w1W": "hyper_net_weight_1.weight", "w1b": "hyper_net_weight_1.bias",
    "w2W": "hyper_net_weight_2.weight", "w2b": "hyper_net_weight_2.bias",
    "b1W": "hyper_net_bias_1.weight", "b1b": "hyper_net_bias_1.bias",
    "b2aW": "hyper_net_bias_2.0.weight", "b2ab": "hyper_net_bias_2.0.bias",
    "b2bW": "hyper_net_bias_2.2.weight", "b2bb": "hyper_net_bias_2.2.bias",
}


class Mixer:
    """QMIX Mix_Net parameters (qmix/_network.py:172-220): GRUCell(N*D -> Hm) + hypernetworks."""

    def __init__(self, n_agents, state_dim, hm=32, k1=32, device="cuda", flat=None, seed=None):
        self.N, self.S, self.Hm, self.K1 = n_agents, state_dim, hm, k1
        self.device = torch.device(device)
        n = c_i64()
        check(lib().mm_mixer_param_count(state_dim, hm, k1, n_agents, ctypes.byref(n)), "mixer_param_count")
        self.n_params = n.value
        self.flat = flat if flat is not None else torch.zeros(self.n_params, device=self.device)
        assert self.flat.numel() == self.n_params
        sh = self.shapes()
        self.offs = [0]
        for k in MIX_KEYS:
            self.offs.append(self.offs[-1] + int(np.prod(sh[k])))
        assert self.offs[-1] == self.n_params
        if seed is not None:
            self.init_default(seed)

    def shapes(self):
        N, S, Hm, K1 = self.N, self.S, self.Hm, self.K1
        return {"gWih": (3 * Hm, S), "gWhh": (3 * Hm, Hm), "gbih": (3 * Hm,), "gbhh": (3 * Hm,),
                "w1W": (N * K1, Hm), "w1b": (N * K1,), "w2W": (K1, Hm), "w2b": (K1,), "b1W": (K1, Hm),
                "b1b": (K1,), "b2aW": (K1, Hm), "b2ab": (K1,), "b2bW": (1, K1), "b2bb": (1,)}

    def view(self, key, t=None):
        t = self.flat if t is None else t
        i = MIX_KEYS.index(key)
        return t[self.offs[i]:self.offs[i + 1]].view(self.shapes()[key])

    def init_default(self, seed):
        g = torch.Generator().manual_seed(int(seed))
        fan = {"gWih": self.Hm, "gWhh": self.Hm, "gbih": self.Hm, "gbhh": self.Hm, "w1W": self.Hm,
               "w1b": self.Hm, "w2W": self.Hm, "w2b": self.Hm, "b1W": self.Hm, "b1b": self.Hm, "b2aW": self.Hm,
               "b2ab": self.Hm, "b2bW": self.K1, "b2bb": self.K1}
        host = torch.empty(self.n_params)
        for i, k in enumerate(MIX_KEYS):
            b = 1.0 / math.sqrt(fan[k])
            host[self.offs[i]:self.offs[i + 1]] = (torch.rand(self.offs[i + 1] - self.offs[i], generator=g) * 2 - 1) * b
        self.flat.copy_(host.to(self.device))

    def load_reference_state(self, sd, prefix=""):
        host = torch.cat([torch.as_tensor(np.asarray(sd[prefix + _MIX_FMT[k]]), dtype=torch.float32).reshape(-1)
                          for k in MIX_KEYS])
        self.flat.copy_(host.to(self.device))

    def state_dict(self):
        host = self.flat.detach().cpu()
        return {_MIX_FMT[k]: self.view(k, host).clone() for k in MIX_KEYS}


class QLearner:
    """mode "qmix" (Train_dqn), "vdn" (Target_Dqn: Q_tot = sum_i Q_i, no mixer) or "qmix_min"
    (qmix/qmix.py train: Huber loss, unweighted sum target, separate agent / mixer clipping)."""

    def __init__(self, behavior, target, mixer=None, target_mixer=None, batch=32, chunk=10, gamma=0.99, lr=1e-3,
                 grad_clip=5.0, betas=(0.9, 0.999), adam_eps=1e-8, mode="qmix", clip_mixer=False, device="cuda",
                 reference_compat=True, mixer_fp16=False, pair_bwd=True, fwd_side=True, pair_fwd=True):
        assert mode in ("qmix", "vdn", "qmix_min", "vdn_double")
        self.mode = mode
        self.has_mixer = mode in ("qmix", "qmix_min")
        self.double = mode == "vdn_double"
        self.loss_flags = {"qmix": 0, "vdn": MM_LOSS_MIX_SUM, "vdn_double": MM_LOSS_MIX_SUM,
                           "qmix_min": MM_LOSS_HUBER | MM_LOSS_TARGET_SUM}[mode]
        # reference_compat=False replaces the reference's TD target w * (sum_i r_i + N * gamma * (1-d) * Q'_tot)
        # (vdn/_train.py:76-77, qmix/_train.py:80-82: the bootstrap is multiplied by the
        # agent count and the IS weight scales the target) by the textbook sum_i r_i + gamma * (1-d) * Q'_tot
        # of qmix/qmix.py:215-217 (no IS weight)
        self.reference_compat = bool(reference_compat)
        # cfg5 mode: the mixer state projection [B*C, N*D] x [N*D, 3Hm] on fp16 MFMA (rtol 2e-3
        # on Q_tot, a tolerance stated apart from the fp32 parity); at B*C >= 2048 also the MIXER's batched
        # weight-gradient products as bf16x3 splits (mm_outer_reduce_batch_bf3, ~2^-16 relative); the agent path
        # stays exact f32
        self.mixer_fp16 = bool(mixer_fp16)
        # the agent BPTT and the mixer recurrence's backward in one launch (pair_bwd=False: side stream)
        self._pair_bwd = bool(pair_bwd)
        # the mixer's forward state projection + recurrence on a side stream (fwd_side=False: in line)
        self._fwd_side = bool(fwd_side)
        # the forward's agent and mixer chains in shared grids (mm_agent_mixer_pre / mm_agent_mixer_rec_seq) where
        # the shapes allow: no fork / join at all (pair_fwd=False: the side stream above)
        self._pair_fwd = bool(pair_fwd)
        self._pair_ok = None
        self._per_next = None          # the PER of the update being recorded (sample_and_grads -> compute_grads)
        self._per_done = False         # its priority update already issued (with the hypernet backward)
        self.fast_pre = False           # opt-in: the fp16x3 agent PRE (not at the fp32 gradient bar, see compute_grads)
        if not self.reference_compat:
            self.loss_flags |= MM_LOSS_TARGET_SUM
        # chunk-sequence launches: agent REC and mixer backward as one launch each for all C steps
        self.seq = not self.double
        self.double_eps = 0.0          # epsilon of the double net's sample_action (vdn/_train.py:124-125)
        self.double_seed = 0x5eed
        self._draws = None
        self.dev = torch.device(device)
        self.beh, self.tgt = behavior, target
        self.mix, self.tmix = mixer, target_mixer
        if self.has_mixer:
            assert mixer is not None and target_mixer is not None
        self.B, self.C = int(batch), int(chunk)
        self.gamma, self.lr, self.clip = float(gamma), float(lr), float(grad_clip)
        self.b1, self.b2, self.aeps = float(betas[0]), float(betas[1]), float(adam_eps)
        d = behavior
        self.N, self.D, self.F1, self.G, self.H, self.A = d.N, d.D, d.F1, d.G, d.H, d.A
        self.SD = self.F1 + self.G + 6 * self.H
        # one flat buffer [theta | phi]; the nets become views into it
        n_t = d.n_params
        n_m = mixer.n_params if mixer is not None else 0
        self.n_agent, self.n = n_t, n_t + n_m
        for net in (behavior, mixer):
            if net is not None and getattr(net, "_owner", None) is not None:
                raise ValueError("this net's parameters already live in another QLearner's flat buffer; "
                                 "give each learner its own AgentQNet / Mixer (copy_from)")
        self.P = torch.empty(self.n, device=self.dev)
        self.P[:n_t].copy_(behavior.flat)
        behavior.flat = self.P[:n_t]
        behavior._owner = self
        behavior.mark_dirty()
        if mixer is not None:
            self.P[n_t:].copy_(mixer.flat)
            mixer.flat = self.P[n_t:]
            mixer._owner = self
        self.Gr = torch.zeros(self.n, device=self.dev)
        self.m = torch.zeros(self.n, device=self.dev)
        self.v = torch.zeros(self.n, device=self.dev)
        self.step_dev = torch.zeros(1, device=self.dev)
        self.partials = torch.zeros(512, device=self.dev)
        self.norm = torch.zeros(2, device=self.dev)
        self.n_clip = self.n if (not self.has_mixer or clip_mixer) else n_t
        self._alloc()
        self.updates = 0

    # ------------------------------------------------------------------ workspace
    def _alloc(self):
        B, C, N, H, A, dev = self.B, self.C, self.N, self.H, self.A, self.dev
        f32 = dict(device=dev, dtype=torch.float32)
        self.s_off = torch.zeros(C * B, dtype=torch.int64, device=dev)
        self.s2_off = torch.zeros(C * B, dtype=torch.int64, device=dev)
        self.acts = torch.zeros(C * B * N, dtype=torch.int32, device=dev)
        self.rew = torch.zeros(C * B * N, **f32)
        self.done = torch.zeros(C * B, **f32)
        self.done8 = torch.zeros(C * B, dtype=torch.uint8, device=dev)
        self.isw = torch.ones(B, **f32)
        self.ones8 = torch.ones(B, dtype=torch.uint8, device=dev)
        self.ones_f = torch.ones(B, **f32)
        self.hb = torch.zeros(2, B, N, H, **f32)
        self.ht = torch.zeros(2, B, N, H, **f32)
        self.asave = torch.zeros(C, B, N, self.SD, **f32)
        self.gi_ab = torch.zeros(C, B, N, 3 * H, **f32)   # agent GRU input projections (split forward)
        self.gi_at = torch.zeros(C, B, N, 3 * H, **f32)
        self.qa = torch.zeros(C, B, N, **f32)
        self.maxq = torch.zeros(C, B, N, **f32)
        self.qtot = torch.zeros(C, B, **f32)
        self.qtot_t = torch.zeros(C, B, **f32)
        self.dq = torch.zeros(C, B, **f32)
        self.dqa = torch.zeros(C, B, N, **f32)
        self.loss_parts = torch.zeros(C, B, **f32)
        self.td_last = torch.zeros(B, **f32)
        self.loss = torch.zeros(1, **f32)
        self.dh = torch.zeros(B, N, H, **f32)
        self.dgi = torch.zeros(C, B, N, 3 * H, **f32)
        self.dgh = torch.zeros(C, B, N, 3 * H, **f32)
        self.dqv = torch.zeros(C, B, N, A, **f32)
        self.dpre2 = torch.zeros(C, B, N, self.G, **f32)
        self.dpre1 = torch.zeros(C, B, N, self.F1, **f32)
        if self.double:
            # the double net's eps-greedy RNG counters (one per chunk step) and epsilon live on the
            # device, so a captured update advances them on every replay (counter = update * C + t,
            # the same values the eager path uses)
            self.dctr = torch.arange(C, dtype=torch.int64, device=dev) - C
            self.deps = torch.zeros(1, **f32)
            self.hd = torch.zeros(2, B, N, H, **f32)
            self.gi_ad = torch.zeros(C, B, N, 3 * H, **f32)
            self.act_d = torch.zeros(C, B, N, dtype=torch.int32, device=dev)
            self.qsel_d = torch.zeros(C, B, N, **f32)
        self.nodes = torch.zeros(B, dtype=torch.int64, device=dev)
        self.slots = torch.zeros(B, dtype=torch.int64, device=dev)
        if self.has_mixer:
            Hm, K1 = self.mix.Hm, self.mix.K1
            self.MSD = lib().mm_mixer_save_dim(Hm, K1, N)
            self.MDD = lib().mm_mixer_delta_dim(Hm, K1, N)
            self.hm = torch.zeros(2, B, Hm, **f32)
            self.hmt = torch.zeros(2, B, Hm, **f32)
            self.msave = torch.zeros(C, B, self.MSD, **f32)
            self.mdelta = torch.zeros(C, B, self.MDD, **f32)
            self.dhm = torch.zeros(B, Hm, **f32)
            self.mhseq = torch.zeros(2, C, B, Hm, **f32)   # mixer hidden sequences (behavior, target)
            self.mxws = torch.zeros(C, B, 4, Hm, **f32)    # hypernet input gradients (mm_mixer_bwd_seq)
            self.gi_b = torch.zeros(C, B, 3 * Hm, **f32)
            self.gi_t = torch.zeros(C, B, 3 * Hm, **f32)
        # split-M outer-reduce partials: the job geometry is fixed, size it once (no launches here)
        jobs = []
        zero = ctypes.c_void_p(0)
        self._agent_wgrad(None, None, zero, zero, C * B, jobs)
        if self.has_mixer:
            self._mixer_wgrad(None, None, zero, zero, C * B, jobs)
        arr = (OuterArgs * len(jobs))(*jobs)
        self._opart = torch.zeros(int(lib().mm_outer_reduce_batch_partial(arr, len(jobs))), **f32)

    # ------------------------------------------------------------------ batch in
    def gather(self, per, store):
        """PER slots (self.slots) -> chunk-store rows -> offsets / actions / rewards / dones."""
        check(lib().mm_lrn_gather(self.B, self.C, self.N, store.row_stride, self.N * self.D, ptr(self.slots),
                                  ctypes.c_void_p(per.slot_rows_ptr()), ptr(store.done), ptr(store.act),
                                  ptr(store.rew), ptr(self.s_off), ptr(self.s2_off), ptr(self.acts), ptr(self.rew),
                                  ptr(self.done), ptr(self.done8), stream_handle(self.dev)), "lrn_gather")

    def load_batch(self, states, actions, rewards, next_states, dones, is_weight):
        """Reference-shaped batch (Replay_buffer.sample outputs, qmix/replay_buffer/per.py:77-81) as the
        learner input: obs rows are laid out in a private buffer and addressed through the offsets."""
        B, C, N, D = self.B, self.C, self.N, self.D
        st = torch.as_tensor(states, dtype=torch.float32).to(self.dev).contiguous()
        ns = torch.as_tensor(next_states, dtype=torch.float32).to(self.dev).contiguous()
        assert st.shape == (B, C, N, D) and ns.shape == (B, C, N, D)
        self._obs_buf = torch.cat([st.reshape(-1), ns.reshape(-1)])
        t = torch.arange(C, device=self.dev).view(C, 1)
        b = torch.arange(B, device=self.dev).view(1, B)
        base = (b * C + t) * (N * D)
        self.s_off.copy_(base.reshape(-1))
        self.s2_off.copy_((base + B * C * N * D).reshape(-1))
        self.acts.copy_(torch.as_tensor(actions).to(self.dev).permute(1, 0, 2).reshape(-1).to(torch.int32))
        self.rew.copy_(torch.as_tensor(rewards, dtype=torch.float32).to(self.dev).permute(1, 0, 2).reshape(-1))
        dn = torch.as_tensor(dones, dtype=torch.float32).to(self.dev).view(B, C).t().reshape(-1)
        self.done.copy_(dn)
        self.done8.copy_((dn > 0.5).to(torch.uint8))
        self.isw.copy_(torch.as_tensor(is_weight, dtype=torch.float32).to(self.dev).view(-1))
        self._obs_ptr = self._obs_buf
        self._reset_obs = self._obs_buf      # never addressed (no -1 offsets in an explicit batch)

    def set_double_draws(self, u=None, rand_act=None):
        """Inject the double net's epsilon-greedy draws per chunk step (the reference's torch.rand(B)
        and torch.randint rows, vdn/_network.py:52-58): u [C, B] f32, rand_act [C, B, N] (only rows
        with u <= epsilon are used). None: device counter RNG."""
        if u is None:
            self._draws = None
            return
        C, B, N = self.C, self.B, self.N
        uu = torch.as_tensor(u, dtype=torch.float32).to(self.dev).reshape(C, B).contiguous()
        ra = torch.as_tensor(rand_act).to(self.dev).to(torch.int32).reshape(C, B, N).contiguous()
        self._draws = (uu, ra)

    # ------------------------------------------------------------------ the update
    def _push_double_eps(self):
        if self.double and self._deps_host != self.double_eps:
            self.deps.fill_(float(self.double_eps))
            self._deps_host = self.double_eps

    _deps_host = None

    def compute_grads(self, obs_base, reset_obs_ptr):
        """Forward C steps, loss, BPTT and all weight gradients into self.Gr (all async)."""
        L, s = lib(), stream_handle(self.dev)
        if not torch.cuda.is_current_stream_capturing():
            self._push_double_eps()
        B, C, N, H, D = self.B, self.C, self.N, self.H, self.D
        CB = C * B
        self._pack(self.beh, s)
        self._pack(self.tgt, s)
        obs_p = ctypes.c_void_p(obs_base) if isinstance(obs_base, int) else ptr(obs_base)
        reset_p = ctypes.c_void_p(reset_obs_ptr) if isinstance(reset_obs_ptr, int) else ptr(reset_obs_ptr)
        ND = N * D
        split = self._mixer_split()
        pair = bool(split) and self._fwd_pair()
        side = self._side_stream() if split else None
        fwd_side = split and self._fwd_side and not pair
        if fwd_side:
            # two streams (captured as a fork / join in the update graph): the mixer's state projection and its
            # GRU recurrence need no agent Q, so they run beside the agent PRE / REC chain
            side.wait_stream(torch.cuda.current_stream(self.dev))
            s_m = ctypes.c_void_p(side.cuda_stream)
        else:
            s_m = s
        if self.has_mixer and not pair:
            # mixer GRU input projections of every (t, b) for both mixers: one MFMA launch
            mx = self.mix
            gi_fn = L.mm_mixer_gi_f16 if self.mixer_fp16 else L.mm_mixer_gi
            check(gi_fn(CB, N, mx.S, mx.Hm, mx.K1, obs_p, reset_p, ptr(mx.flat), ptr(self.s_off),
                        ptr(self.gi_b), ptr(self.tmix.flat), ptr(self.s2_off), ptr(self.gi_t), s_m), "mixer gi")
            if split:
                self._mixer_seq_call(L, L.mm_mixer_fwd_seq_rec, s_m, "mixer fwd seq (recurrence)")
        # ---- forward over the chunk: the non-recurrent part (layers 1-2, W_ih x2) of every (t, b) of
        # both nets in ONE launch, then one recurrent step (W_hh h, gates, Q head) per t
        pb, pt = QFwdIO(), QFwdIO()
        for io, off, gi in ((pb, self.s_off, self.gi_ab), (pt, self.s2_off, self.gi_at)):
            io.obs, io.obs_se, io.obs_sa, io.obs_off = obs_p.value, 1, D, 0
            io.obs_row = off.data_ptr()
            io.reset_obs = reset_p.value
            io.h_in = self.hb.data_ptr()       # unused by PRE
            io.gi = gi.data_ptr()
        pb.save = self.asave.data_ptr()
        # the agent PRE stays exact f32 in every mode: on the fp16x3 image (mm_agent_q_pre2_h3) the split weights'
        # lo parts of a wide layer 1 (D = 300, |W| ~ 0.06) fall into f16's subnormal range, and the few ReLU masks that
        # flip against f32 put ~0.3 % of dW1 / dW2 outside the fp32 bar (test_learner_cfg5_benched_path_vs_oracle)
        pre_fn = L.mm_agent_q_pre2_h3 if (self.mixer_fp16 and CB >= 2048 and self.fast_pre) else L.mm_agent_q_pre2
        if pair:
            # + the mixers' state projection (mm_mixer_gi) in the same grid
            mx = self.mix
            check(L.mm_agent_mixer_pre(ctypes.byref(self.beh.dims), ptr(self.beh.packed), ctypes.byref(pb),
                                       ptr(self.tgt.packed), ctypes.byref(pt), CB, N, mx.S, mx.Hm, mx.K1, obs_p,
                                       reset_p, ptr(mx.flat), ptr(self.s_off), ptr(self.gi_b), ptr(self.tmix.flat),
                                       ptr(self.s2_off), ptr(self.gi_t), s), "learner fwd pre + mixer gi")
        else:
            check(pre_fn(ctypes.byref(self.beh.dims), ptr(self.beh.packed), ctypes.byref(pb), CB,
                         ptr(self.tgt.packed), ctypes.byref(pt), CB, s), "learner fwd pre")
        if self.double:   # the double net (behavior weights) on s'
            pd = QFwdIO()
            pd.obs, pd.obs_se, pd.obs_sa, pd.obs_off = obs_p.value, 1, D, 0
            pd.obs_row = self.s2_off.data_ptr()
            pd.reset_obs = reset_p.value
            pd.h_in = self.hb.data_ptr()
            pd.gi = self.gi_ad.data_ptr()
            check(L.mm_agent_q_pre2(ctypes.byref(self.beh.dims), ptr(self.beh.packed), ctypes.byref(pd), CB,
                                    None, None, 0, s), "learner fwd pre (double)")
        gstep = 4 * B * N * 3 * H
        if self.double and self._draws is None:
            self.dctr.add_(C)             # stream-ordered: captured into the update graph
        if self.seq:
            self._forward_seq(L, s, obs_p, reset_p, split, join=fwd_side, pair=pair)
        for t in range(0 if not self.seq else C, C):
            ib, it = QFwdIO(), QFwdIO()
            for io, h, gi in ((ib, self.hb, self.gi_ab), (it, self.ht, self.gi_at)):
                io.obs = obs_p.value               # unused by REC
                io.h_in = h[t % 2].data_ptr()
                io.h_out = h[(t + 1) % 2].data_ptr()
                io.hin_se = io.hout_se = N * H
                io.hin_sa = io.hout_sa = H
                io.hin_sf = io.hout_sf = 1
                io.reset = self.ones8.data_ptr() if t == 0 else self.done8.data_ptr() + (t - 1) * B
                io.gi = gi.data_ptr() + t * gstep
            ib.mode = MM_Q_GATHER
            ib.act_in, ib.act_se = self.acts.data_ptr() + 4 * t * B * N, N
            ib.qsel_out = self.qa[t].data_ptr()
            ib.save = self.asave[t].data_ptr()
            it.mode = MM_Q_MAX
            it.qsel_out = self.maxq[t].data_ptr()
            if self.double:
                # behavior on s_t + the double net's eps-greedy actions on s'_t, then the target net's
                # Q at those actions (Target_Double_Dqn, vdn/_train.py:121-130)
                idd = QFwdIO()
                idd.obs = obs_p.value
                idd.h_in, idd.h_out = self.hd[t % 2].data_ptr(), self.hd[(t + 1) % 2].data_ptr()
                idd.hin_se = idd.hout_se = N * H
                idd.hin_sa = idd.hout_sa = H
                idd.hin_sf = idd.hout_sf = 1
                idd.reset = it.reset
                idd.gi = self.gi_ad.data_ptr() + t * gstep
                idd.mode = MM_Q_ACT
                idd.act_out = self.act_d[t].data_ptr()
                idd.qsel_out = self.qsel_d[t].data_ptr()
                idd.epsilon = float(self.double_eps)
                idd.eps_ptr = self.deps.data_ptr()
                if self._draws is not None:
                    idd.u = self._draws[0][t].data_ptr()
                    idd.rand_act = self._draws[1][t].data_ptr()
                else:
                    idd.seed = self.double_seed
                    idd.counter_ptr = self.dctr.data_ptr() + 8 * t
                check(L.mm_agent_q_rec2(ctypes.byref(self.beh.dims), ptr(self.beh.packed), ctypes.byref(ib), B,
                                        ptr(self.beh.packed), ctypes.byref(idd), B, s), "learner fwd rec")
                it.mode = MM_Q_GATHER
                it.act_in, it.act_se = self.act_d[t].data_ptr(), N
                check(L.mm_agent_q_rec2(ctypes.byref(self.beh.dims), ptr(self.tgt.packed), ctypes.byref(it), B,
                                        None, None, 0, s), "learner fwd rec (target at double actions)")
            else:
                check(L.mm_agent_q_rec2(ctypes.byref(self.beh.dims), ptr(self.beh.packed), ctypes.byref(ib), B,
                                        ptr(self.tgt.packed), ctypes.byref(it), B, s), "learner fwd rec")
            if self.has_mixer:
                mx = self.mix
                nets = (MixNetIO * 2)()
                for k, (P, q, off, h, qt, sv, gi) in enumerate(
                        ((self.mix.flat, self.qa[t], self.s_off, self.hm, self.qtot[t], self.msave[t], self.gi_b[t]),
                         (self.tmix.flat, self.maxq[t], self.s2_off, self.hmt, self.qtot_t[t], None, self.gi_t[t]))):
                    n = nets[k]
                    n.P, n.q, n.gi = P.data_ptr(), q.data_ptr(), gi.data_ptr()
                    n.s_off = off.data_ptr() + 8 * t * B
                    n.h_in, n.h_out = h[t % 2].data_ptr(), h[(t + 1) % 2].data_ptr()
                    n.reset = self.ones8.data_ptr() if t == 0 else self.done8.data_ptr() + (t - 1) * B
                    n.qtot = qt.data_ptr()
                    n.save = sv.data_ptr() if sv is not None else None
                check(L.mm_mixer_fwd(B, N, mx.S, mx.Hm, mx.K1, obs_p, reset_p, nets, 2, s), "mixer fwd")
        # ---- loss, dQ_tot, priorities
        check(L.mm_lrn_loss_ex(B, C, N, self.gamma, ptr(self.rew), ptr(self.done), ptr(self.isw), ptr(self.qtot),
                               ptr(self.qtot_t), self.loss_flags, ptr(self.qa), ptr(self.maxq), ptr(self.dq),
                               ptr(self.dqa), ptr(self.loss_parts), ptr(self.td_last), ptr(self.loss), s), "loss")
        # ---- backward through time (data-gradient chains only)
        agent_seq = self.seq and B < 512 and self.H in (32, 64)
        pair_bwd = bool(split) and agent_seq and self.has_mixer and self._pair_bwd
        o = self.beh.offs
        P = self.P
        if self.seq:
            if self.has_mixer:
                mx = self.mix
                margs = (B, N, mx.S, mx.Hm, mx.K1, ptr(mx.flat), ptr(self.msave), ptr(self.qa), ptr(self.dq),
                         ptr(self.done), ptr(self.ones_f), ptr(self.dhm), ptr(self.dqa), ptr(self.mdelta),
                         ptr(self.mxws), C)
                if split:
                    # the hypernet pass (-> dqa for the agents), then the mixer recurrence's backward beside the
                    # agent BPTT: one shared launch below (mm_agent_mixer_bwd_seq), or the side stream joined
                    # before the weight gradients. A sampled update's priority update rides along (the loss's TDs
                    # are final): one more block of the hypernet launch
                    if self._per_next is not None:
                        check(L.mm_mixer_bwd_seq_hyper_per(*margs, self._per_next._h, ptr(self.nodes),
                                                           ptr(self.td_last), self.B, s),
                              "mixer bwd seq (hypernets) + priority update")
                        self._per_done = True
                    else:
                        check(L.mm_mixer_bwd_seq_hyper(*margs, s), "mixer bwd seq (hypernets)")
                    if not pair_bwd:
                        side.wait_stream(torch.cuda.current_stream(self.dev))
                        check(L.mm_mixer_bwd_seq_rec(*margs, s_m), "mixer bwd seq (recurrence)")
                else:
                    check(L.mm_mixer_bwd_seq(*margs, s), "mixer bwd seq")
        self._per_next = None
        if pair_bwd:
            # the agent BPTT chain and the mixer recurrence's backward sharing one grid
            mx = self.mix
            check(L.mm_agent_mixer_bwd_seq(ctypes.byref(self.beh.dims), ptr(P), o[8], o[5], B, ptr(self.asave),
                                           ptr(self.acts), ptr(self.dqa), ptr(self.done), ptr(self.ones_f),
                                           ptr(self.dh), ptr(self.dgi), ptr(self.dgh), ptr(self.dqv), C, mx.S, mx.Hm,
                                           mx.K1, ptr(mx.flat), ptr(self.msave), ptr(self.qa), ptr(self.dq),
                                           ptr(self.dhm), ptr(self.mdelta), ptr(self.mxws), s), "agent+mixer bwd seq")
        elif agent_seq:
            # the agent BPTT chain over all C steps in one launch (W_hh in LDS, dh carried in registers)
            check(L.mm_agent_bwd_seq(ctypes.byref(self.beh.dims), ptr(P), o[8], o[5], B, ptr(self.asave),
                                     ptr(self.acts), ptr(self.dqa), ptr(self.done), ptr(self.ones_f), ptr(self.dh),
                                     ptr(self.dgi), ptr(self.dgh), ptr(self.dqv), C, s), "agent bwd seq")
        for t in range(C - 1, -1, -1):
            if agent_seq:
                break
            dn = self.ones_f if t == C - 1 else self.done[t * B:(t + 1) * B]
            if self.has_mixer and not self.seq:
                mx = self.mix
                check(L.mm_mixer_bwd(B, N, mx.S, mx.Hm, mx.K1, ptr(mx.flat), ptr(self.msave[t]), ptr(self.qa[t]),
                                     ptr(self.dq[t]), ptr(dn), ptr(self.dhm), ptr(self.dqa[t]), ptr(self.mdelta[t]),
                                     s), "mixer bwd")
            check(L.mm_agent_bwd(ctypes.byref(self.beh.dims), ptr(P), o[8], o[5], B, ptr(self.asave[t]),
                                 ctypes.c_void_p(self.acts.data_ptr() + 4 * t * B * N), ptr(self.dqa[t]), ptr(dn),
                                 ptr(self.dh), ptr(self.dgi[t]), ptr(self.dgh[t]), ptr(self.dqv[t]), s), "agent bwd")
        if split and not pair_bwd:
            torch.cuda.current_stream(self.dev).wait_stream(side)   # join: the mixer deltas are complete
        # ---- deferred weight gradients: batched over all C*B rows, grouped by agent; every
        # outer product of the update (agent + mixer) in ONE split-M launch (+ its partial sum)
        jobs = []
        self._agent_wgrad(L, s, obs_p, reset_p, CB, jobs)
        mjobs = []
        if self.has_mixer:
            self._mixer_wgrad(L, s, obs_p, reset_p, CB, mjobs)
        if self.mixer_bf3:
            # fast mode at large batches: the agent weight gradients stay exact f32 (the fp32 parity bar); only
            # the MIXER's products run as bf16x3 splits (~2^-16 relative), a second launch over the same partials
            arr = (OuterArgs * len(jobs))(*jobs)
            check(L.mm_outer_reduce_batch(arr, len(jobs), ptr(self._opart), self._opart.numel(), s), "outer batch")
            marr = (OuterArgs * len(mjobs))(*mjobs)
            check(L.mm_outer_reduce_batch_bf3(marr, len(mjobs), ptr(self._opart), self._opart.numel(), s),
                  "outer batch (mixer, bf16x3)")
            return
        jobs += mjobs
        arr = (OuterArgs * len(jobs))(*jobs)
        check(L.mm_outer_reduce_batch(arr, len(jobs), ptr(self._opart), self._opart.numel(), s), "outer batch")

    @property
    def mixer_bf3(self):
        """cfg5 fast mode at large batches: the mixer's weight-gradient products as bf16x3 splits."""
        return self.mixer_fp16 and self.has_mixer and self.C * self.B >= 2048

    def _side_stream(self):
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.dev)
        return self._side

    def _fwd_pair(self):
        """Both paired forward launches apply (QMIX, exact-f32 state projection, the B = 32 shapes)."""
        if self._pair_ok is None:
            mx = self.mix
            self._pair_ok = bool(self._pair_fwd and self.has_mixer and not self.double and not self.mixer_fp16 and
                                 lib().mm_agent_mixer_pair_supported(ctypes.byref(self.beh.dims), self.B, self.C,
                                                                     self.N, mx.S, mx.Hm, mx.K1) == 3)
        return self._pair_ok

    def _mixer_split(self):
        """The mixer's state projection + GRU recurrence run on a second stream beside the agent chain (and its
        recurrence backward beside the agent BPTT): sequence path, both split mixer kernels available."""
        if not (self.has_mixer and self.seq and self.B < 512):
            return False
        mx = self.mix
        return bool(lib().mm_mixer_seq_split(self.B, self.N, mx.S, mx.Hm, mx.K1, ptr(mx.flat), ptr(self.mxws),
                                             self.C))

    def _mixer_nets(self):
        nets = (MixNetIO * 2)()
        for k, (Pm, q, qt, sv, gi) in enumerate(((self.mix.flat, self.qa, self.qtot, self.msave, self.gi_b),
                                                  (self.tmix.flat, self.maxq, self.qtot_t, None, self.gi_t))):
            n = nets[k]
            n.P, n.q, n.gi, n.qtot = Pm.data_ptr(), q.data_ptr(), gi.data_ptr(), qt.data_ptr()
            n.s_off = self.s_off.data_ptr()
            n.h_in, n.h_out = self.hm[0].data_ptr(), self.mhseq[k].data_ptr()
            n.reset = self.ones8.data_ptr()
            n.save = sv.data_ptr() if sv is not None else None
        return nets

    def _mixer_seq_call(self, L, fn, s, what):
        mx = self.mix
        check(fn(self.B, self.N, mx.S, mx.Hm, mx.K1, self._mixer_nets(), 2, self.C, ptr(self.done8), s), what)

    def _forward_seq(self, L, s, obs_p, reset_p, split=False, join=False, pair=False):
        """REC of both nets over all C steps in one chunk-sequence launch, then the mixers per step."""
        B, C, N, H = self.B, self.C, self.N, self.H
        ib, it = QFwdIO(), QFwdIO()
        for io, gi in ((ib, self.gi_ab), (it, self.gi_at)):
            io.obs = obs_p.value
            io.gi = gi.data_ptr()
        ib.mode = MM_Q_GATHER
        ib.act_in, ib.act_se = self.acts.data_ptr(), N
        ib.qsel_out = self.qa.data_ptr()
        ib.save = self.asave.data_ptr()
        it.mode = MM_Q_MAX
        it.qsel_out = self.maxq.data_ptr()
        if pair:
            # + the mixers' GRU over the state (mm_mixer_fwd_seq_rec) in the same grid, then the hypernet pass
            mx = self.mix
            check(L.mm_agent_mixer_rec_seq(ctypes.byref(self.beh.dims), ptr(self.beh.packed), ctypes.byref(ib),
                                           ptr(self.tgt.packed), ctypes.byref(it), B, C, ptr(self.done8), N, mx.S,
                                           mx.Hm, mx.K1, self._mixer_nets(), 2, ptr(self.done8), s),
                  "rec seq + mixer recurrence")
            self._mixer_seq_call(L, L.mm_mixer_fwd_seq_hyper, s, "mixer fwd seq (hypernets)")
            return
        check(L.mm_agent_q_rec_seq2(ctypes.byref(self.beh.dims), ptr(self.beh.packed), ctypes.byref(ib), B,
                                    ptr(self.tgt.packed), ctypes.byref(it), B, C, ptr(self.done8), s), "rec seq")
        if self.has_mixer:
            mx = self.mix
            if split:
                # join the mixer recurrence (side stream), then the hypernet pass over the agents' Q
                if join:
                    torch.cuda.current_stream(self.dev).wait_stream(self._side_stream())
                self._mixer_seq_call(L, L.mm_mixer_fwd_seq_hyper, s, "mixer fwd seq (hypernets)")
                return
            if L.mm_mixer_fwd_seq_fits(B, N, mx.Hm, mx.K1):
                # all C steps of both mixers in ONE launch: weights staged once into LDS, the mixer
                # hidden carried in LDS (bit-identical to the per-step launches below)
                self._mixer_seq_call(L, L.mm_mixer_fwd_seq, s, "mixer fwd seq")
                return
            # per-step mixer launches (B >= 512: 8 samples per block share the weight reads), reading
            # the REC outputs of every step
            for t in range(C):
                nets = (MixNetIO * 2)()
                for k, (Pm, q, off, h, qt, sv, gi) in enumerate(
                        ((self.mix.flat, self.qa[t], self.s_off, self.hm, self.qtot[t], self.msave[t], self.gi_b[t]),
                         (self.tmix.flat, self.maxq[t], self.s2_off, self.hmt, self.qtot_t[t], None, self.gi_t[t]))):
                    n = nets[k]
                    n.P, n.q, n.gi = Pm.data_ptr(), q.data_ptr(), gi.data_ptr()
                    n.s_off = off.data_ptr() + 8 * t * B
                    n.h_in, n.h_out = h[t % 2].data_ptr(), h[(t + 1) % 2].data_ptr()
                    n.reset = self.ones8.data_ptr() if t == 0 else self.done8.data_ptr() + (t - 1) * B
                    n.qtot = qt.data_ptr()
                    n.save = sv.data_ptr() if sv is not None else None
                check(L.mm_mixer_fwd(B, N, mx.S, mx.Hm, mx.K1, obs_p, reset_p, nets, 2, s), "mixer fwd")

    def apply_grads(self, grad_scale=1.0, per=None, sample_next=None):
        """clip_grad_norm_ + Adam (grads scaled first, e.g. 1/world after an all-reduce), then repack
        the behavior fragments for the next forward; with ``per`` also the priority update of the sampled
        chunks (returns True when that update was issued here); with ``sample_next`` = (per, seed, counter) and no
        ``per``, the next update's PER draws in the same launch (its sample_and_grads then runs presampled)."""
        s = stream_handle(self.dev)
        if not self._uses_h3():
            # one launch after the norm's partial sums: the Adam step writes the exact-f32 image from the new values
            # (no pack launch) and one more block updates the priorities (mm_clip_adam_pack)
            two = self.mode == "qmix_min"   # clip agent net and mixer separately (qmix/qmix.py:235-238)
            check(lib().mm_clip_adam_pack(ptr(self.P), ptr(self.Gr), ptr(self.m), ptr(self.v), self.n,
                                          self.n_agent if two else self.n_clip, int(two), self.clip, self.lr, self.b1,
                                          self.b2, self.aeps, ptr(self.step_dev), ptr(self.partials), ptr(self.norm),
                                          float(grad_scale), ctypes.byref(self.beh.dims), ptr(self.beh.packed),
                                          per._h if per is not None else None,
                                          ptr(self.nodes) if per is not None else None,
                                          ptr(self.td_last) if per is not None else None, self.B,
                                          sample_next[0]._h if sample_next else None,
                                          sample_next[1] if sample_next else 0, sample_next[2] if sample_next else 0,
                                          ptr(self.nodes) if sample_next else None,
                                          ptr(self.slots) if sample_next else None,
                                          ptr(self.isw) if sample_next else None, s), "clip_adam_pack")
            self.beh.mark_h3_stale()       # the exact-f32 image is current, the fp16x3 image is not
            self.updates += 1
            return per is not None
        if self.mode == "qmix_min":   # clip agent net and mixer separately (qmix/qmix.py:235-238)
            check(lib().mm_clip2_adam(ptr(self.P), ptr(self.Gr), ptr(self.m), ptr(self.v), self.n, self.n_agent,
                                      self.clip, self.lr, self.b1, self.b2, self.aeps, ptr(self.step_dev),
                                      ptr(self.partials), ptr(self.norm), float(grad_scale), s), "clip2_adam")
        else:
            check(lib().mm_clip_adam(ptr(self.P), ptr(self.Gr), ptr(self.m), ptr(self.v), self.n, self.n_clip,
                                     self.clip, self.lr, self.b1, self.b2, self.aeps, ptr(self.step_dev),
                                     ptr(self.partials), ptr(self.norm), float(grad_scale), s), "clip_adam")
        self.beh.mark_dirty()
        self._pack(self.beh, s)
        self.updates += 1
        return False

    def _uses_h3(self):
        """Whether this learner's own forward reads the fp16x3 image (the opt-in fast PRE)."""
        return self.mixer_fp16 and self.C * self.B >= 2048 and self.fast_pre

    def _pack(self, net, s=None):
        """Repack what the learner's forward reads: the exact-f32 image only, unless the fast PRE runs (the
        rollout's fp16x3 image is then refreshed lazily by its own full pack before the next rollout step)."""
        if self._uses_h3():
            net.pack(s)
        else:
            net.pack_f32(s)

    def train_step(self, obs_base, reset_obs_ptr):
        self.compute_grads(obs_base, reset_obs_ptr)
        self.apply_grads()

    def _outer(self, L, s, U, u_g, u_m, V, v_g, v_m, dW, w_g, db, b_g, M, R, Cc, groups, v_off=None, v_reset=None,
               jobs=None):
        a = OuterArgs()
        a.U, a.u_g, a.u_m = U, u_g, u_m
        a.V, a.v_g, a.v_m = V, v_g, v_m
        a.v_off = v_off
        a.v_reset = v_reset
        a.dW, a.w_g = dW, w_g
        a.db, a.b_g = db, b_g
        a.M, a.R, a.Cc, a.accumulate, a.groups = M, R, Cc, 0, groups
        if jobs is not None:
            jobs.append(a)
        else:
            check(L.mm_outer_reduce(ctypes.byref(a), s), "outer_reduce")

    def _tmv(self, L, s, W, w_g, X, x_g, x_m, Z, z_g, z_m, Y, y_g, y_m, M, R, Cc, groups):
        a = TmvArgs()
        a.W, a.w_g, a.X, a.x_g, a.x_m, a.Z, a.z_g, a.z_m, a.Y, a.y_g, a.y_m = W, w_g, X, x_g, x_m, Z, z_g, z_m, Y, y_g, y_m
        a.M, a.R, a.Cc, a.groups = M, R, Cc, groups
        check(L.mm_tmv(ctypes.byref(a), s), "tmv")

    def _agent_wgrad(self, L, s, obs_p, reset_p, M, jobs):
        N, D, F1, G, H, A, SD = self.N, self.D, self.F1, self.G, self.H, self.A, self.SD
        o = self.beh.offs          # W1 b1 W2 b2 Wih Whh bih bhh Wq bq
        gp, pp = self.Gr.data_ptr(), self.P.data_ptr()
        sv = self.asave.data_ptr()
        f = 4
        # data gradients of the feed-forward layers first (the outer products below only read them)
        # dpre2 = (x2 > 0) * Wih^T dgi ; dpre1 = (x1 > 0) * W2^T dpre2
        if L is not None:
            self._tmv(L, s, pp + f * o[4], 3 * H * G, self.dgi.data_ptr(), 3 * H, N * 3 * H, sv + f * F1, SD,
                      N * SD, self.dpre2.data_ptr(), G, N * G, M, 3 * H, G, N)
            self._tmv(L, s, pp + f * o[2], G * F1, self.dpre2.data_ptr(), G, N * G, sv, SD, N * SD,
                      self.dpre1.data_ptr(), F1, N * F1, M, G, F1, N)
        # Wq, bq <- dq (one-hot) x h_out
        self._outer(L, s, self.dqv.data_ptr(), A, N * A, sv + f * (F1 + G + 5 * H), SD, N * SD,
                    gp + f * o[8], A * H, gp + f * o[9], A, M, A, H, N, jobs=jobs)
        # Whh, bhh <- dgh x h_in
        self._outer(L, s, self.dgh.data_ptr(), 3 * H, N * 3 * H, sv + f * (F1 + G), SD, N * SD,
                    gp + f * o[5], 3 * H * H, gp + f * o[7], 3 * H, M, 3 * H, H, N, jobs=jobs)
        # Wih, bih <- dgi x x2
        self._outer(L, s, self.dgi.data_ptr(), 3 * H, N * 3 * H, sv + f * F1, SD, N * SD,
                    gp + f * o[4], 3 * H * G, gp + f * o[6], 3 * H, M, 3 * H, G, N, jobs=jobs)
        # W2, b2 <- dpre2 x x1
        self._outer(L, s, self.dpre2.data_ptr(), G, N * G, sv, SD, N * SD,
                    gp + f * o[2], G * F1, gp + f * o[3], G, M, G, F1, N, jobs=jobs)
        # W1, b1 <- dpre1 x obs (gathered through the s_t offsets)
        self._outer(L, s, self.dpre1.data_ptr(), F1, N * F1, obs_p.value, D, 0,
                    gp + f * o[0], F1 * D, gp + f * o[1], F1, M, F1, D, N,
                    v_off=self.s_off.data_ptr(), v_reset=reset_p.value, jobs=jobs)

    def _mixer_wgrad(self, L, s, obs_p, reset_p, M, jobs):
        mx = self.mix
        Hm, K1, N, S = mx.Hm, mx.K1, self.N, mx.S
        MSD, MDD = self.MSD, self.MDD
        base = self.Gr.data_ptr() + 4 * self.n_agent
        mo = {k: base + 4 * mx.offs[i] for i, k in enumerate(MIX_KEYS)}
        dl, sv = self.mdelta.data_ptr(), self.msave.data_ptr()
        f = 4
        hm1 = sv + f * 5 * Hm
        # GRU input weights <- dgi x state (gathered), recurrent <- dgh x hm0
        self._outer(L, s, dl, 0, MDD, obs_p.value, 0, 0, mo["gWih"], 0, mo["gbih"], 0, M, 3 * Hm, S, 1,
                    v_off=self.s_off.data_ptr(), v_reset=reset_p.value, jobs=jobs)
        self._outer(L, s, dl + f * 3 * Hm, 0, MDD, sv, 0, MSD, mo["gWhh"], 0, mo["gbhh"], 0, M, 3 * Hm, Hm, 1, jobs=jobs)
        # hypernetworks <- deltas x hm1
        self._outer(L, s, dl + f * 6 * Hm, 0, MDD, hm1, 0, MSD, mo["w1W"], 0, mo["w1b"], 0, M, N * K1, Hm, 1, jobs=jobs)
        self._outer(L, s, dl + f * (6 * Hm + N * K1), 0, MDD, hm1, 0, MSD, mo["b1W"], 0, mo["b1b"], 0, M, K1, Hm, 1, jobs=jobs)
        self._outer(L, s, dl + f * (6 * Hm + N * K1 + K1), 0, MDD, hm1, 0, MSD, mo["w2W"], 0, mo["w2b"], 0, M, K1,
                    Hm, 1, jobs=jobs)
        self._outer(L, s, dl + f * (6 * Hm + N * K1 + 2 * K1), 0, MDD, hm1, 0, MSD, mo["b2aW"], 0, mo["b2ab"], 0, M,
                    K1, Hm, 1, jobs=jobs)
        # final b2 layer <- dQ x relu(b2 hidden)
        self._outer(L, s, dl + f * (6 * Hm + N * K1 + 3 * K1), 0, MDD, sv + f * (6 * Hm + N * K1 + 2 * K1), 0, MSD,
                    mo["b2bW"], 0, mo["b2bb"], 0, M, 1, K1, 1, jobs=jobs)

    # ------------------------------------------------------------------ full update from the PER
    def sample_and_grads(self, per, store, reset_obs_ptr, fracs=None, seed=0, counter=0, presampled=False):
        """PER sample (injected fractions or the device counter RNG) -> gather -> forward/backward (presampled: the
        draws already issued by the previous update's step launch)."""
        L, s = lib(), stream_handle(self.dev)
        if presampled:
            pass
        elif fracs is not None:
            fr = torch.as_tensor(fracs, dtype=torch.float64).to(self.dev).contiguous()
            check(L.mm_per_sample(per._h, self.B, ptr(fr), ptr(self.nodes), ptr(self.slots), ptr(self.isw), s),
                  "per_sample")
        else:
            check(L.mm_per_sample_rng(per._h, self.B, seed, counter, ptr(self.nodes), ptr(self.slots),
                                      ptr(self.isw), s), "per_sample_rng")
        self.gather(per, store)
        self._per_next, self._per_done = per, False
        self.compute_grads(store.obs, reset_obs_ptr)

    def sample_uniform_and_grads(self, per, store, reset_obs_ptr, seed=0, counter=0):
        """Uniform chunk replay (qmix/qmix.py ReplayBuffer.sample_chunk) -> gather -> forward/backward."""
        check(lib().mm_per_sample_uniform(per._h, self.B, seed, counter, ptr(self.slots), ptr(self.isw),
                                          stream_handle(self.dev)), "per_sample_uniform")
        self.gather(per, store)
        self.compute_grads(store.obs, reset_obs_ptr)

    def update_uniform(self, per, store, reset_obs_ptr, seed=0, counter=0, allreduce=None):
        """One qmix/qmix.py train iteration from the device chunk store (no priority update)."""
        self.sample_uniform_and_grads(per, store, reset_obs_ptr, seed, counter)
        scale = 1.0
        if allreduce is not None:
            scale = 1.0 / allreduce(self.Gr)
        self.apply_grads(scale)

    def apply_and_reprioritize(self, per, grad_scale=1.0, sample_next=None):
        """Returns True when the next update's draws (``sample_next`` = (seed, counter)) were issued with the step."""
        if self._per_done:              # issued with the hypernet backward (compute_grads)
            self._per_done = False
            ahead = sample_next is not None and not self._uses_h3()
            self.apply_grads(grad_scale, sample_next=(per,) + tuple(sample_next) if ahead else None)
            return ahead
        if self.apply_grads(grad_scale, per=per):
            return False
        check(lib().mm_per_update(per._h, ptr(self.nodes), ptr(self.td_last), self.B, stream_handle(self.dev)),
              "per_update")
        return False

    def update(self, per, store, reset_obs_ptr, fracs=None, seed=0, counter=0, allreduce=None):
        """One reference update iteration: sample -> gather -> grads [-> all-reduce] -> clip/Adam ->
        priority update. ``allreduce(G)`` sums the flat gradient over ranks (RCCL); grads are then
        averaged by 1/world inside the clip/Adam kernel."""
        self.sample_and_grads(per, store, reset_obs_ptr, fracs, seed, counter)
        scale = 1.0
        if allreduce is not None:
            scale = 1.0 / allreduce(self.Gr)
        self.apply_and_reprioritize(per, scale)

    # ------------------------------------------------------------------ HIP graph of an update
    def capture_update(self, per, store, reset_obs_ptr, seed=0, per_replay=1):
        """Capture [sample -> gather -> fwd/bwd] and [clip/Adam -> repack -> reprioritize] as two HIP
        graphs (the RCCL all-reduce, when used, runs between them eagerly; its 1/world scale is baked
        into the second graph from ``_graph_scale``). ``per=None`` captures the update of the batch
        placed by ``load_batch`` instead (no sampling, no priority update). ``per_replay`` > 1 also captures that
        many consecutive single-replica updates as one graph (``replay_updates``: the trainer's update_iter
        updates after an episode, Train_dqn.train called update_iter times, qmix/main.py:240-250)."""
        self._pack(self.beh)
        self._pack(self.tgt)
        self._push_double_eps()
        torch.cuda.synchronize(self.dev)
        n0 = self.updates
        g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with graph_capture(g1):
            if per is None:          # the batch loaded by load_batch (tests, reference-shaped callers)
                self.compute_grads(self._obs_ptr, self._reset_obs)
            else:
                self.sample_and_grads(per, store, reset_obs_ptr, seed=seed)
        with graph_capture(g2):
            if per is None:
                self.apply_grads(self._graph_scale)
            else:
                self.apply_and_reprioritize(per, self._graph_scale)
        # single-replica updates replay ONE graph holding both parts (one graph launch per update
        # instead of two: the B = 32 update is launch-latency bound)
        g12 = torch.cuda.CUDAGraph()
        with graph_capture(g12):
            if per is None:
                self.compute_grads(self._obs_ptr, self._reset_obs)
                self.apply_grads(self._graph_scale)
            else:
                self.sample_and_grads(per, store, reset_obs_ptr, seed=seed)
                self.apply_and_reprioritize(per, self._graph_scale)
        self.graph_multi, self._per_replay = None, int(per_replay)
        if self._per_replay > 1:
            gk = torch.cuda.CUDAGraph()
            with graph_capture(gk):
                ahead = False   # each update's step launch also draws the next update's batch
                for i in range(self._per_replay):
                    if per is None:
                        self.compute_grads(self._obs_ptr, self._reset_obs)
                        self.apply_grads(self._graph_scale)
                    else:
                        self.sample_and_grads(per, store, reset_obs_ptr, seed=seed, presampled=ahead)
                        ahead = self.apply_and_reprioritize(per, self._graph_scale,
                                                            sample_next=(seed, 0) if i + 1 < self._per_replay else None)
            self.graph_multi = gk
        self.updates = n0
        self.graphs = (g1, g2)
        self.graph_fused = g12
        return self.graphs

    _graph_scale = 1.0
    graph_multi, _per_replay = None, 1

    def replay_updates(self, n, allreduce=None):
        """``n`` consecutive updates: single-replica ones as replays of the captured ``per_replay``-update graph
        (one graph launch per ``per_replay`` updates: the B = 32 update is launch-latency bound), the rest (and every
        update with an all-reduce between its halves) one by one."""
        k = self._per_replay
        if allreduce is None and self.graph_multi is not None and n >= k:
            self._pack(self.tgt)
            self._pack(self.beh)
            self._push_double_eps()
            while n >= k:
                self.graph_multi.replay()
                self.updates += k
                n -= k
            if not self._uses_h3():
                self.beh.mark_h3_stale()
        for _ in range(n):
            self.replay_update(allreduce)

    def replay_update(self, allreduce=None):
        g1, g2 = self.graphs
        self._pack(self.tgt)            # target synced since capture: repack eagerly (no-op otherwise)
        self._pack(self.beh)
        self._push_double_eps()
        if allreduce is None and getattr(self, "graph_fused", None) is not None:
            self.graph_fused.replay()
        else:
            g1.replay()
            if allreduce is not None:
                allreduce(self.Gr)      # the 1/world scale was baked at capture (set _graph_scale first)
            g2.replay()
        if not self._uses_h3():
            self.beh.mark_h3_stale()    # the graph refreshed the f32 image only
        self.updates += 1

    # ------------------------------------------------------------------ checkpoint (minimarl.checkpoint)
    def release(self):
        """Hand the nets their parameters back as standalone tensors (copies of the current values) and
        drop the ownership marks, so another QLearner can take them; returns the Adam state (m, v, step)
        for a successor over the same nets."""
        torch.cuda.synchronize(self.dev)
        self.beh.flat = self.P[:self.n_agent].clone()
        self.beh._owner = None
        self.beh.mark_dirty()
        if self.mix is not None:
            self.mix.flat = self.P[self.n_agent:].clone()
            self.mix._owner = None
        return self.m.clone(), self.v.clone(), self.step_dev.clone(), self.updates

    def adopt_adam(self, state):
        """Continue from a predecessor's Adam state over the same parameter layout (``release``)."""
        m, v, step, updates = state
        assert m.numel() == self.n, "adopt_adam: parameter layout differs"
        self.m.copy_(m)
        self.v.copy_(v)
        self.step_dev.copy_(step)
        self.updates = int(updates)

    def checkpoint_tensors(self):
        ts = {"P": self.P, "m": self.m, "v": self.v, "step": self.step_dev, "target": self.tgt.flat}
        if self.tmix is not None:
            ts["target_mixer"] = self.tmix.flat
        return ts, {"updates": int(self.updates), "mode": self.mode}

    def restore_tensors(self, ts, scalars):
        from .checkpoint import copy_into
        for k, dst in (("P", self.P), ("m", self.m), ("v", self.v), ("step", self.step_dev),
                       ("target", self.tgt.flat)):
            copy_into(dst, ts[k], k)
        if self.tmix is not None:
            copy_into(self.tmix.flat, ts["target_mixer"], "target_mixer")
        self.beh.mark_dirty()
        self.tgt.mark_dirty()
        self.updates = int(scalars.get("updates", 0))
        if self.double:
            self.dctr.copy_(torch.arange(self.C, dtype=torch.int64) + (self.updates - 1) * self.C)

    def sync_target(self, mixer=False):
        """target <- behavior (qmix/main.py:255-256 syncs the agent net only; mixer=True also the mixer)."""
        self.tgt.copy_from(self.beh)
        if mixer and self.mix is not None:
            self.tmix.flat.copy_(self.mix.flat)
