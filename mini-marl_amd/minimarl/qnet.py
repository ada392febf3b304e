"""Per-agent Q-network on the MI355X: flat fp32 parameters in HBM + the fused HIP forward.

Mirrors the reference's ``Q_Net`` (qmix/_network.py:5-77, vdn/_network.py:61-91):
N agents with their OWN weights, Linear(D,F1)+ReLU, Linear(F1,G)+ReLU,
GRUCell(G,H), Linear(H,A). The forward is one ``mm_agent_q_fwd`` launch for all
envs x agents (see csrc/agent_fwd.hip).
"""
import contextlib
import ctypes
import gc
import math

import numpy as np
import torch

from ._lib import (MM_Q_ACT, MM_Q_GATHER, MM_Q_MAX, MM_Q_NONE, QFwdIO, QnetDims, c_i64, check, lib)

KEYS = ["W1", "b1", "W2", "b2", "Wih", "Whh", "bih", "bhh", "Wq", "bq"]

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

# minimal QMIX QNet naming (qmix/qmix.py:102-131)
_MIN_FMT = {
    "W1": "agent_feature_{i}.0.weight", "b1": "agent_feature_{i}.0.bias",
    "W2": "agent_feature_{i}.2.weight", "b2": "agent_feature_{i}.2.bias",
    "Wih": "agent_gru_{i}.weight_ih", "Whh": "agent_gru_{i}.weight_hh",
    "bih": "agent_gru_{i}.bias_ih", "bhh": "agent_gru_{i}.bias_hh",
    "Wq": "agent_q_{i}.weight", "bq": "agent_q_{i}.bias",
}
_FMTS = {"qmix": _QMIX_FMT, "vdn": _VDN_FMT, "min": _MIN_FMT}


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


@contextlib.contextmanager
def graph_capture(g):
    """``torch.cuda.graph(g)`` with the garbage collector held off: a collection inside the capture can
    destroy an earlier graph or native handle, whose device calls are illegal mid-capture (abort)."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(g):
            yield
    finally:
        if was:
            gc.enable()


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class AgentQNet:
    """Device-resident parameters of N per-agent Q-networks + their MFMA fragment image."""

    def __init__(self, n_agents, obs_dim, n_actions, f1=64, g=32, h=32, device="cuda", seed=None, flat=None):
        self.N, self.D, self.A, self.F1, self.G, self.H = n_agents, obs_dim, n_actions, f1, g, h
        self.device = torch.device(device)
        self.dims = QnetDims(n_agents, obs_dim, f1, g, h, n_actions)
        offs = (c_i64 * 11)()
        check(lib().mm_qnet_param_offsets(ctypes.byref(self.dims), offs), "qnet_param_offsets")
        self.offs = list(offs)
        self.n_params = self.offs[10]
        if flat is not None:          # a view into a larger buffer (e.g. the learner's [agent | mixer] params)
            assert flat.numel() == self.n_params and flat.is_contiguous() and flat.dtype == torch.float32
            self.flat = flat
        else:
            self.flat = torch.zeros(self.n_params, dtype=torch.float32, device=self.device)
        n_packed = lib().mm_qnet_packed_count(ctypes.byref(self.dims))
        if n_packed < 0:
            check(-22, "qnet_packed_count")
        self.packed = torch.zeros(n_packed, dtype=torch.float32, device=self.device)
        self._dirty = True
        self._h3_stale = False      # exact-f32 image current, fp16x3 image + flags not (pack_f32)
        if seed is not None:
            self.init_default(seed)

    # ------------------------------------------------------------------ parameters
    def shapes(self):
        N, D, F1, G, H, A = self.N, self.D, self.F1, self.G, self.H, self.A
        return {"W1": (N, F1, D), "b1": (N, F1), "W2": (N, G, F1), "b2": (N, G), "Wih": (N, 3 * H, G),
                "Whh": (N, 3 * H, H), "bih": (N, 3 * H), "bhh": (N, 3 * H), "Wq": (N, A, H), "bq": (N, A)}

    def view(self, key, t=None):
        t = self.flat if t is None else t
        i = KEYS.index(key)
        return t[self.offs[i]:self.offs[i + 1]].view(self.shapes()[key])

    def params(self):
        return {k: self.view(k) for k in KEYS}

    def mark_dirty(self):
        self._dirty = True

    def init_default(self, seed):
        """PyTorch default init (Linear: U(+-1/sqrt(fan_in)), GRUCell: U(+-1/sqrt(H))), generated on the host."""
        g = torch.Generator().manual_seed(int(seed))
        fan = {"W1": self.D, "b1": self.D, "W2": self.F1, "b2": self.F1, "Wih": self.H, "Whh": self.H,
               "bih": self.H, "bhh": self.H, "Wq": self.H, "bq": self.H}
        host = torch.empty(self.n_params)
        for k in KEYS:
            b = 1.0 / math.sqrt(fan[k])
            i = KEYS.index(k)
            host[self.offs[i]:self.offs[i + 1]] = (torch.rand(self.offs[i + 1] - self.offs[i], generator=g) * 2 - 1) * b
        self.flat.copy_(host.to(self.device))
        self.mark_dirty()

    def load_reference_state(self, sd, prefix="", style="qmix"):
        """Load a reference Q_Net / QNet state_dict (dict name -> array/tensor); style "qmix"
        (qmix/_network.py), "vdn" (vdn/_network.py) or "min" (qmix/qmix.py)."""
        fmt = _FMTS[style]
        host = torch.empty(self.n_params)
        for k in KEYS:
            parts = [torch.as_tensor(np.asarray(sd[prefix + fmt[k].format(i=i)]), dtype=torch.float32)
                     for i in range(self.N)]
            i = KEYS.index(k)
            host[self.offs[i]:self.offs[i + 1]] = torch.stack(parts).reshape(-1)
        self.flat.copy_(host.to(self.device))
        self.mark_dirty()

    def state_dict(self, style="qmix"):
        fmt = _FMTS[style]
        host = self.flat.detach().cpu()
        out = {}
        for k in KEYS:
            v = self.view(k, host)
            for i in range(self.N):
                out[fmt[k].format(i=i)] = v[i].clone()
        return out

    def copy_from(self, other):
        self.flat.copy_(other.flat)
        self.mark_dirty()

    def pack(self, stream=None):
        """Both fragment images (exact f32 and fp16x3) + the fp16x3 range flags, when the params changed."""
        if self._dirty or self._h3_stale:
            check(lib().mm_qnet_pack(ctypes.byref(self.dims), ptr(self.flat), ptr(self.packed),
                                     stream or stream_handle(self.device)), "qnet_pack")
            self._dirty = self._h3_stale = False

    def pack_f32(self, stream=None):
        """Only the exact-f32 image (the learner's own forward after an Adam step); the fp16x3 image is then
        repacked by the next ``pack`` (the rollout's, before its next large-E forward)."""
        if self._dirty:
            check(lib().mm_qnet_pack_f32(ctypes.byref(self.dims), ptr(self.flat), ptr(self.packed),
                                         stream or stream_handle(self.device)), "qnet_pack_f32")
            self._dirty, self._h3_stale = False, True

    def mark_h3_stale(self):
        """The exact-f32 image was refreshed by a replayed graph (pack_f32 captured): only the fp16x3 image is old."""
        self._dirty, self._h3_stale = False, True

    # ------------------------------------------------------------------ forward
    def forward_io(self, n_envs, io, stream=None):
        self.pack(stream)
        check(lib().mm_agent_q_fwd(ctypes.byref(self.dims), ptr(self.packed), ctypes.byref(io), int(n_envs),
                                   stream or stream_handle(self.device)), "agent_q_fwd")

    def make_io(self, obs, hidden, h_out=None, q_out=None, mode=MM_Q_NONE, reset=None):
        """io for contiguous obs [E,N,D] and hidden [E,N,H] (any strides on hidden)."""
        io = QFwdIO()
        io.obs = obs.data_ptr()
        io.obs_se, io.obs_sa = obs.stride(0), obs.stride(1)
        assert obs.stride(2) == 1, "obs feature stride must be 1"
        io.h_in = hidden.data_ptr()
        io.hin_se, io.hin_sa, io.hin_sf = hidden.stride()
        if h_out is not None:
            io.h_out = h_out.data_ptr()
            io.hout_se, io.hout_sa, io.hout_sf = h_out.stride()
        if q_out is not None:
            assert q_out.stride(2) == 1
            io.q_out = q_out.data_ptr()
            io.q_se, io.q_sa = q_out.stride(0), q_out.stride(1)
        if reset is not None:
            io.reset = reset.data_ptr()
        io.mode = mode
        return io

    def _check_in(self, obs, hidden):
        E = obs.shape[0]
        assert obs.shape == (E, self.N, self.D), f"obs shape {tuple(obs.shape)} != (E,{self.N},{self.D})"
        assert hidden.shape == (E, self.N, self.H), f"hidden shape {tuple(hidden.shape)}"
        assert obs.dtype == torch.float32 and hidden.dtype == torch.float32
        assert obs.is_cuda and hidden.is_cuda
        return E

    @torch.no_grad()
    def forward(self, obs, hidden):
        """q [E,N,A], next_hidden [E,N,H] (qmix/_network.py:44-64)."""
        obs = obs.contiguous()
        E = self._check_in(obs, hidden)
        q = torch.empty(E, self.N, self.A, device=self.device)
        h2 = torch.empty(E, self.N, self.H, device=self.device)
        self.forward_io(E, self.make_io(obs, hidden, h2, q, MM_Q_NONE))
        return q, h2

    @torch.no_grad()
    def act(self, obs, hidden, epsilon, u=None, rand_actions=None, seed=0, counter=0, reset=None):
        """Fused forward + epsilon-greedy: (action int32 [E,N], q_taken [E,N], next_hidden, q)."""
        obs = obs.contiguous()
        E = self._check_in(obs, hidden)
        q = torch.empty(E, self.N, self.A, device=self.device)
        h2 = torch.empty(E, self.N, self.H, device=self.device)
        act = torch.empty(E, self.N, dtype=torch.int32, device=self.device)
        qsel = torch.empty(E, self.N, device=self.device)
        io = self.make_io(obs, hidden, h2, q, MM_Q_ACT, reset)
        io.epsilon = float(epsilon)
        if u is not None:
            u = u.to(self.device, torch.float32).contiguous()
            ra = rand_actions.to(self.device, torch.int32).contiguous()
            io.u, io.rand_act = u.data_ptr(), ra.data_ptr()
        io.seed, io.counter = int(seed), int(counter)
        io.act_out, io.qsel_out = act.data_ptr(), qsel.data_ptr()
        self.forward_io(E, io)
        return act, qsel, h2, q

    @torch.no_grad()
    def max_q(self, obs, hidden):
        obs = obs.contiguous()
        E = self._check_in(obs, hidden)
        h2 = torch.empty(E, self.N, self.H, device=self.device)
        qmax = torch.empty(E, self.N, device=self.device)
        io = self.make_io(obs, hidden, h2, None, MM_Q_MAX)
        io.qsel_out = qmax.data_ptr()
        self.forward_io(E, io)
        return qmax, h2


class _Space:
    def __init__(self, shape=None, n=None):
        self.shape = shape
        self.n = n


class Q_Net:
    """Drop-in for the reference ``Q_Net(observation_space, action_space, args)``
    (qmix/_network.py:5-77; vdn/_network.py:61-91) backed by the HIP forward.

    Differences by design: tensors stay on the GPU (the reference's ``.to("cpu")``
    of q at qmix/_network.py:64 is the per-step host copy this engine removes).
    ``sample_action`` consumes the torch CPU RNG exactly like the reference
    (``torch.rand(B)`` then ``torch.randint``), so equal seeds give equal actions.
    """

    def __init__(self, observation_space, action_space, args=None, f1=64, g=32, h=32, device="cuda"):
        if args is not None and not getattr(args, "use_recurrent", True):
            raise NotImplementedError("use_recurrent=False is not supported by the fused kernel")
        self.num_agents = len(observation_space)
        self.obs_dim = observation_space[0].shape[0]
        self.n_actions = action_space[0].n
        self.gru_hidden_size = h
        self.net = AgentQNet(self.num_agents, self.obs_dim, self.n_actions, f1, g, h, device)

    def load_state_dict(self, state_dict, style="qmix"):
        if isinstance(state_dict, Q_Net):
            self.net.copy_from(state_dict.net)
        else:
            self.net.load_reference_state({k: v.cpu().numpy() if torch.is_tensor(v) else v
                                           for k, v in state_dict.items()}, style=style)

    def state_dict(self, style="qmix"):
        return self.net.state_dict(style)

    def _dev(self, x):
        return torch.as_tensor(x, dtype=torch.float32).to(self.net.device)

    def __call__(self, obs, hidden):
        return self.forward(obs, hidden)

    def _packed(self):
        """The fragment image, repacked by the ``minimarl::qnet_pack`` op when the params changed — or when only
        the exact-f32 image is current (``_h3_stale``: a learner update ran ``pack_f32``), since a large-batch
        forward reads the fp16x3 image and its range flags (qnet_pack writes all three)."""
        from .ops import dims, load
        if self.net._dirty or self.net._h3_stale:
            load().qnet_pack(self.net.flat, dims(self.net), self.net.packed)
            self.net._dirty = self.net._h3_stale = False
        return self.net.packed

    def forward(self, obs, hidden):
        """q [B,N,A], next hidden [B,N,H] through ``torch.ops.minimarl.agent_q_fwd``."""
        from .ops import dims, load
        obs, hidden = self._dev(obs).contiguous(), self._dev(hidden)
        B, N = obs.shape[0], self.num_agents
        q = torch.empty(B, N, self.n_actions, device=self.net.device)
        h2 = torch.empty(B, N, self.gru_hidden_size, device=self.net.device)
        load().agent_q_fwd(self._packed(), dims(self.net), obs, hidden, h2, q)
        return q, h2

    def sample_action(self, obs, hidden, epsilon):
        """qmix/_network.py:66-74 through ``torch.ops.minimarl.agent_q_act``: the row mask and random
        actions come from the torch CPU RNG in the reference's order, so equal seeds give equal actions."""
        from .ops import dims, load
        obs, hidden = self._dev(obs).contiguous(), self._dev(hidden)
        B, N = obs.shape[0], self.num_agents
        u = torch.rand(size=(B,))                        # qmix/_network.py:68
        mask = u <= epsilon
        ra = torch.zeros(B, N, dtype=torch.int32)
        ra[mask] = torch.randint(low=0, high=self.n_actions, size=(int(mask.sum()), N)).int()
        dev = self.net.device
        act = torch.empty(B, N, dtype=torch.int32, device=dev)
        qsel = torch.empty(B, N, device=dev)
        h2 = torch.empty(B, N, self.gru_hidden_size, device=dev)
        q = torch.empty(B, N, self.n_actions, device=dev)
        load().agent_q_act(self._packed(), dims(self.net), obs, hidden, float(epsilon), u.to(dev), ra.to(dev), 0, 0,
                           h2, act, qsel, q)
        return act.float(), h2, q

    def init_hidden(self, batch_size=1):
        return torch.zeros((batch_size, self.num_agents, self.gru_hidden_size), device=self.net.device)
