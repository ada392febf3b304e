"""Device-resident rollout engine: E lockstep envs x N agents, chunked into the PER store.

Replaces the reference runners' per-step loop (vdn/main.py:80-171,
qmix/main.py:100-237): for every env at every step

  1. behavior Q_Net forward + epsilon-greedy      (sample_action, qmix/_network.py:66-74)
  2. env step (terminal next obs into the chunk store, auto-reset current obs)
  3. target Q_Net forward on the next obs -> max_a (qmix/main.py:191-193)
  4. rollout TD error accumulated into the chunk priority, transition stored
     (cal_td_error + chunk lists, qmix/_utils.py:86-97, qmix/main.py:204-233)
  5. every C steps: the E finished chunks go into the prioritized replay at once

ONE launch per step where the fused rollout step applies (``fused``: the restated Checkers env, local obs,
E >= 2048; mm_rollout_step): the env step of step t, the target fwd of step t and the behavior fwd of
step t+1 in one kernel, the TD/store of step t-1 folded into it; the env state, RNG counter, rewards and
max Q' alternate by step parity and the behavior outputs rotate through 3 buffers (so the graph cycle is
lcm(C, 6) steps). Otherwise two launches per step: env(t) — fused with the TD/store of step t-1 inside
a chunk, with the chunk-start copy of the current obs into the new staging rows at a chunk's first
step — and the target fwd of step t fused with the behavior fwd of step t+1. The chunk's last step adds
the PER insert (its first launch also running that step's TD/store). All stream-ordered on one HIP
stream, no host sync; a chunk of steps is captured once as a HIP graph and replayed. The store/TD of
the last executed step therefore lands with the next step (``flush_td()`` writes it now).
Hidden states reset at episode ends (the reference re-inits them per episode,
vdn/main.py:137-138); chunks span episode boundaries like the reference's
global ``count_step`` (vdn/main.py:151-167).

Chunk store row layout (one chunk per row, ``rows = capacity + E``):
  obs  [rows, C+1, N, D] f32   slot 0 = s_0, slot t+1 = s'_t (terminal obs at episode ends)
  act  [rows, C, N] u8, rew [rows, C, N] f32, done [rows, C] u8
s_t for t >= 1 is s'_{t-1} unless done_{t-1} (then the reset obs). The PER maps
slot -> row; inserts swap the finished staging rows in and take the evicted
rows back as the next staging rows (no chunk copy).
"""
import ctypes
import math

import torch

from ._lib import MM_Q_ACT, MM_Q_MAX, QFwdIO, RollChunkIO, RollStepIO, check, lib
from .env import make_env
from .qnet import AgentQNet, graph_capture, ptr, stream_handle
from .replay import DevicePER


class ChunkStore:
    def __init__(self, rows, chunk, n_agents, obs_dim, device):
        self.rows, self.C, self.N, self.D = rows, chunk, n_agents, obs_dim
        self.obs = torch.zeros(rows, chunk + 1, n_agents, obs_dim, device=device)
        self.act = torch.zeros(rows, chunk, n_agents, dtype=torch.uint8, device=device)
        self.rew = torch.zeros(rows, chunk, n_agents, device=device)
        self.done = torch.zeros(rows, chunk, dtype=torch.uint8, device=device)
        self.row_stride = (chunk + 1) * n_agents * obs_dim

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in (self.obs, self.act, self.rew, self.done))


class RolloutEngine:
    def __init__(self, n_envs, n_agents, obs_dim=None, n_actions=5, f1=64, g=32, h=32, chunk=10,
                 capacity=None, gamma=0.99, max_steps=100, step_cost=-0.01, full_observable=False,
                 per_flavor="qmix", per_kwargs=None, seed=0, env="checkers", fused=None, persistent=None,
                 device="cuda"):
        self.device = torch.device(device)
        self.E, self.N, self.C = int(n_envs), int(n_agents), int(chunk)
        self.gamma = float(gamma)
        self.env_kind = env
        self.env = make_env(env, self.E, self.N, max_steps, step_cost, full_observable, device=self.device)
        self.D = self.env.obs_dim
        assert obs_dim is None or obs_dim == self.D
        self.A = n_actions
        self.behavior = AgentQNet(self.N, self.D, self.A, f1, g, h, self.device, seed=seed)
        self.target = AgentQNet(self.N, self.D, self.A, f1, g, h, self.device)
        self.target.copy_from(self.behavior)
        self.H = h
        self.capacity = int(capacity or 4 * self.E)
        self.per = DevicePER(self.capacity, per_flavor, device=self.device, **(per_kwargs or {}))
        # S staging row sets [S][E] (every mode allocates them, so the store has the same rows in every mode and a
        # checkpoint moves between modes): the chunk-persistent launches write chunk k into set k % S, so ONE launch
        # can run up to S - 1 whole chunks (plus the partial ones at its ends) with the chunks' PER inserts after it;
        # the other modes use set 0
        self.S = self.N_STAGING_SETS
        self.store = ChunkStore(self.capacity + self.S * self.E, self.C, self.N, self.D, self.device)
        self.staging_all = torch.arange(self.capacity, self.capacity + self.S * self.E, dtype=torch.int64,
                                        device=self.device).view(self.S, self.E)
        E, N, D, H = self.E, self.N, self.D, self.H
        dev = self.device
        ok = env == "checkers" and lib().mm_rollout_step_supported(self.env.handle(), ctypes.byref(self.behavior.dims),
                                                                    E) != 0
        okc = env == "checkers" and lib().mm_rollout_chunk_supported(self.env.handle(),
                                                                      ctypes.byref(self.behavior.dims), E) != 0
        if fused and not ok:
            raise ValueError("RolloutEngine(fused=True): the fused rollout step does not support this configuration")
        if persistent and not okc:
            raise ValueError("RolloutEngine(persistent=True): the chunk-persistent rollout does not support this "
                             "configuration (or the grid does not fit the device's CUs)")
        # step modes: "chunk" (chunk-persistent launches, mm_rollout_chunk: the default where it fits), "fused" (one
        # launch per step, mm_rollout_step; fused=True asks for it explicitly), "two-launch" (fused=False)
        self.chunked = bool(persistent) if persistent is not None else (okc and fused is None)
        self.fused = False if self.chunked else (ok if fused is None else bool(fused))
        nb = 3 if self.fused else 2
        if self.fused:
            self.env.state_buffer = lambda: self.t % 2
        # current obs s_{t+1} is never materialised: it is slot c+1 of row cur_row[e] of the chunk
        # store (the env's terminal next obs), or the env's reset obs where cur_row[e] = -1
        self.cur_row = torch.full((E,), -1, dtype=torch.int64, device=dev)
        self.init_obs = torch.empty(E, N, D, device=dev)
        # hidden states feature-major [N, H, E] (env fastest): the forward's lane = env, so every
        # hidden load / store of a wave is one coalesced 128-byte run per feature row
        # hidden states [N][H][E] (env-contiguous: a wave's 16 envs of one feature are 64 contiguous bytes; the chunk
        # kernel reads / writes them with buffer ops at SGPR feature offsets)
        self.h = torch.zeros(N, H, E, device=dev)
        self.ht = torch.zeros(N, H, E, device=dev)
        # ping-pong buffers indexed by step parity: done_t in slot t % 2; act_t, q_taken_t in slot t % nb (nb = 3
        # in the fused mode, whose launch writes step t+1's actions while it reads step t-1's); the fused mode
        # also alternates rew_t / max Q'_t (slot t % 2), the other mode uses slot 0 only
        self.done_buf = [torch.zeros(E, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.act_buf = [torch.zeros(E, N, dtype=torch.int32, device=dev) for _ in range(nb)]
        self.qsel_buf = [torch.zeros(E, N, device=dev) for _ in range(nb)]
        self.maxq_buf = [torch.zeros(E, N, device=dev) for _ in range(2)]
        self.rew_buf = [torch.zeros(E, N, device=dev) for _ in range(2)]
        self.maxq, self.rew = self.maxq_buf[0], self.rew_buf[0]
        self.chunk_td = torch.zeros(E, device=dev)
        # sticky device error bits of the rollout kernels (bit 0: a staging row outside the chunk store was skipped;
        # bit 1: a chunk-persistent launch timed out waiting for a hand-off); polled by check_errors()
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.eps_dev = torch.zeros(1, device=dev)
        # rollout step counter (RNG stream); the fused mode double-buffers it (slot t % 2 is read at step t)
        self.counter_dev = torch.zeros(2, dtype=torch.int64, device=dev)
        self._eps_host = None
        self._primed = False
        self._td_pending = False     # last step's TD/store not yet written (fused into the next env step)
        self._td_flushed = False
        self.graph = None
        self._region_graphs = {}
        self.t = 0
        self.seed = int(seed)
        self.chunks_inserted = 0
        if self.chunked:
            C, T = self.C, (E + 255) // 256
            # per-step rings of RL = S C steps: act / Q(a) of step t at [t % RL] (written one step ahead by the
            # previous step's behavior forward), max Q', rewards, dones of step t at [t % RL]; a launch runs at most
            # (S - 1) C steps, so its rings never overwrite a step its chunks' folds still read
            self.RL = RL = self.S * C
            self.act_r = torch.zeros(RL, E, N, dtype=torch.int32, device=dev)
            self.qsel_r = torch.zeros(RL, E, N, device=dev)
            self.maxq_r = torch.zeros(RL, E, N, device=dev)
            self.rew_r = torch.zeros(RL, E, N, device=dev)
            self.done_r = torch.zeros(RL, E, dtype=torch.uint8, device=dev)
            # launch state owned by the chunk kernel: launch sequence, env state buffer, arrival ticket
            self.ctl = torch.zeros(3, dtype=torch.int64, device=dev)
            # tagged hand-off words [T][RL][N][32] (slot = launch step): (launch sequence + 1) << 32 | 8 envs' actions
            self.hx = torch.zeros(T * RL * N * 32, dtype=torch.int64, device=dev)
            self.env.state_buffer = lambda: int(self.ctl[1].item()) & 1
        self._build_io()
        self.env.reset(self.init_obs)

    N_STAGING_SETS = 4

    @property
    def staging(self):
        """[E] staging rows of the current chunk (chunk mode: set (t // C) % S; the other modes: set 0)."""
        return self.staging_all[(self.t // self.C) % self.S] if self.chunked else self.staging_all[0]

    def staging_set(self, t=None):
        """index of the staging set chunk t // C writes"""
        t = self.t if t is None else t
        return (t // self.C) % self.S if self.chunked else 0

    @property
    def step_mode(self):
        """"chunk" (mm_rollout_chunk), "fused" (mm_rollout_step) or "two-launch" (env launch + dual forward)."""
        return "chunk" if self.chunked else ("fused" if self.fused else "two-launch")

    def _carry_views(self):
        """The mode-specific buffers holding the step state every mode shares at a chunk boundary t (no TD pending):
        act / Q(a) of step t (written one step ahead), done of step t - 1, the RNG step counter read at step t."""
        t, C = self.t, self.C
        if self.chunked:
            i = self._act_idx(t)
            return self.act_r[i], self.qsel_r[i], self.done_r[(t - 1) % self.RL], self.counter_dev[0:1]
        nb = len(self.act_buf)
        ctr = self.counter_dev[t % 2:t % 2 + 1] if self.fused else self.counter_dev[0:1]
        return self.act_buf[t % nb], self.qsel_buf[t % nb], self.done_buf[(t - 1) % 2], ctr

    def carry_state(self):
        """Mode-independent step state (name -> tensor) at a chunk boundary: with the common buffers of
        state_buffers() it lets a checkpoint written in one step mode resume in another (the modes are bit-identical
        step for step, tests/test_gpu_chunk.py). None mid-chunk, where each mode holds the chunk's steps in its own
        rings / pending TD."""
        if self.t % self.C != 0 or self._td_pending:
            return None
        act, qsel, done_prev, ctr = self._carry_views()
        return {"act": act, "qsel": qsel, "done_prev": done_prev, "counter": ctr}

    def load_carry(self, carry, copy, staging_all, src_set):
        """Inverse of carry_state() (``copy(dst, src, name)``); the engine's step count must already be restored.
        ``staging_all`` = the saved staging sets, whose set ``src_set`` is the current chunk's in the saved mode: the
        sets are rotated so it lands where this mode reads it (every other set holds free rows in every mode)."""
        assert self.t % self.C == 0
        for name, dst in zip(("act", "qsel", "done_prev", "counter"), self._carry_views()):
            copy(dst, carry[name], "carry/" + name)
        copy(self.staging_all, torch.roll(staging_all, self.staging_set() - src_set, 0), "staging_all")
        self._td_pending = self._td_flushed = False

    COMMON_STATE = ("cur_row", "init_obs", "h", "ht", "chunk_td", "eps_dev", "staging_all")

    def state_buffers(self):
        """The per-step device buffers a checkpoint must carry (name -> tensor)."""
        out = {k: getattr(self, k) for k in self.COMMON_STATE}
        out.update(counter_dev=self.counter_dev)
        if self.chunked:   # (the launch sequence / hand-off flags are the engine's own, never restored)
            out.update({k: getattr(self, k) for k in ("act_r", "qsel_r", "maxq_r", "rew_r", "done_r")})
            return out
        for k in range(2):
            out[f"done_buf{k}"] = self.done_buf[k]
            out[f"maxq_buf{k}"] = self.maxq_buf[k]
            out[f"rew_buf{k}"] = self.rew_buf[k]
        for k in range(len(self.act_buf)):
            out[f"act_buf{k}"] = self.act_buf[k]
            out[f"qsel_buf{k}"] = self.qsel_buf[k]
        return out

    @property
    def last_rew(self):
        """rewards [E, N] of the last executed step"""
        if self.chunked:
            return self.rew_r[(self.t - 1) % self.RL]
        return self.rew_buf[(self.t - 1) % 2] if self.fused else self.rew

    @property
    def last_done(self):
        """done flags [E] of the last executed step"""
        if self.chunked:
            return self.done_r[(self.t - 1) % self.RL]
        return self.done_buf[(self.t - 1) % 2]

    def _act_idx(self, t):
        """chunk mode: ring index of the actions / Q(a) (and rewards, dones, max Q') of step t"""
        return t % self.RL

    def current_obs(self):
        """s_{t+1} [E,N,D] as the next behavior forward reads it (materialised for tests only)."""
        c = (self.t - 1) % self.C + 1 if self.t > 0 else 0
        out = self.init_obs.clone()
        valid = self.cur_row >= 0
        out[valid] = self.store.obs[self.cur_row[valid], c]
        return out

    @property
    def act(self):
        """actions [E, N] of the last executed step"""
        if self.chunked:
            return self.act_r[self._act_idx(max(self.t - 1, 0))]
        return self.act_buf[(self.t - 1) % len(self.act_buf)] if self.t > 0 else self.act_buf[0]

    def _io_behavior(self, k):
        """behavior fwd writing slot k (acts for step t with t % 2 == k); reset = done_{t-1}."""
        E, N, D, H = self.E, self.N, self.D, self.H
        b = QFwdIO()
        b.obs, b.obs_se, b.obs_sa = self.store.obs.data_ptr(), self.store.row_stride, D
        b.obs_row = self.cur_row.data_ptr()
        b.reset_obs = self.env.reset_obs_ptr()
        b.h_in = b.h_out = self.h.data_ptr()
        b.hin_sa, b.hin_sf, b.hin_se = self.h.stride()   # (self.h is [N][H][E])
        b.hout_sa, b.hout_se, b.hout_sf = b.hin_sa, b.hin_se, b.hin_sf
        b.reset = self.done_buf[1 - k].data_ptr()
        b.mode = MM_Q_ACT
        b.act_out, b.qsel_out = self.act_buf[k].data_ptr(), self.qsel_buf[k].data_ptr()
        b.seed = self.seed
        b.eps_ptr, b.counter_ptr = self.eps_dev.data_ptr(), self.counter_dev.data_ptr()
        return b

    def _io_target(self, k):
        """target fwd of step t (t % 2 == k) on s'_t read from the staging rows; reset = done_{t-1}."""
        N, D, H = self.N, self.D, self.H
        t = QFwdIO()
        t.obs, t.obs_se, t.obs_sa = self.store.obs.data_ptr(), self.store.row_stride, D
        t.obs_row = self.staging.data_ptr()
        t.reset_obs = self.env.reset_obs_ptr()
        t.h_in = t.h_out = self.ht.data_ptr()
        t.hin_sa, t.hin_sf, t.hin_se = self.ht.stride()   # (self.ht is [N][H][E])
        t.hout_sa, t.hout_se, t.hout_sf = t.hin_sa, t.hin_se, t.hin_sf
        t.reset = self.done_buf[1 - k].data_ptr()
        t.mode = MM_Q_MAX
        t.qsel_out = self.maxq.data_ptr()
        return t

    def _build_io(self):
        self.io_b = [self._io_behavior(0), self._io_behavior(1)]
        self.io_t = [self._io_target(0), self._io_target(1)]
        if self.fused:
            # step t (k2 = t % 2, k3 = t % 3): target -> max Q'_t in maxq_buf[k2], reset = done_{t-1}; behavior ->
            # act / Q(a) of step t+1 in slot (k3 + 1) % 3, RNG counter slot k2, reset = this step's dones (in-kernel)
            self.fio_t, self.fio_b = [], {}
            for k2 in range(2):
                it = self._io_target(k2)
                it.qsel_out = self.maxq_buf[k2].data_ptr()
                self.fio_t.append(it)
                for k3 in range(3):
                    ib = self._io_behavior(0)
                    ib.reset = None
                    ib.act_out = self.act_buf[(k3 + 1) % 3].data_ptr()
                    ib.qsel_out = self.qsel_buf[(k3 + 1) % 3].data_ptr()
                    ib.counter_ptr = self.counter_dev.data_ptr() + 8 * k2
                    self.fio_b[(k2, k3)] = ib
        if self.chunked:
            # the chunk launch's target (max Q' into the ring) and behavior (act / Q(a) into the rings) io; the
            # reset flags come from the env inside the kernel
            self.cio_t = self._io_target(0)
            self.cio_t.reset = None
            self.cio_t.qsel_out = self.maxq_r.data_ptr()
            self.cio_b = self._io_behavior(0)
            self.cio_b.reset = None
            self.cio_b.act_out, self.cio_b.qsel_out = self.act_r.data_ptr(), self.qsel_r.data_ptr()
            self.cio_b.counter_ptr = None
        # the prologue behavior fwd (step 0) uses its own RNG counter so it never repeats step 1's draws
        self.io_b0 = self._io_behavior(0)
        self.io_b0.counter_ptr = None
        self.io_b0.counter = 0x7FFFFFFFFFFFFFFF
    def check_errors(self, clear=True):
        """Raise if a rollout kernel set a sticky error bit (synchronous): bit 0 = a staging row outside the chunk
        store was met and that env's stores were skipped (a corrupt PER slot map), bit 1 = a chunk-persistent launch
        gave up waiting for a tile's action hand-off (its blocks were not co-resident)."""
        w = int(self.err.item())
        if clear:
            self.err.zero_()
        if w:
            raise RuntimeError(f"rollout engine device error bits {w:#x}: "
                               + ("corrupt staging row skipped; " if w & 1 else "")
                               + ("chunk-persistent hand-off timed out; " if w & 2 else ""))

    def sync_target(self):
        self.target.copy_from(self.behavior)

    def set_epsilon(self, epsilon):
        if epsilon != self._eps_host:
            self.eps_dev.fill_(float(epsilon))
            self._eps_host = epsilon

    def step(self, epsilon=None):
        """One lockstep env step for all E envs (3-5 launches, no host sync)."""
        if epsilon is not None:
            self.set_epsilon(epsilon)
        self._step_launch()

    def _prologue(self, s):
        if self.chunked:   # the first step's actions / Q(a) into their ring position; fresh hiddens
            ia, EN = self._act_idx(self.t), self.E * self.N
            self.io_b0.act_out = self.act_r.data_ptr() + 4 * ia * EN
            self.io_b0.qsel_out = self.qsel_r.data_ptr() + 4 * ia * EN
            self.io_b0.reset = None
        self.behavior.forward_io(self.E, self.io_b0, s)
        self._primed = True

    def _advance(self, n):
        """Launch the next n steps: chunk mode as chunk-persistent launches of up to (S - 1) C steps each (across chunk
        boundaries; the folds and PER inserts of the launch's chunks follow it), the other modes one step at a time."""
        n = int(n)
        while n > 0:
            m = min(n, (self.S - 1) * self.C) if self.chunked else 1
            self._launch_chunk(m) if self.chunked else self._step_launch()
            n -= m

    def _launch_chunk(self, n):
        """Steps t .. t + n - 1 in ONE chunk-persistent launch (mm_rollout_chunk, across chunk boundaries), then per
        chunk piece of the span its TD / chunk-store fold (mm_td_fold_range) or, where the piece ends its chunk, the
        fold inside the PER insert (mm_per_insert_fold) — the chunks' inserts in chunk order, each swapping its own
        staging set, with nothing sampling in between (the reference's insert-per-chunk semantics)."""
        s = stream_handle(self.device)
        L = lib()
        t, C, E, N, RL = self.t, self.C, self.E, self.N, self.RL
        c0, EN, p = t % C, E * N, t % RL
        assert 1 <= n <= (self.S - 1) * C
        if not self._primed:
            self._prologue(s)
        x = RollChunkIO()
        x.store_obs, x.row_stride, x.n_rows = ptr(self.store.obs), self.store.row_stride, self.store.rows
        x.staging, x.cur_row = ptr(self.staging_all), ptr(self.cur_row)
        x.c0, x.n_steps, x.chunk_len, x.n_sets = c0, n, C, self.S
        x.set0, x.ring_len, x.ring_pos, x.handoff_len = self.staging_set(t), RL, p, RL
        x.act0 = self.act_r.data_ptr() + 4 * p * EN
        x.done_prev = self.done_r.data_ptr() + ((t - 1) % RL) * E
        x.rew, x.done = self.rew_r.data_ptr(), self.done_r.data_ptr()
        x.counter, x.ctl, x.handoff, x.err = ptr(self.counter_dev), ptr(self.ctl), ptr(self.hx), ptr(self.err)
        self.behavior.pack(s)
        self.target.pack(s)
        check(L.mm_rollout_chunk(self.env.handle(), ctypes.byref(self.target.dims), ptr(self.target.packed),
                                 ctypes.byref(self.cio_t), ptr(self.behavior.packed), ctypes.byref(self.cio_b), E,
                                 ctypes.byref(x), s), "rollout_chunk")
        tt = t
        while tt < t + n:   # the span's chunk pieces in order
            a = tt % C
            m = min(C - a, t + n - tt)
            q = tt % RL
            fold = (E, N, self.gamma, self.rew_r.data_ptr() + 4 * q * EN, self.done_r.data_ptr() + q * E,
                    self.qsel_r.data_ptr() + 4 * q * EN, self.maxq_r.data_ptr() + 4 * q * EN,
                    self.act_r.data_ptr() + 4 * q * EN, EN, a, m, C, ptr(self.chunk_td), ptr(self.store.act),
                    ptr(self.store.rew), ptr(self.store.done), ptr(self.staging_all[self.staging_set(tt)]),
                    self.store.rows, ptr(self.err))
            if a + m == C:   # the chunk's end: its last piece's fold rides in the PER insert's first launch
                check(L.mm_per_insert_fold(self.per._h, *fold, None, s), "per_insert_fold")
                self.chunks_inserted += E
            else:
                check(L.mm_td_fold_range(*fold, s), "td_fold_range")
            tt += m
        self._td_pending = False
        self.t += n

    def _step_launch(self):
        """Step t: env(t) -> [target fwd(t) + behavior fwd(t+1)] in ONE launch -> TD/store(t)."""
        if self.chunked:
            return self._launch_chunk(1)
        if self.fused:
            return self._step_launch_fused()
        s = stream_handle(self.device)
        L = lib()
        t = self.t
        c, k = t % self.C, t % 2
        ND = self.N * self.D
        if not self._primed:
            self._prologue(s)
        nxt = ctypes.c_void_p(self.store.obs.data_ptr() + 4 * (c + 1) * ND)
        if c == 0:
            # chunk start folded into the env launch: slot 0 of the new staging rows <- the current obs
            # (slot C of the previous rows, or the reset obs), then the step into slot 1
            check(self.env.step_rows_begin(ptr(self.act_buf[k]), ptr(self.store.obs), self.store.row_stride, self.C,
                                           ptr(self.staging), ptr(self.cur_row), ptr(self.rew), ptr(self.done_buf[k]),
                                           s), "env_step_begin")
        elif not self._td_flushed:
            # env(t) fused with the TD/store of step t-1 (same staging rows inside a chunk)
            kp = 1 - k
            check(self.env.step_rows_td(ptr(self.act_buf[k]), nxt, self.store.row_stride,
                                        ptr(self.staging), ptr(self.cur_row), ptr(self.rew), ptr(self.done_buf[k]),
                                        self.gamma, ptr(self.rew), ptr(self.done_buf[kp]), ptr(self.qsel_buf[kp]),
                                        ptr(self.maxq), ptr(self.act_buf[kp]), ptr(self.chunk_td), c - 1, self.C,
                                        ptr(self.store.act), ptr(self.store.rew), ptr(self.store.done),
                                        ptr(self.staging), ptr(self.counter_dev), s), "env_step_td")
        else:
            check(self.env.step_rows(ptr(self.act_buf[k]), nxt, self.store.row_stride,
                                     ptr(self.staging), None, ptr(self.cur_row), ptr(self.rew),
                                     ptr(self.done_buf[k]), s), "env_step")
        self._td_flushed = False
        iot, iob = self.io_t[k], self.io_b[1 - k]
        iot.obs_off = iob.obs_off = (c + 1) * ND
        self.behavior.pack(s)
        self.target.pack(s)
        check(L.mm_agent_q_fwd2(ctypes.byref(self.target.dims), ptr(self.target.packed), ctypes.byref(iot), self.E,
                                ptr(self.behavior.packed), ctypes.byref(iob), self.E, s), "agent_q_fwd2")
        if c == self.C - 1:
            # the chunk's last TD / store folded into the PER insert's first launch (the insert needs the chunk
            # priorities before the next env step)
            check(L.mm_per_insert_td(self.per._h, self.E, self.N, self.gamma, ptr(self.rew), ptr(self.done_buf[k]),
                                     ptr(self.qsel_buf[k]), ptr(self.maxq), ptr(self.act_buf[k]), ptr(self.chunk_td),
                                     c, self.C, ptr(self.store.act), ptr(self.store.rew), ptr(self.store.done),
                                     ptr(self.counter_dev), ptr(self.staging), None, s), "per_insert_td")
            self.chunks_inserted += self.E
            self._td_pending = False
        else:
            self._td_pending = True
        self.t += 1

    def _step_launch_fused(self):
        """Step t in ONE launch (mm_rollout_step): env(t) + target fwd(t) + behavior fwd(t+1), the TD/store of
        step t-1 folded in; the chunk's last step adds the PER insert with its own TD/store."""
        s = stream_handle(self.device)
        L = lib()
        t = self.t
        c, k2, k3 = t % self.C, t % 2, t % 3
        if not self._primed:
            self._prologue(s)
        x = RollStepIO()
        x.act, x.store_obs, x.row_stride = ptr(self.act_buf[k3]), ptr(self.store.obs), self.store.row_stride
        x.slot, x.chunk_len, x.begin = c + 1, self.C, int(c == 0)
        x.staging, x.cur_row = ptr(self.staging), ptr(self.cur_row)
        x.rew, x.done, x.state_in, x.counter = ptr(self.rew_buf[k2]), ptr(self.done_buf[k2]), k2, ptr(self.counter_dev)
        x.n_rows, x.err = self.store.rows, ptr(self.err)
        if c >= 1 and not self._td_flushed:
            kp, kp3 = 1 - k2, (t - 1) % 3
            x.td_on, x.td_slot, x.gamma = 1, c - 1, self.gamma
            x.td_rew, x.td_done = ptr(self.rew_buf[kp]), ptr(self.done_buf[kp])
            x.td_qsel, x.td_maxq, x.td_act = ptr(self.qsel_buf[kp3]), ptr(self.maxq_buf[kp]), ptr(self.act_buf[kp3])
            x.chunk_td = ptr(self.chunk_td)
            x.store_act, x.store_rew, x.store_done = ptr(self.store.act), ptr(self.store.rew), ptr(self.store.done)
        self._td_flushed = False
        self.behavior.pack(s)
        self.target.pack(s)
        check(L.mm_rollout_step(self.env.handle(), ctypes.byref(self.target.dims), ptr(self.target.packed),
                                ctypes.byref(self.fio_t[k2]), ptr(self.behavior.packed),
                                ctypes.byref(self.fio_b[(k2, k3)]), self.E, ctypes.byref(x), s), "rollout_step")
        if c == self.C - 1:
            check(L.mm_per_insert_td(self.per._h, self.E, self.N, self.gamma, ptr(self.rew_buf[k2]),
                                     ptr(self.done_buf[k2]), ptr(self.qsel_buf[k3]), ptr(self.maxq_buf[k2]),
                                     ptr(self.act_buf[k3]), ptr(self.chunk_td), c, self.C, ptr(self.store.act),
                                     ptr(self.store.rew), ptr(self.store.done), None, ptr(self.staging), None, s),
                  "per_insert_td")
            self.chunks_inserted += self.E
            self._td_pending = False
        else:
            self._td_pending = True
        self.t += 1

    def flush_td(self):
        """Write the last step's TD / transition store now (eager use: it is otherwise fused into the
        next step's env launch); the next step then runs the unfused env kernel."""
        if self._td_pending:
            t = self.t - 1
            self._td_standalone(stream_handle(self.device), t % 2, t % self.C)
            self._td_pending = False
            self._td_flushed = True

    def _td_standalone(self, s, k, c):
        if self.fused:   # step t = self.t - 1: its buffers by parity / ring slot; the RNG counter is per launch
            t = self.t - 1
            rew, qsel, maxq, act, ctr = (self.rew_buf[t % 2], self.qsel_buf[t % 3], self.maxq_buf[t % 2],
                                         self.act_buf[t % 3], None)
        else:
            rew, qsel, maxq, act, ctr = self.rew, self.qsel_buf[k], self.maxq, self.act_buf[k], ptr(self.counter_dev)
        check(lib().mm_td_chunk_step_rows(self.E, self.N, self.gamma, ptr(rew), ptr(self.done_buf[k]),
                                          ptr(qsel), ptr(maxq), ptr(act),
                                          ptr(self.chunk_td), c, self.C, ptr(self.store.act), ptr(self.store.rew),
                                          ptr(self.store.done), ptr(self.staging), ctr, s),
              "td_chunk")

    # ------------------------------------------------------------------ HIP graph replay
    def graph_steps(self):
        """Steps after which every parity-indexed buffer is back at its start (the graph cycle)."""
        if self.chunked:
            return self.RL
        if self.fused:
            return self.C * 6 // math.gcd(self.C, 6)
        return self.C if self.C % 2 == 0 else 2 * self.C

    def capture(self):
        """Capture one chunk of steps (C launches-groups; 2C if C is odd so the done/done_prev
        ping-pong returns to its start) into a HIP graph. Must start at a chunk boundary."""
        assert self.t % self.C == 0, "capture must start at a chunk boundary"
        self.behavior.pack()
        self.target.pack()
        if not self._primed:
            self._prologue(stream_handle(self.device))
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        t0, ins0, n0 = self.t, self.chunks_inserted, len(self.per)
        with graph_capture(g):
            self._advance(self.graph_steps())
        # capture does not execute: rewind the host bookkeeping (PER fill-count mirror too)
        self.t, self.chunks_inserted = t0, ins0
        lib().mm_per_set_size(self.per._h, n0)
        self.graph = g
        self._graph_phase = t0 % self.graph_steps()
        return g

    _graph_phase = 0

    def run_graph(self, epsilon=None):
        """Replay one captured chunk (graph_steps() env steps)."""
        if epsilon is not None:
            self.set_epsilon(epsilon)
        if self.graph is None:
            self.capture()
        assert self.t % self.graph_steps() == self._graph_phase, "run_graph at another graph phase than captured"
        self.behavior.pack()          # weights changed since capture (learner / target sync): repack eagerly
        self.target.pack()
        self.graph.replay()
        n = self.graph_steps()
        self.t += n
        self._td_pending = False
        self.chunks_inserted += self.E * (n // self.C)
        self.per.n_mirror_add(self.E * (n // self.C))

    def capture_steps(self):
        """Capture one single-step HIP graph per phase of the graph cycle, so any number of steps
        (not only whole chunks) can be replayed: ``run_steps``. Same launches as ``capture``."""
        G = self.graph_steps()
        self.behavior.pack()
        self.target.pack()
        if not self._primed:
            self._prologue(stream_handle(self.device))
        torch.cuda.synchronize(self.device)
        saved = (self.t, self.chunks_inserted, self._td_pending, self._td_flushed)
        n0 = len(self.per)
        graphs = []
        for ph in range(G):
            self.t = ph
            self._td_flushed = False
            g = torch.cuda.CUDAGraph()
            with graph_capture(g):
                self._step_launch()
            graphs.append(g)
        self.t, self.chunks_inserted, self._td_pending, self._td_flushed = saved
        lib().mm_per_set_size(self.per._h, n0)
        self.step_graphs = graphs
        return graphs

    step_graphs = None

    def run_steps(self, n_steps, epsilon=None):
        """Advance exactly ``n_steps`` lockstep steps by graph replay: whole-chunk graphs while the
        step count is at a graph-cycle boundary, single-step graphs otherwise."""
        if epsilon is not None:
            self.set_epsilon(epsilon)
        assert not self._td_flushed, "run_steps after flush_td(): continue with step() to the chunk end"
        G = self.graph_steps()
        if (self.t % G, int(n_steps)) in self._region_graphs:
            return self.run_region(n_steps)
        left = int(n_steps)
        while left > 0:
            if self.t % G == 0 and left >= G:
                self.run_graph()
                left -= G
                continue
            if self.step_graphs is None:
                self.capture_steps()
            self.behavior.pack()
            self.target.pack()
            c = self.t % self.C
            self.step_graphs[self.t % G].replay()
            self.t += 1
            if c == self.C - 1:
                self.chunks_inserted += self.E
                self.per.n_mirror_add(self.E)
                self._td_pending = False
            else:
                self._td_pending = not self.chunked
            left -= 1

    def capture_region(self, n_steps, start=None):
        """Capture ONE HIP graph of exactly ``n_steps`` lockstep steps starting at step ``start`` (default: the
        current step; only its graph phase ``start % graph_steps()`` matters), so a timed region of n steps is
        one graph launch instead of a run of chunk / single-step graph replays: on MI355X each graph launch
        after the first leaves the GPU idle for ~9 us (rocprofv3 kernel trace of tools/region_probe.py), i.e.
        ~90 us per 20-step region entered mid-chunk. Same launches as ``capture`` in the same order; graphs are
        cached per (phase, n_steps) and ``run_steps`` replays them."""
        G = self.graph_steps()
        start = self.t if start is None else int(start)
        key = (start % G, int(n_steps))
        if key in self._region_graphs:
            return self._region_graphs[key]
        assert not self._td_flushed, "capture_region after flush_td(): continue with step() to the chunk end"
        self.behavior.pack()
        self.target.pack()
        if not self._primed:
            self._prologue(stream_handle(self.device))
        torch.cuda.synchronize(self.device)
        saved = (self.t, self.chunks_inserted, self._td_pending, self._td_flushed)
        n0 = len(self.per)
        self.t = start
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            self._advance(int(n_steps))
        inserts = self.chunks_inserted - saved[1]
        self.t, self.chunks_inserted, self._td_pending, self._td_flushed = saved
        lib().mm_per_set_size(self.per._h, n0)
        self._region_graphs[key] = (g, inserts)
        return self._region_graphs[key]

    def run_region(self, n_steps, epsilon=None):
        """Replay the captured ``n_steps`` region graph of the current phase (``capture_region``)."""
        if epsilon is not None:
            self.set_epsilon(epsilon)
        G = self.graph_steps()
        g, inserts = self._region_graphs.get((self.t % G, int(n_steps))) or self.capture_region(n_steps)
        self.behavior.pack()
        self.target.pack()
        g.replay()
        self.t += int(n_steps)
        self.chunks_inserted += inserts
        self.per.n_mirror_add(inserts)
        self._td_pending = self.t % self.C != 0 and not self.chunked

    _region_graphs = None

    def run(self, n_steps, epsilon):
        for _ in range(n_steps):
            self.step(epsilon)

    def env_only(self, k=0):
        """The step's env launch on its own (mid-chunk form with the TD folded in); for timing the dual
        forward in its rollout context (bench.py: (env + forward) - env)."""
        s = stream_handle(self.device)
        nxt = ctypes.c_void_p(self.store.obs.data_ptr() + 4 * 2 * self.N * self.D)
        kp = 1 - k
        check(self.env.step_rows_td(ptr(self.act_buf[k]), nxt, self.store.row_stride, ptr(self.staging),
                                    ptr(self.cur_row), ptr(self.rew), ptr(self.done_buf[k]), self.gamma, ptr(self.rew),
                                    ptr(self.done_buf[kp]), ptr(self.qsel_buf[kp]), ptr(self.maxq),
                                    ptr(self.act_buf[kp]), ptr(self.chunk_td), 1, self.C, ptr(self.store.act),
                                    ptr(self.store.rew), ptr(self.store.done), ptr(self.staging), ptr(self.counter_dev),
                                    s), "env_step_td")

    def fused_step_only(self, t=1):
        """The fused mode's one launch on its own (mid-chunk phase t, no TD fold); for timing. Reads env state
        buffer t % 2 and writes the other, so repeated launches recompute the same transition."""
        s = stream_handle(self.device)
        c, k2, k3 = t % self.C, t % 2, t % 3
        x = RollStepIO()
        x.act, x.store_obs, x.row_stride = ptr(self.act_buf[k3]), ptr(self.store.obs), self.store.row_stride
        x.slot, x.chunk_len, x.begin = c + 1, self.C, 0
        x.staging, x.cur_row = ptr(self.staging), ptr(self.cur_row)
        x.rew, x.done, x.state_in, x.counter = ptr(self.rew_buf[k2]), ptr(self.done_buf[k2]), k2, ptr(self.counter_dev)
        x.n_rows, x.err = self.store.rows, ptr(self.err)
        check(lib().mm_rollout_step(self.env.handle(), ctypes.byref(self.target.dims), ptr(self.target.packed),
                                    ctypes.byref(self.fio_t[k2]), ptr(self.behavior.packed),
                                    ctypes.byref(self.fio_b[(k2, k3)]), self.E, ctypes.byref(x), s), "rollout_step")

    def chunk_only(self, n=None):
        """The chunk mode's one launch on its own (steps 0 .. n - 1 from a ring / staging-set cycle start, no TD fold /
        insert); for timing. Advances the env / hidden state like the real launch (the host step count is left alone)."""
        n = self.C if n is None else int(n)
        assert 1 <= n <= (self.S - 1) * self.C
        s = stream_handle(self.device)
        C, E, N, RL = self.C, self.E, self.N, self.RL
        x = RollChunkIO()
        x.store_obs, x.row_stride, x.n_rows = ptr(self.store.obs), self.store.row_stride, self.store.rows
        x.staging, x.cur_row = ptr(self.staging_all), ptr(self.cur_row)
        x.c0, x.n_steps, x.chunk_len, x.n_sets = 0, n, C, self.S
        x.set0, x.ring_len, x.ring_pos, x.handoff_len = 0, RL, 0, RL
        x.act0, x.done_prev = self.act_r.data_ptr(), self.done_r.data_ptr() + (RL - 1) * E
        x.rew, x.done = self.rew_r.data_ptr(), self.done_r.data_ptr()
        x.counter, x.ctl, x.handoff, x.err = ptr(self.counter_dev), ptr(self.ctl), ptr(self.hx), ptr(self.err)
        check(lib().mm_rollout_chunk(self.env.handle(), ctypes.byref(self.target.dims), ptr(self.target.packed),
                                     ctypes.byref(self.cio_t), ptr(self.behavior.packed), ctypes.byref(self.cio_b), E,
                                     ctypes.byref(x), s), "rollout_chunk")

    def fused_forward(self, k=0):
        """The step's dominant launch on its own (target fwd + behavior fwd); for timing."""
        s = stream_handle(self.device)
        check(lib().mm_agent_q_fwd2(ctypes.byref(self.target.dims), ptr(self.target.packed),
                                    ctypes.byref(self.io_t[k]), self.E, ptr(self.behavior.packed),
                                    ctypes.byref(self.io_b[1 - k]), self.E, s), "agent_q_fwd2")
