"""Offpolicy episode replay on the MI355X: ``RecReplayBuffer`` / ``PrioritizedRecReplayBuffer``.

Mirrors offpolicy/utils/rec_buffer.py:10-324 (same constructor arguments, ``insert`` / ``sample`` /
``update_priorities`` / ``__len__``, same return tuples and layouts) over the C ABI ``mm_erb_*``
(include/minimarl.h, csrc/recbuf.hip). Each policy's episodes, SumSegmentTree and MinSegmentTree
(offpolicy/utils/segment_tree.py) live in HBM; sampled batches come back as device tensors already
in the layout ``OffQMix.train_policy_on_batch`` consumes, and ``update_priorities`` takes the
trainer's device priorities, so a collect -> sample -> train -> re-prioritise cycle never syncs.

Differences from the reference, by necessity or by switch:
* the numpy draws (``np.random.random`` in ``_sample_proportional``, ``np.random.choice`` in the
  uniform ``sample``) come from the device counter RNG, or are injected (``fracs=`` / ``inds=``);
* ``leaf_mode="reference"`` (default) keeps the reference's insert, which writes max_priority **
  alpha into leaves 0..n-1 rather than the inserted slots (rec_buffer.py:265-268); ``"slots"``
  writes the slots' leaves;
* the reference's asserts in ``update_priorities`` (:315-318) run on the host for host inputs; for
  device inputs the kernel skips offending entries and flags them (``check_errors``);
* ``use_avail_acts=True`` is rejected: the reference's ``insert`` does not forward ``avail_acts``
  to the policy buffer and fails there; ``use_reward_normalization`` is not built.
There is no CPU path.
"""
import ctypes

import numpy as np
import torch

from ._lib import ErbDims, ErbFields, check, lib, release
from .qnet import ptr, stream_handle

FIELDS = ("obs", "share_obs", "acts", "rewards", "dones", "dones_env")


def _dim(space):
    """utils/util.py get_dim_from_space for the spaces the magym runner uses."""
    if hasattr(space, "n"):
        return int(space.n)
    if hasattr(space, "shape"):
        return int(space.shape[0])
    if isinstance(space, (list, tuple)):
        return int(sum(space))
    raise NotImplementedError(type(space))


class _PolicyStore:
    """One policy's device buffer (RecPolicyBuffer + its two trees)."""

    def __init__(self, buffer_size, T, N, D, S, A, same_share, prioritized, leaf_mode, alpha, device):
        self.T, self.N, self.D, self.S, self.A = T, N, D, S, A
        self.same_share = same_share
        self.device = device
        self.dims = ErbDims(T, N, D, S, A, int(same_share), int(prioritized), 0 if leaf_mode == "reference" else 1)
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            check(lib().mm_erb_create(ctypes.byref(self.dims), int(buffer_size), float(alpha), ctypes.byref(h)),
                  "erb_create")
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._h = None
            try:
                release("mm_erb_destroy", h)   # deferred while a graph capture is running
            except Exception:   # interpreter shutdown: module globals already gone
                pass

    def out_shapes(self, B):
        T, N = self.T, self.N
        share = (T + 1, B, self.S) if self.same_share else (N, T + 1, B, self.S)
        return {"obs": (N, T + 1, B, self.D), "share_obs": share, "acts": (N, T, B, self.A),
                "rewards": (N, T, B, 1), "dones": (N, T, B, 1), "dones_env": (T, B, 1)}

    def gather(self, idx, B):
        out = {k: torch.empty(s, device=self.device) for k, s in self.out_shapes(B).items()}
        f = ErbFields(*[ptr(out[k]) for k in FIELDS])
        check(lib().mm_erb_gather(self._h, int(B), ptr(idx), ctypes.byref(f), stream_handle(self.device)), "erb_gather")
        return out


class RecReplayBuffer:
    """rec_buffer.py:10-82 (uniform episode sampling)."""
    prioritized = False

    def __init__(self, policy_info, policy_agents, buffer_size, episode_length, use_same_share_obs, use_avail_acts,
                 use_reward_normalization=False, device="cuda", seed=0, leaf_mode="reference", _alpha=0.6):
        if use_avail_acts:
            raise NotImplementedError("use_avail_acts: the reference's RecReplayBuffer.insert does not pass "
                                      "avail_acts on (rec_buffer.py:56-59) and fails in RecPolicyBuffer.insert")
        if use_reward_normalization:
            raise NotImplementedError("use_reward_normalization is not built (off in the reference's configs)")
        assert leaf_mode in ("reference", "slots")
        self.policy_info = policy_info
        self.buffer_size, self.episode_length = int(buffer_size), int(episode_length)
        self.use_same_share_obs = bool(use_same_share_obs)
        self.device = torch.device(device)
        self.seed, self._draws = int(seed), 0
        self.policy_buffers = {}
        for p_id, info in policy_info.items():
            n = len(policy_agents[p_id])
            D = _dim(info["obs_space"])
            S = _dim(info["share_obs_space"])
            A = _dim(info["act_space"])
            self.policy_buffers[p_id] = _PolicyStore(self.buffer_size, self.episode_length, n, D, S, A,
                                                     self.use_same_share_obs, self.prioritized, leaf_mode, _alpha,
                                                     self.device)

    def __len__(self):
        return int(lib().mm_erb_len(self.policy_buffers["policy_0"]._h))

    def _dev(self, x):
        t = x if torch.is_tensor(x) else torch.as_tensor(np.asarray(x))
        return t.to(device=self.device, dtype=torch.float32).contiguous()

    def insert(self, num_insert_episodes, obs, share_obs, acts, rewards, dones, dones_env, avail_acts=None):
        """rec_buffer.py:39-60 / 146-190: returns the ring slots written (np.ndarray)."""
        n = int(num_insert_episodes)
        idx = np.zeros(n, np.int64)
        keep = []
        for p_id, pb in self.policy_buffers.items():
            src = [self._dev(d[p_id]) for d in (obs, share_obs, acts, rewards, dones, dones_env)]
            T = self.episode_length
            assert tuple(src[2].shape[:2]) == (T, n), ("different dimension!", tuple(src[2].shape))
            keep.append(src)
            f = ErbFields(*[ptr(t) for t in src])
            check(lib().mm_erb_insert(pb._h, n, ctypes.byref(f), idx.ctypes.data_as(ctypes.c_void_p),
                                      stream_handle(self.device)), "erb_insert")
        self._keep = keep           # alive until the copies ran (stream-ordered reuse is safe after)
        return idx

    def _next_counter(self):
        self._draws += 1
        return self._draws - 1

    def sample(self, batch_size, inds=None):
        """rec_buffer.py:62-82: B episodes uniformly (device RNG, or the injected ``inds``)."""
        B = int(batch_size)
        pb0 = self.policy_buffers["policy_0"]
        if inds is None:
            idx = torch.empty(B, dtype=torch.int64, device=self.device)
            check(lib().mm_erb_sample_uniform(pb0._h, B, self.seed, self._next_counter(), ptr(idx),
                                              stream_handle(self.device)), "erb_sample_uniform")
        else:
            if not torch.is_tensor(inds):
                # numpy fancy indexing into the [.., buffer_size, ..] arrays (rec_buffer.py:192-240):
                # indices in [len, buffer_size) read the never-written defaults (0, dones 1), negative
                # ones wrap, only |index| beyond buffer_size raises
                ii = np.asarray(inds, np.int64)
                size = self.buffer_size
                if len(ii) and (ii.min() < -size or ii.max() >= size):
                    raise IndexError(f"sample: index out of bounds for a buffer of size {size}")
                inds = np.where(ii < 0, ii + size, ii)
            idx = torch.as_tensor(inds).to(device=self.device, dtype=torch.int64).contiguous()
        return self._gather_all(idx, B) + (None, None)

    def _gather_all(self, idx, B):
        res = {k: {} for k in FIELDS}
        avail = {}
        for p_id, pb in self.policy_buffers.items():
            out = pb.gather(idx, B)
            for k in FIELDS:
                res[k][p_id] = out[k]
            avail[p_id] = None
        return tuple(res[k] for k in FIELDS) + (avail,)

    # -- inspection (tests, checkpoints) -------------------------------------------------------
    def state(self, p_id="policy_0"):
        """Device copies (stream-ordered) of (sum tree f64 [2 itcap], min tree, max_priority f32 [1],
        error word i32 [1])."""
        pb = self.policy_buffers[p_id]
        n = 2 * int(lib().mm_erb_it_capacity(pb._h))
        st = (torch.empty(n, dtype=torch.float64, device=self.device),
              torch.empty(n, dtype=torch.float64, device=self.device),
              torch.empty(1, dtype=torch.float32, device=self.device),
              torch.empty(1, dtype=torch.int32, device=self.device))
        check(lib().mm_erb_copy_state(pb._h, *[ptr(t) for t in st], stream_handle(self.device)), "erb_copy_state")
        return st

    def trees(self, p_id="policy_0"):
        """(sum tree, min tree) as host f64 arrays."""
        s, m, _, _ = self.state(p_id)
        return s.cpu().numpy(), m.cpu().numpy()

    def max_priority(self, p_id="policy_0"):
        return float(self.state(p_id)[2].cpu()[0])

    def check_errors(self, p_id="policy_0"):
        """Raise AssertionError if a device-side update_priorities hit the reference's asserts."""
        e = int(self.state(p_id)[3].cpu()[0])
        assert e & 1 == 0, "update_priorities: index outside [0, len)"
        assert e & 2 == 0, "update_priorities: priority <= 0"
        assert e & 4 == 0, "sample: episode index outside the buffer"


class PrioritizedRecReplayBuffer(RecReplayBuffer):
    """rec_buffer.py:243-324 (proportional prioritisation over SumSegmentTree / MinSegmentTree)."""
    prioritized = True

    def __init__(self, alpha, policy_info, policy_agents, buffer_size, episode_length, use_same_share_obs,
                 use_avail_acts, use_reward_normalization=False, device="cuda", seed=0, leaf_mode="reference"):
        self.alpha = alpha
        super().__init__(policy_info, policy_agents, buffer_size, episode_length, use_same_share_obs, use_avail_acts,
                         use_reward_normalization, device=device, seed=seed, leaf_mode=leaf_mode, _alpha=alpha)

    def sample(self, batch_size, beta=0, p_id=None, fracs=None):
        """rec_buffer.py:278-304. Returns (obs, share_obs, acts, rewards, dones, dones_env, avail_acts,
        weights, batch_inds): dict fields of device tensors in the sample layout, weights device f64 [B],
        batch_inds device int64 [B]. ``fracs``: the uniform draws to use instead of the device RNG."""
        B = int(batch_size)
        assert len(self) > B, "Cannot sample with no completed episodes in the buffer!"
        assert beta > 0
        pb = self.policy_buffers[p_id if p_id is not None else "policy_0"]
        idx = torch.empty(B, dtype=torch.int64, device=self.device)
        w = torch.empty(B, dtype=torch.float64, device=self.device)
        fr = None
        if fracs is not None:
            fr = torch.as_tensor(np.asarray(fracs, np.float64) if not torch.is_tensor(fracs) else fracs).to(
                device=self.device, dtype=torch.float64).contiguous()
        check(lib().mm_erb_sample_prioritized(pb._h, B, float(beta), ptr(fr), self.seed,
                                              self._next_counter() if fr is None else 0, ptr(idx), ptr(w), None,
                                              stream_handle(self.device)), "erb_sample_prioritized")
        self._keep_fr = fr
        return self._gather_all(idx, B) + (w, idx)

    def update_priorities(self, idxes, priorities, p_id=None):
        """rec_buffer.py:306-324 (device or host inputs)."""
        pb = self.policy_buffers[p_id if p_id is not None else "policy_0"]
        if not torch.is_tensor(idxes) or not torch.is_tensor(priorities):
            pi = np.asarray(priorities if not torch.is_tensor(priorities) else priorities.cpu())
            ii = np.asarray(idxes if not torch.is_tensor(idxes) else idxes.cpu())
            assert len(ii) == len(pi)
            assert np.min(pi) > 0
            assert np.min(ii) >= 0
            assert np.max(ii) < len(self)
        idx = torch.as_tensor(idxes).to(device=self.device, dtype=torch.int64).contiguous()
        pr = torch.as_tensor(priorities).to(device=self.device, dtype=torch.float32).contiguous()
        assert idx.numel() == pr.numel()
        check(lib().mm_erb_update_priorities(pb._h, ptr(idx), ptr(pr), int(idx.numel()), stream_handle(self.device)),
              "erb_update_priorities")
        self._keep_up = (idx, pr)


__all__ = ["RecReplayBuffer", "PrioritizedRecReplayBuffer"]
