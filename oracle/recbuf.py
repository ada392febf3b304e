"""Oracle (test infrastructure only): the offpolicy episode replay buffer.

Restates, in numpy with the reference's dtypes and summation orders:
  * SumSegmentTree / MinSegmentTree (offpolicy/utils/segment_tree.py:18-165): f64 heap, root at 1,
    leaves at [cap, 2cap), ``__setitem__`` re-derives every ancestor of the written leaves as
    op(left, right) (:74-89), ``reduce(0, end)`` follows ``_reduce_helper`` (:42-56) — with start 0 the
    recursion is a right fold over the fully covered left children met on the way down —,
    ``find_prefixsum_idx`` the vectorised descent (:115-146: go right when value[left] <= mass);
  * RecPolicyBuffer (rec_buffer.py:85-240): episode ring of [L, cap, ...] fields, ``insert`` wraps
    the index range (:167-171), ``sample_inds`` casts [L, B, N, X] -> [N, L, B, X] (:6-7, 207-240);
  * PrioritizedRecReplayBuffer (rec_buffer.py:243-324): ``insert`` writes max_priority ** alpha into
    leaves ``range(len(idx_range))`` — i.e. leaves 0..n-1, NOT the inserted slots (:265-268, a
    reference quirk kept by ``leaf_mode="reference"``; ``leaf_mode="slots"`` writes the slots);
    ``sample`` draws mass = u * sum(0, len-1) (:272-276) and the IS weights of :293-296;
    ``update_priorities`` (:306-324) writes priorities ** alpha (float32 priorities, float32 pow:
    numpy treats the Python-float alpha as weak) and keeps max_priority as max(1.0, max prio).

The numpy random draws are injected: ``fracs`` = what ``np.random.random(size=B)`` returned
(:274), ``inds`` = what ``np.random.choice(len, B)`` returned (:76).
"""
import numpy as np


class SegTree:
    def __init__(self, capacity, kind):
        assert capacity > 0 and capacity & (capacity - 1) == 0
        self.cap = capacity
        self.kind = kind
        self.neutral = 0.0 if kind == "sum" else float("inf")
        self.v = np.full(2 * capacity, self.neutral, np.float64)

    def op(self, a, b):
        return np.add(a, b) if self.kind == "sum" else np.minimum(a, b)

    def set(self, idx, val):
        """segment_tree.py:74-89 (fancy assignment: last duplicate wins)."""
        idx = np.atleast_1d(np.asarray(idx, np.int64))
        nodes = idx + self.cap
        self.v[nodes] = val
        p = np.unique(nodes // 2)
        while len(p) > 1 or p[0] > 0:
            self.v[p] = self.op(self.v[2 * p], self.v[2 * p + 1])
            p = np.unique(p // 2)

    def reduce_prefix(self, end):
        """reduce(0, end + 1) (segment_tree.py:42-72 with start 0): v[l1] op (v[l2] op (... v[last]))."""
        node, ns, ne = 1, 0, self.cap - 1         # start == node_start at every level
        lefts = []
        while end != ne:
            mid = (ns + ne) // 2
            if end <= mid:
                node, ne = 2 * node, mid
            else:
                lefts.append(2 * node)
                node, ns = 2 * node + 1, mid + 1
        acc = self.v[node]
        for l in reversed(lefts):
            acc = self.op(self.v[l], acc)
        return acc

    def find_prefixsum_idx(self, mass):
        """segment_tree.py:115-146."""
        mass = np.asarray(mass, np.float64).copy()
        idx = np.ones(len(mass), np.int64)
        cont = np.ones(len(mass), bool)
        while np.any(cont):
            idx[cont] = 2 * idx[cont]
            new = np.where(self.v[idx] <= mass, mass - self.v[idx], mass)
            idx = np.where(np.logical_or(self.v[idx] > mass, np.logical_not(cont)), idx, idx + 1)
            mass = new
            cont = idx < self.cap
        return idx - self.cap


def _reduce_ref(tree, end):
    """Direct recursion of _reduce_helper (segment_tree.py:42-56), start 0; cross-check of reduce_prefix."""
    def rec(start, e, node, ns, ne):
        if start == ns and e == ne:
            return tree.v[node]
        mid = (ns + ne) // 2
        if e <= mid:
            return rec(start, e, 2 * node, ns, mid)
        if mid + 1 <= start:
            return rec(start, e, 2 * node + 1, mid + 1, ne)
        return tree.op(rec(start, mid, 2 * node, ns, mid), rec(mid + 1, e, 2 * node + 1, mid + 1, ne))
    return rec(0, end, 1, 0, tree.cap - 1)


class RecBufferOracle:
    """One policy's RecPolicyBuffer + the prioritized wrapper's trees (use_same_share_obs, no
    avail_acts, no reward normalisation — the reference's magym configuration)."""

    def __init__(self, buffer_size, T, N, D, S, A, alpha=0.6, prioritized=True, leaf_mode="reference",
                 same_share=True):
        self.size, self.T, self.N = buffer_size, T, N
        self.same_share = same_share
        self.filled, self.current = 0, 0
        self.obs = np.zeros((T + 1, buffer_size, N, D), np.float32)
        self.share = (np.zeros((T + 1, buffer_size, S), np.float32) if same_share
                      else np.zeros((T + 1, buffer_size, N, S), np.float32))
        self.acts = np.zeros((T, buffer_size, N, A), np.float32)
        self.rew = np.zeros((T, buffer_size, N, 1), np.float32)
        self.dones = np.ones((T, buffer_size, N, 1), np.float32)
        self.dones_env = np.ones((T, buffer_size, 1), np.float32)
        self.prioritized, self.leaf_mode = prioritized, leaf_mode
        self.alpha = alpha
        itcap = 1
        while itcap < buffer_size:
            itcap *= 2
        self.sum, self.min = SegTree(itcap, "sum"), SegTree(itcap, "min")
        self.max_p = 1.0

    def __len__(self):
        return self.filled

    def insert(self, n, obs, share, acts, rew, dones, dones_env):
        """rec_buffer.py:146-190 (+ :262-270)."""
        if self.current + n <= self.size:
            rng = np.arange(self.current, self.current + n)
        else:
            left = self.current + n - self.size
            rng = np.concatenate((np.arange(self.current, self.size), np.arange(left)))
        if self.same_share:
            share = share[:, :, 0]
        self.obs[:, rng] = obs
        self.share[:, rng] = share
        self.acts[:, rng] = acts
        self.rew[:, rng] = rew
        self.dones[:, rng] = dones
        self.dones_env[:, rng] = dones_env
        self.current = rng[-1] + 1
        self.filled = min(self.filled + len(rng), self.size)
        if self.prioritized:
            leaves = np.arange(len(rng)) if self.leaf_mode == "reference" else rng
            val = self.max_p ** self.alpha       # Python float, or np.float32 once a priority exceeded 1
            for i in leaves:                     # one __setitem__ per leaf, as the reference loops
                self.sum.set(i, val)
                self.min.set(i, val)
        return rng

    def sample_inds(self, inds):
        """rec_buffer.py:192-240 without reward normalisation."""
        cast = lambda x: x.transpose(2, 0, 1, 3)
        share = self.share[:, inds] if self.same_share else cast(self.share[:, inds])
        return (cast(self.obs[:, inds]), share, cast(self.acts[:, inds]), cast(self.rew[:, inds]),
                cast(self.dones[:, inds]), self.dones_env[:, inds])

    def sample(self, B, beta, fracs):
        """rec_buffer.py:272-304: returns (batch tuple, weights f64, idx)."""
        assert len(self) > B and beta > 0
        # sum(0, len - 1) = reduce(0, len - 1), whose end -= 1 (segment_tree.py:71) leaves out the
        # last filled leaf: the fold covers leaves [0, len - 2]
        total = self.sum.reduce_prefix(len(self) - 2)
        mass = np.asarray(fracs, np.float64) * total
        idx = self.sum.find_prefixsum_idx(mass)
        p_min = self.min.v[1] / self.sum.v[1]
        max_w = (p_min * len(self)) ** (-beta)
        p_s = self.sum.v[idx + self.sum.cap] / self.sum.v[1]
        w = (p_s * len(self)) ** (-beta) / max_w
        return self.sample_inds(idx), w, idx

    def update_priorities(self, idx, prio):
        """rec_buffer.py:306-324."""
        prio = np.asarray(prio, np.float32)
        assert np.min(prio) > 0 and np.min(idx) >= 0 and np.max(idx) < len(self)
        val = prio ** self.alpha                 # float32 ** weak Python float -> float32
        self.sum.set(idx, val)
        self.min.set(idx, val)
        self.max_p = max(self.max_p, np.max(prio))
