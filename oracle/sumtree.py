"""Oracle (test infrastructure only): chunk-level prioritized replay (SumTree + PER).

Restates vdn/replay_buffer/sumtree.py:8-66 + buffer.py:10-90 and
qmix/replay_buffer/sumtree.py:8-72 + per.py:10-81 in numpy fp64 with the
reference's heap layout (array of 2*cap-1 nodes, leaves at [cap-1, 2cap-2],
children 2i+1 / 2i+2, descent goes left when s <= left).

``flavor``: "vdn" (min-leaf eviction via argsort of the leaves, whole-tree
x step_weight after every sample, buffer.py:72-73) or "qmix" (first leaf in the
full-tree argsort, sumtree.py:45-53; no decay).
"""
import numpy as np


class SumTreeOracle:
    def __init__(self, capacity, flavor="vdn", alpha=0.4, beta=0.4, eps=1e-6, step_weight=0.99,
                 use_step_weight=True, alpha_inc=0.0, beta_inc=0.0):
        self.cap = int(capacity)
        self.tree = np.zeros(2 * self.cap - 1, np.float64)
        self.n_data = 0
        self.flavor = flavor
        self.alpha, self.beta, self.eps = float(alpha), float(beta), float(eps)
        self.step_weight = step_weight
        self.use_step_weight = use_step_weight and flavor == "vdn"
        self.alpha_inc, self.beta_inc = alpha_inc, beta_inc

    # sumtree.py:16-22 / _propagate
    def update_leaf(self, node, priority):
        change = priority - self.tree[node]
        self.tree[node] = priority
        while node != 0:
            node = (node - 1) // 2
            self.tree[node] += change

    def priority(self, td):
        return (td + self.eps) ** self.alpha                      # buffer.py:34-35

    def evict_slot(self):
        """Leaf slot replaced when full: argmin of leaves (vdn) / first leaf of full argsort (qmix)."""
        if self.flavor == "vdn":
            return int(np.argsort(self.tree[self.cap - 1:])[0])   # vdn/replay_buffer/sumtree.py:45
        order = np.argsort(self.tree)                              # qmix/replay_buffer/sumtree.py:45-53
        for node in order:
            if node >= self.cap - 1:
                return int(node - (self.cap - 1))
        raise AssertionError

    def add(self, td):
        """collect_sample: priority from td, fill sequentially then evict; returns data slot."""
        p = self.priority(td)
        if self.n_data < self.cap:
            slot = self.n_data
        else:
            slot = self.evict_slot()
        self.update_leaf(slot + self.cap - 1, p)
        if self.n_data < self.cap:
            self.n_data += 1
        return slot

    def add_batch(self, tds):
        """Batched insert rule of the device engine: free slots first (in order), then the
        k smallest leaves (ties -> lowest slot), taken in ascending slot order, receive the
        remaining inserts in order.
        Identical to sequential add() whenever no new priority is among the evicted minima."""
        tds = list(tds)
        slots = []
        free = min(len(tds), self.cap - self.n_data)
        for j in range(free):
            slots.append(self.n_data + j)
        rest = len(tds) - free
        if rest > 0:
            leaves = self.tree[self.cap - 1:].copy()
            if free > 0:
                leaves[self.n_data:self.n_data + free] = np.inf   # just-filled slots are not victims
            order = np.lexsort((np.arange(self.cap), leaves))
            slots.extend(sorted(int(x) for x in order[:rest]))   # victims in ascending slot order
        for slot, td in zip(slots, tds):
            self.tree[slot + self.cap - 1] = self.priority(td)
        self.n_data = min(self.cap, self.n_data + len(tds))
        self.rebuild()
        return slots

    def rebuild(self):
        """tree[i] = tree[2i+1] + tree[2i+2] bottom-up, vectorised over index ranges [a, b) whose
        children all lie above b (2a + 1 >= b), so every range only reads finished nodes."""
        b = self.cap - 1
        while b > 0:
            a = b // 2
            self.tree[a:b] = self.tree[2 * a + 1:2 * b:2] + self.tree[2 * a + 2:2 * b + 1:2]
            b = a

    def retrieve(self, s):
        """_retrieve_max (sumtree.py:26-35): iterative descent."""
        idx = 0
        n = len(self.tree)
        while True:
            left = 2 * idx + 1
            if left >= n:
                return idx
            if s <= self.tree[left]:
                idx = left
            else:
                s = s - self.tree[left]
                idx = left + 1

    def sample(self, batch, fracs):
        """PER.sample (buffer.py:42-86): stratified s_k = a + (b-a)*f_k; IS weights
        (cap * p / total)^-beta normalised by their max; alpha/beta anneal before the draws.
        Returns (node indices, data slots, priorities, is_weight)."""
        total = self.tree[0]
        seg = total / batch
        self.alpha = float(np.min([1.0, self.alpha + self.alpha_inc]))
        self.beta = float(np.min([1.0, self.beta + self.beta_inc]))
        nodes, pri = [], []
        for k in range(batch):
            a = seg * k
            b = seg * (k + 1)
            s = a + (b - a) * fracs[k]
            node = self.retrieve(s)
            nodes.append(node)
            pri.append(self.tree[node])
        if self.use_step_weight:
            self.tree = self.step_weight * self.tree               # buffer.py:72-73
        probs = np.array(pri) / self.tree[0]
        w = np.power(self.cap * probs, -self.beta)
        w /= w.max()
        nodes = np.array(nodes, np.int64)
        return nodes, nodes - (self.cap - 1), np.array(pri), w.astype(np.float32)

    def update(self, node, td):
        """PER.update: leaf = (td + eps)^alpha, delta propagated to the root."""
        self.update_leaf(int(node), self.priority(td))
