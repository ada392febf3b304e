"""Pins oracle/recbuf.py (episode replay + segment trees) to the reference's own outputs
(tests/golden/recbuf_*.npz, made by tests/golden/make_golden_recbuf.py from
offpolicy/utils/rec_buffer.py + segment_tree.py)."""
import os

import numpy as np
import pytest

from oracle.recbuf import RecBufferOracle, SegTree, _reduce_ref

GOLD = os.path.join(os.path.dirname(__file__), "golden")
FIELDS = ["obs", "share_obs", "acts", "rewards", "dones", "dones_env"]


def replay(z, check):
    SIZE, T, N, D, S, A, pri, same = [int(x) for x in z["meta"]]
    ora = RecBufferOracle(SIZE, T, N, D, S, A, alpha=float(z["alpha"]), prioritized=bool(pri), same_share=bool(same))
    for kind, n, i in z["ops"]:
        p = f"op{i}_"
        if kind == 0:
            rng = ora.insert(int(n), *[z[p + k] for k in FIELDS])
            check(p + "idx_range", rng, z[p + "idx_range"])
        elif kind == 1:
            if pri:
                batch, w, idx = ora.sample(int(n), float(z[p + "beta"]), z[p + "fracs"])
                check(p + "idx", idx, z[p + "idx"])
                check(p + "weights", w, z[p + "weights"])
            else:
                batch = ora.sample_inds(z[p + "idx"])
            for k, x in zip(FIELDS, batch):
                check(p + "out_" + k, x, z[p + "out_" + k])
        else:
            ora.update_priorities(z[p + "idx"], z[p + "prio"])
        if pri:
            check(p + "sum", ora.sum.v, z[p + "sum"])
            check(p + "min", ora.min.v, z[p + "min"])
            check(p + "max_p", np.float64(ora.max_p), z[p + "max_p"])
        check(p + "len", len(ora), z[p + "len"])
    return ora


@pytest.mark.parametrize("name", ["per", "uni", "per_edge"])
def test_recbuf_oracle_matches_reference(name):
    z = np.load(os.path.join(GOLD, f"recbuf_{name}.npz"))

    def check(k, a, b):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b), err_msg=k)
    replay(z, check)


def test_prefix_reduce_matches_recursion():
    rng = np.random.default_rng(0)
    t = SegTree(32, "sum")
    t.set(np.arange(32), rng.random(32) * 10)
    for end in range(32):
        assert t.reduce_prefix(end) == _reduce_ref(t, end)
