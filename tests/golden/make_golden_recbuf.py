"""Golden vectors for the offpolicy episode replay (``PrioritizedRecReplayBuffer`` /
``RecReplayBuffer``, offpolicy/utils/rec_buffer.py:10-324 over SumSegmentTree / MinSegmentTree,
offpolicy/utils/segment_tree.py:18-165).

Runs ONLY in the build container (imports /root/reference, read-only); the GPU box reads
``recbuf_*.npz`` only. A scripted op sequence (inserts that wrap the ring, prioritized samples,
priority updates with duplicate indices and priorities above 1) is run through the reference
classes; the numpy draws each ``sample`` makes internally (``np.random.random`` at :274,
``np.random.choice`` at :76) are read off beforehand from a saved RNG state so tests can inject them.
Recorded after every op: both trees, max_priority, and every sample's indices / weights / batch.

  recbuf_per.npz  PrioritizedRecReplayBuffer, use_same_share_obs=True (the magym runner's setting)
  recbuf_uni.npz  RecReplayBuffer (uniform), use_same_share_obs=False
  recbuf_per_edge.npz  PrioritizedRecReplayBuffer sampled while the last filled leaf holds mass
                   (first insert fills leaves 0..len-1; sum(0, len - 1) leaves leaf len-1 out)

Usage (from /root/repo):  python tests/golden/make_golden_recbuf.py
"""
import importlib
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden_offq import Box, Discrete, install_gym  # noqa: E402

REF = "/root/reference/offpolicy"
SIZE, T, N, D, A = 12, 5, 3, 7, 4
S = N * D


def load():
    install_gym()
    sys.path.insert(0, REF)
    try:
        return importlib.import_module("utils.rec_buffer")
    finally:
        sys.path.pop(0)


def episodes(rng, n):
    obs = rng.standard_normal((T + 1, n, N, D)).astype(np.float32)
    share = np.repeat(obs.reshape(T + 1, n, 1, S), N, axis=2).copy()
    a = rng.integers(0, A, (T, n, N))
    acts = np.eye(A, dtype=np.float32)[a]
    rew = rng.standard_normal((T, n, N, 1)).astype(np.float32)
    dones = (rng.random((T, n, N, 1)) < 0.2).astype(np.float32)
    dones_env = (rng.random((T, n, 1)) < 0.2).astype(np.float32)
    return obs, share, acts, rew, dones, dones_env


FIELDS = ["obs", "share_obs", "acts", "rewards", "dones", "dones_env"]


SCRIPTS = {
    "main": [("insert", 3), ("insert", 2), ("sample", 4, 0.4), ("update",), ("insert", 5), ("sample", 4, 0.55),
             ("update",), ("insert", 4), ("sample", 5, 0.7), ("update",), ("insert", 1), ("insert", 1),
             ("sample", 4, 0.85), ("update",), ("insert", 3), ("sample", 6, 1.0), ("update",), ("sample", 3, 0.9)],
    "edge": [("insert", 5), ("sample", 4, 0.5), ("update",), ("sample", 4, 0.6), ("insert", 3), ("sample", 7, 0.7),
             ("update",), ("insert", 6), ("sample", 11, 0.8)],
}


def run(rb_mod, prioritized, same_share, seed, script="main"):
    np.random.seed(seed)
    rng = np.random.default_rng(seed + 1)
    pinfo = {"policy_0": {"obs_space": Box(shape=(D,)), "share_obs_space": Box(shape=(S,)),
                          "act_space": Discrete(A)}}
    pagents = {"policy_0": list(range(N))}
    if prioritized:
        buf = rb_mod.PrioritizedRecReplayBuffer(0.6, pinfo, pagents, SIZE, T, same_share, False)
    else:
        buf = rb_mod.RecReplayBuffer(pinfo, pagents, SIZE, T, same_share, False)
    out, ops = {}, []
    script = SCRIPTS[script]
    last_idx = None
    for i, op in enumerate(script):
        p = f"op{i}_"
        if op[0] == "insert":
            ep = episodes(rng, op[1])
            rngidx = buf.insert(op[1], *[{"policy_0": x} for x in ep])
            for k, x in zip(FIELDS, ep):
                out[p + k] = x
            out[p + "idx_range"] = np.asarray(rngidx, np.int64)
            ops.append([0, op[1], i])
        elif op[0] == "sample":
            B = op[1]
            st = np.random.get_state()
            if prioritized:
                fr = np.random.random(size=B)
                np.random.set_state(st)
                res = buf.sample(B, op[2], "policy_0")
                out[p + "fracs"] = fr
                out[p + "weights"] = np.asarray(res[7], np.float64)
                out[p + "idx"] = np.asarray(res[8], np.int64)
                last_idx = out[p + "idx"]
            else:
                inds = np.random.choice(len(buf), B)
                np.random.set_state(st)
                res = buf.sample(B)
                out[p + "idx"] = np.asarray(inds, np.int64)
            out[p + "beta"] = np.float64(op[2])
            for k, x in zip(FIELDS, res[:6]):
                out[p + "out_" + k] = np.asarray(x["policy_0"], np.float32)
            ops.append([1, B, i])
        else:
            if not prioritized:
                continue
            prio = (0.2 + 2.8 * rng.random(len(last_idx))).astype(np.float32)
            idx = last_idx.copy()
            idx[-1] = idx[0]                                   # a duplicate index: last write wins
            buf.update_priorities(idx, prio, "policy_0")
            out[p + "idx"], out[p + "prio"] = idx, prio
            ops.append([2, len(idx), i])
        if prioritized:
            out[p + "sum"] = np.asarray(buf._it_sums["policy_0"]._value, np.float64).copy()
            out[p + "min"] = np.asarray(buf._it_mins["policy_0"]._value, np.float64).copy()
            out[p + "max_p"] = np.float64(buf.max_priorities["policy_0"])
        out[p + "len"] = np.int64(len(buf))
    out["ops"] = np.asarray(ops, np.int64)
    out["meta"] = np.array([SIZE, T, N, D, S, A, int(prioritized), int(same_share)], np.int64)
    out["alpha"] = np.float64(0.6)
    return out


def main():
    rb = load()
    for name, pri, same, seed, script in (("per", True, True, 11, "main"), ("uni", False, False, 12, "main"),
                                          ("per_edge", True, True, 13, "edge")):
        out = run(rb, pri, same, seed=seed, script=script)
        np.savez_compressed(os.path.join(HERE, f"recbuf_{name}.npz"), **out)
        print(f"wrote recbuf_{name}.npz ({len(out['ops'])} ops)")


if __name__ == "__main__":
    main()
