"""Device episode replay (mm_erb_*, minimarl.recbuf) vs the reference's own op sequences
(tests/golden/recbuf_*.npz from offpolicy/utils/rec_buffer.py + segment_tree.py) and the oracle.

Tolerances: batches, indices, ring slots and lengths are bit-exact; tree nodes within 4e-7 relative
(a leaf is float32 prio ** alpha — numpy's libm powf vs the device's correctly rounded f64 pow can
differ by one float32 ulp, 1.2e-7); IS weights within 1e-6 relative.
"""
import os

import numpy as np
import pytest
import torch

from oracle.recbuf import RecBufferOracle

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
FIELDS = ["obs", "share_obs", "acts", "rewards", "dones", "dones_env"]


class Box:
    def __init__(self, shape):
        self.shape = shape


class Discrete:
    def __init__(self, n):
        self.n = n


def make(pri, size, T, N, D, S, A, same=True, leaf_mode="reference", seed=0):
    from minimarl.recbuf import PrioritizedRecReplayBuffer, RecReplayBuffer
    pinfo = {"policy_0": {"obs_space": Box((D,)), "share_obs_space": Box((S,)), "act_space": Discrete(A)}}
    pag = {"policy_0": list(range(N))}
    if pri:
        return PrioritizedRecReplayBuffer(0.6, pinfo, pag, size, T, same, False, device="cuda", seed=seed,
                                          leaf_mode=leaf_mode)
    return RecReplayBuffer(pinfo, pag, size, T, same, False, device="cuda", seed=seed)


def tree_close(a, b, what):
    fin = np.isfinite(b)
    np.testing.assert_array_equal(np.isfinite(a), fin, err_msg=what)
    np.testing.assert_allclose(a[fin], b[fin], rtol=4e-7, atol=0, err_msg=what)


@pytest.mark.parametrize("name", ["per", "uni", "per_edge"])
def test_recbuf_replays_reference_sequence(name):
    z = np.load(os.path.join(GOLD, f"recbuf_{name}.npz"))
    SIZE, T, N, D, S, A, pri, same = [int(x) for x in z["meta"]]
    buf = make(bool(pri), SIZE, T, N, D, S, A, bool(same))
    for kind, n, i in z["ops"]:
        p = f"op{i}_"
        if kind == 0:
            ep = [{"policy_0": z[p + k]} for k in FIELDS]
            rng = buf.insert(int(n), *ep)
            np.testing.assert_array_equal(rng, z[p + "idx_range"])
        elif kind == 1:
            if pri:
                res = buf.sample(int(n), float(z[p + "beta"]), "policy_0", fracs=z[p + "fracs"])
                np.testing.assert_array_equal(res[8].cpu().numpy(), z[p + "idx"], err_msg=p)
                np.testing.assert_allclose(res[7].cpu().numpy(), z[p + "weights"], rtol=1e-6, err_msg=p)
            else:
                res = buf.sample(int(n), inds=z[p + "idx"])
            for k, x in zip(FIELDS, res[:6]):
                np.testing.assert_array_equal(x["policy_0"].cpu().numpy(), z[p + "out_" + k], err_msg=p + k)
        else:
            buf.update_priorities(torch.as_tensor(z[p + "idx"]).cuda(), torch.as_tensor(z[p + "prio"]).cuda(),
                                  "policy_0")
        if pri:
            s, m = buf.trees()
            tree_close(s, z[p + "sum"], p + "sum")
            tree_close(m, z[p + "min"], p + "min")
            assert np.float32(buf.max_priority()) == np.float32(z[p + "max_p"]), p
        assert len(buf) == int(z[p + "len"])
    if pri:
        buf.check_errors()


def _episodes(rng, n, T, N, D, A):
    S = N * D
    obs = rng.standard_normal((T + 1, n, N, D)).astype(np.float32)
    share = np.repeat(obs.reshape(T + 1, n, 1, S), N, axis=2).copy()
    acts = np.eye(A, dtype=np.float32)[rng.integers(0, A, (T, n, N))]
    rew = rng.standard_normal((T, n, N, 1)).astype(np.float32)
    dones = (rng.random((T, n, N, 1)) < 0.1).astype(np.float32)
    de = (rng.random((T, n, 1)) < 0.1).astype(np.float32)
    return obs, share, acts, rew, dones, de


@pytest.mark.parametrize("leaf_mode", ["reference", "slots"])
def test_recbuf_vs_oracle_at_scale(leaf_mode):
    """300-episode ring (itcap 512), 40-episode inserts that wrap, 64-episode samples with injected
    draws, device priorities fed back; the oracle runs the same sequence."""
    SIZE, T, N, D, A = 300, 20, 4, 11, 5
    S = N * D
    rng = np.random.default_rng(3)
    buf = make(True, SIZE, T, N, D, S, A, leaf_mode=leaf_mode)
    ora = RecBufferOracle(SIZE, T, N, D, S, A, alpha=0.6, prioritized=True, leaf_mode=leaf_mode)
    for it in range(12):
        ep = _episodes(rng, 40, T, N, D, A)
        np.testing.assert_array_equal(buf.insert(40, *[{"policy_0": x} for x in ep]), ora.insert(40, *ep))
        if len(ora) <= 64:
            continue
        fr = rng.random(64)
        beta = 0.4 + 0.05 * it
        res = buf.sample(64, beta, "policy_0", fracs=fr)
        ob, w, idx = ora.sample(64, beta, fr)
        np.testing.assert_array_equal(res[8].cpu().numpy(), idx)
        np.testing.assert_allclose(res[7].cpu().numpy(), w, rtol=1e-6)
        for k, x, y in zip(FIELDS, res[:6], ob):
            np.testing.assert_array_equal(x["policy_0"].cpu().numpy(), y, err_msg=k)
        prio = torch.as_tensor((0.05 + 3 * rng.random(64)).astype(np.float32)).cuda()
        buf.update_priorities(res[8], prio, "policy_0")
        ora.update_priorities(idx, prio.cpu().numpy())
        s, m = buf.trees()
        tree_close(s, ora.sum.v, f"sum it {it}")
        tree_close(m, ora.min.v, f"min it {it}")
    buf.check_errors()


def test_recbuf_device_rng_and_error_word():
    SIZE, T, N, D, A = 64, 6, 2, 5, 3
    rng = np.random.default_rng(5)
    buf = make(True, SIZE, T, N, D, N * D, A, leaf_mode="slots", seed=9)
    buf.insert(50, *[{"policy_0": x} for x in _episodes(rng, 50, T, N, D, A)])
    # only slots 0..49 hold mass: device draws land there, weights are 1 (all leaves equal)
    res = buf.sample(32, 0.5, "policy_0")
    idx = res[8].cpu().numpy()
    assert idx.min() >= 0 and idx.max() < 50
    np.testing.assert_allclose(res[7].cpu().numpy(), 1.0, rtol=1e-12)
    res2 = buf.sample(32, 0.5, "policy_0")
    assert not np.array_equal(res2[8].cpu().numpy(), idx)          # fresh stream per call
    uni = make(False, SIZE, T, N, D, N * D, A, seed=9)
    uni.insert(50, *[{"policy_0": x} for x in _episodes(rng, 50, T, N, D, A)])
    u = uni.sample(200)
    assert u[-1] is None and u[-2] is None
    # a bad device index and a non-positive priority are flagged, not written
    buf.update_priorities(torch.tensor([3, 60], device="cuda"), torch.tensor([2.0, 1.0], device="cuda"))
    with pytest.raises(AssertionError, match="index"):
        buf.check_errors()
    s, _ = buf.trees()
    assert s[64 + 60] == 0.0


def test_recbuf_feeds_offpolicy_trainer():
    """collect -> PrioritizedRecReplayBuffer.sample -> OffQMix.train_policy_on_batch -> update_priorities,
    all on the device: the trainer sees exactly the batch the oracle gathers, and the trees after the
    update equal the oracle's given the trainer's priorities."""
    from minimarl.offq import OffQMix
    T, N, D, A, B = 25, 2, 47, 5, 8          # the trainer's supported shapes (Checkers obs)
    rng = np.random.default_rng(8)
    buf = make(True, 40, T, N, D, N * D, A, leaf_mode="slots")
    ora = RecBufferOracle(40, T, N, D, N * D, A, alpha=0.6, prioritized=True, leaf_mode="slots")
    ep = _episodes(rng, 30, T, N, D, A)
    buf.insert(30, *[{"policy_0": x} for x in ep])
    ora.insert(30, *ep)
    tr = OffQMix(N, D, A, T, B, mixer="qmix", device="cuda", seed=4)
    fr = rng.random(B)
    sample = buf.sample(B, 0.4, "policy_0", fracs=fr)
    ob, w, idx = ora.sample(B, 0.4, fr)
    for k, x, y in zip(FIELDS, sample[:6], ob):
        np.testing.assert_array_equal(x["policy_0"].cpu().numpy(), y, err_msg=k)
    info, prio, idxes = tr.train_policy_on_batch(sample)
    assert torch.isfinite(info["loss"]).item() and prio is not None
    buf.update_priorities(idxes, prio, "policy_0")
    ora.update_priorities(idx, prio.cpu().numpy())
    s, m = buf.trees()
    tree_close(s, ora.sum.v, "sum")
    tree_close(m, ora.min.v, "min")
    assert np.float32(buf.max_priority()) == np.float32(ora.max_p)


def test_recbuf_gather_guards_bad_indices():
    """Host indices follow numpy indexing of the reference's [.., buffer_size, ..] arrays: [len, size)
    reads the never-written defaults (zeros, dones 1), negatives wrap, beyond the size raises IndexError;
    device indices outside the ring gather zeros and set the error word instead of reading out of bounds."""
    SIZE, T, N, D, A = 16, 4, 2, 3, 3
    rng = np.random.default_rng(1)
    uni = make(False, SIZE, T, N, D, N * D, A)
    ep = _episodes(rng, 5, T, N, D, A)
    uni.insert(5, *[{"policy_0": x} for x in ep])
    with pytest.raises(IndexError):
        uni.sample(2, inds=np.array([0, SIZE]))
    with pytest.raises(IndexError):
        uni.sample(2, inds=np.array([-SIZE - 1, 0]))
    got = uni.sample(3, inds=np.array([7, -12, 2]))      # -12 -> slot 4
    obs = got[0]["policy_0"].cpu().numpy()               # [N, T+1, B, D]
    assert np.all(obs[:, :, 0] == 0)
    np.testing.assert_array_equal(obs[:, :, 1], ep[0][:, 4].transpose(1, 0, 2))
    np.testing.assert_array_equal(obs[:, :, 2], ep[0][:, 2].transpose(1, 0, 2))
    assert np.all(got[4]["policy_0"].cpu().numpy()[:, :, 0] == 1)   # dones default to True
    out = uni.sample(2, inds=torch.tensor([1, 99], device="cuda"))
    assert float(out[0]["policy_0"][:, :, 1].abs().sum()) == 0.0
    with pytest.raises(AssertionError, match="gather|outside the buffer"):
        uni.check_errors()
