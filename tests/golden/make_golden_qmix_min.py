"""Golden vectors for the minimal QMIX learner ``qmix/qmix.py``.

Runs ONLY in the build container (imports /root/reference, read-only); the GPU box reads the
``qmix_min_train.npz`` fixture only. ``qmix/qmix.py`` imports ``gym`` at module level (never
used by ``QNet`` / ``MixNet`` / ``train``), so an empty in-memory ``gym`` module stands in.

The fixture holds one ``train()`` iteration (update_iter = 1, recurrent = True) on a fixed batch:
the reference's ``memory.sample_chunk`` is replaced by a stub returning that batch (the same
tensors ``ReplayBuffer.sample_chunk`` builds, qmix/qmix.py:19-46), so no RNG is consumed there.
Recorded: initial state dicts (behavior / target QNet and MixNet), the batch, the gradients after
``clip_grad_norm_`` on each net (qmix/qmix.py:235-238) and the parameters after the Adam step.

Usage (from /root/repo):  python tests/golden/make_golden_qmix_min.py
"""
import importlib
import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = "/root/reference/qmix"
OUT = os.path.dirname(os.path.abspath(__file__))


class Box:
    def __init__(self, d):
        self.shape = (d,)


class Discrete:
    def __init__(self, n):
        self.n = n


def load():
    sys.modules.setdefault("gym", types.ModuleType("gym"))
    sys.path.insert(0, REF)
    try:
        sys.modules.pop("qmix", None)
        return importlib.import_module("qmix")
    finally:
        sys.path.pop(0)


def sd(prefix, module):
    return {f"{prefix}{k}": v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


def gen_obs(rng, shape):
    o = (rng.random(shape) < 0.2).astype(np.float32)
    o[..., :2] = rng.random(shape[:-1] + (2,)).astype(np.float32)
    return o


def main():
    q = load()
    N, D, A, B, C = 3, 47, 5, 8, 5
    gamma, lr = 0.99, 1e-3
    torch.manual_seed(42)
    obs_sp = [Box(D) for _ in range(N)]
    act_sp = [Discrete(A) for _ in range(N)]
    qn = q.QNet(obs_sp, act_sp, recurrent=True)
    qt = q.QNet(obs_sp, act_sp, recurrent=True)
    qt.load_state_dict(qn.state_dict())
    mn = q.MixNet(obs_sp, recurrent=True)
    mt = q.MixNet(obs_sp, recurrent=True)
    # a distinct target mixer so the target path is checked independently of the behavior one
    with torch.no_grad():
        for p in mt.parameters():
            p.add_(0.01 * torch.randn_like(p))
    out = {}
    out.update(sd("q.", qn))
    out.update(sd("qt.", qt))
    out.update(sd("m.", mn))
    out.update(sd("mt.", mt))
    rng = np.random.default_rng(7)
    s = gen_obs(rng, (B, C, N, D))
    s2 = gen_obs(rng, (B, C, N, D))
    a = rng.integers(0, A, (B, C, N)).astype(np.float32)
    r = rng.choice(np.array([-0.01, 0.99, -1.01, 9.99, -10.01], np.float32), (B, C, N))
    d = (rng.random((B, C, 1)) < 0.15).astype(np.float32)
    batch = tuple(torch.tensor(x) for x in (s, a, r, s2, d))

    class Mem:
        def sample_chunk(self, batch_size, chunk_size):
            assert (batch_size, chunk_size) == (B, C)
            return batch

    opt = torch.optim.Adam([{"params": qn.parameters()}, {"params": mn.parameters()}], lr=lr)
    q.train(qn, qt, mn, mt, Mem(), opt, gamma, B, update_iter=1, chunk_size=C)
    out.update({"s": s, "a": a, "r": r, "s2": s2, "done": d})
    for name, mod in (("q.", qn), ("m.", mn)):
        for k, p in mod.named_parameters():
            out[f"grad.{name}{k}"] = p.grad.detach().numpy().copy()
            out[f"post.{name}{k}"] = p.detach().numpy().copy()
    out["meta"] = np.array([N, D, A, B, C], np.int64)
    out["gamma_lr"] = np.array([gamma, lr], np.float64)
    np.savez_compressed(os.path.join(OUT, "qmix_min_train.npz"), **out)
    print("wrote qmix_min_train.npz", len(out), "arrays")


if __name__ == "__main__":
    main()
