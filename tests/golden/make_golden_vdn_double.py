"""Golden vectors for VDN Double-DQN (``Target_Double_Dqn.train``, vdn/_train.py:104-158).

Runs ONLY in the build container (imports /root/reference, read-only); the GPU box reads the
``vdn_double_train.npz`` fixture only. Same setup as vdn_train.npz (make_golden.py): a reference
PER filled with synthetic chunks, one update (update_iter = 1). The double network's
epsilon-greedy draws (``torch.rand(B)`` then ``torch.randint`` for the random rows, per chunk
step, vdn/_network.py:52-58) are recorded so the build replays them as injected inputs.

Usage (from /root/repo):  python tests/golden/make_golden_vdn_double.py
"""
import os
import random
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as mg  # noqa: E402


class DrawRecorder:
    """Records torch.rand / torch.randint outputs (in call order) made inside the block."""

    def __enter__(self):
        self.rand, self.randint = torch.rand, torch.randint
        self.u, self.ra = [], []

        def rand(*a, **k):
            out = self.rand(*a, **k)
            self.u.append(out.detach().clone())
            return out

        def randint(*a, **k):
            out = self.randint(*a, **k)
            self.ra.append(out.detach().clone())
            return out

        torch.rand, torch.randint = rand, randint
        return self

    def __exit__(self, *exc):
        torch.rand, torch.randint = self.rand, self.randint


def main():
    torch.set_num_threads(1)
    vm = mg.load_pkg("vdn")
    n, d, a, b, c = 2, 94, 5, 32, 10
    eps = 0.3
    mg.seed_all(43)
    obs_sp, act_sp = mg.spaces(n, d, a)
    args = types.SimpleNamespace(use_recurrent=True, use_cuda=False, batch_size=b, update_iter=1, chunk_size=c,
                                 gamma=0.99, grad_clip_norm=5, lr=1e-3)
    target = vm.network.Q_Net(obs_sp, act_sp, args)
    behavior = vm.network.Q_Net(obs_sp, act_sp, args)
    target.load_state_dict(behavior.state_dict())
    with torch.no_grad():
        for p in target.parameters():
            p.add_(torch.randn_like(p) * 0.05)
    per = vm.per.Prioritized_Experience_Replay(mg.per_args("vdn", 64))
    mg.fill_per(per, 48, c, n, d, np.random.default_rng(41))
    cap = mg.CapturePER(per)
    opt = torch.optim.Adam(params=behavior.parameters(), lr=1e-3)
    before = mg.sd_arrays("before.", behavior)
    tgt = mg.sd_arrays("target.", target)
    grads = mg.grads_capture(opt)
    random.seed(779)
    module = vm.train.Target_Double_Dqn(cap, behavior, target, args, torch.device("cpu"))
    with mg.UniformRecorder(), DrawRecorder() as dr:
        loss = module.train(target_network=target, optimizer=opt, epsilon=eps)
    s, act, r, s2, dn, idx, w = cap.samples[0]
    after = mg.sd_arrays("after.", behavior)
    # per step: one torch.rand(B) and one torch.randint(rows_masked, N) -> dense [C, B, N]
    assert len(dr.u) == c and len(dr.ra) == c
    u = torch.stack(dr.u).numpy().astype(np.float32)
    ra = np.zeros((c, b, n), np.int32)
    for t in range(c):
        rows = np.nonzero(u[t] <= np.float32(eps))[0]
        ra[t, rows] = dr.ra[t].numpy().reshape(len(rows), n)
    np.savez_compressed(os.path.join(mg.OUT, "vdn_double_train.npz"), states=s.numpy(), actions=act.numpy(),
                        rewards=r.numpy(), next_states=s2.numpy(), dones=dn.numpy(), is_weight=w.numpy(),
                        loss=np.float32(loss.item()), new_td=np.array([x[1] for x in cap.updates]),
                        gamma=np.float32(0.99), lr=np.float32(1e-3), grad_clip=np.float32(5.0),
                        epsilon=np.float32(eps), double_u=u, double_rand_act=ra, **before, **tgt, **after, **grads)
    print("wrote vdn_double_train.npz; random rows per step:", [int((u[t] <= eps).sum()) for t in range(c)])


if __name__ == "__main__":
    main()
