"""Generate golden vectors for the QMIX / VDN hot path by importing the reference.

Runs ONLY in the build container (needs /root/reference, read-only). The GPU box
never runs this script: it only reads the ``*.npz`` fixtures written next to it.

Every fixture is data: fixed-seed weights (state_dict arrays), inputs, the
reference's outputs, and every RNG draw the reference made (so the build can
replay them as injected inputs). Reference call sites covered:

  qnet_*.npz        qmix/_network.py:44-64 Q_Net.forward, vdn/_network.py:71-83
  sample_action.npz qmix/_network.py:66-74, vdn/_network.py:52-58,85-88
  td_error.npz      vdn/_utils.py:44-52 (== qmix/_utils.py:86-97)
  mixnet.npz        qmix/_network.py:199-217 Mix_Net.forward
  per_vdn.npz       vdn/replay_buffer/buffer.py, vdn/replay_buffer/sumtree.py
  per_qmix.npz      qmix/replay_buffer/per.py, qmix/replay_buffer/sumtree.py
  vdn_train.npz     vdn/_train.py:184-235 Target_Dqn.train (one update)
  qmix_train.npz    qmix/_train.py:19-121 Train_dqn.train (one update)

Usage (from /root/repo):  python tests/golden/make_golden.py
"""
import importlib
import os
import random
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

_MODS = ["_network", "_train", "_utils", "_config", "replay_buffer",
         "replay_buffer.per", "replay_buffer.sumtree", "replay_buffer.buffer"]


def load_pkg(pkg):
    """Import a reference script package (vdn | qmix) in isolation."""
    for m in _MODS:
        sys.modules.pop(m, None)
    sys.path.insert(0, os.path.join(REF, pkg))
    try:
        mods = types.SimpleNamespace()
        mods.network = importlib.import_module("_network")
        mods.train = importlib.import_module("_train")
        if pkg == "vdn":
            mods.per = importlib.import_module("replay_buffer.buffer")
        else:
            mods.per = importlib.import_module("replay_buffer.per")
        mods.sumtree = importlib.import_module("replay_buffer.sumtree")
    finally:
        sys.path.pop(0)
    return mods


class Box:
    def __init__(self, d):
        self.shape = (d,)


class Discrete:
    def __init__(self, n):
        self.n = n


def spaces(n_agents, obs_dim, n_actions):
    return [Box(obs_dim) for _ in range(n_agents)], [Discrete(n_actions) for _ in range(n_agents)]


def sd_arrays(prefix, module):
    return {f"{prefix}{k}": v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


def seed_all(s):
    random.seed(s)
    np.random.seed(s)
    torch.manual_seed(s)


# ---------------------------------------------------------------- Q_Net forward
def gen_qnet(qm, vm):
    out = {}
    for tag, mods, n, d, b in [("qmix_n2", qm, 2, 47, 5), ("qmix_n8", qm, 8, 47, 32),
                               ("vdn_n2", vm, 2, 94, 32)]:
        seed_all(42)
        obs_sp, act_sp = spaces(n, d, 5)
        args = types.SimpleNamespace(use_recurrent=True, use_cuda=False)
        net = mods.network.Q_Net(obs_sp, act_sp, args)
        g = torch.Generator().manual_seed(7)
        obs = torch.rand(b, n, d, generator=g)
        hid = torch.randn(b, n, 32, generator=g) * 0.5
        with torch.no_grad():
            q, h2 = net(obs, hid)
        out[tag] = dict(obs=obs.numpy(), hidden=hid.numpy(), q=q.numpy(), next_hidden=h2.numpy(),
                        **sd_arrays("p.", net))
    for tag, d in out.items():
        np.savez_compressed(os.path.join(OUT, f"qnet_{tag}.npz"), **d)


# ---------------------------------------------------------------- sample_action
def gen_sample_action(qm, vm):
    res = {}
    for tag, mods in [("qmix", qm), ("vdn", vm)]:
        seed_all(42)
        n, d, a, b, eps = 8, 47, 5, 32, 0.5
        obs_sp, act_sp = spaces(n, d, a)
        args = types.SimpleNamespace(use_recurrent=True, use_cuda=False)
        net = mods.network.Q_Net(obs_sp, act_sp, args)
        g = torch.Generator().manual_seed(11)
        obs = torch.rand(b, n, d, generator=g)
        hid = torch.randn(b, n, 32, generator=g) * 0.5
        torch.manual_seed(1234)
        with torch.no_grad():
            action, h2, q = net.sample_action(obs, hid, eps)
        # replay the RNG draws the reference made (forward consumes none)
        torch.manual_seed(1234)
        u = torch.rand(b)
        mask = u <= eps
        ra = torch.randint(0, a, (int(mask.sum()), n))
        rand_actions = np.zeros((b, n), np.int32)
        rand_actions[mask.numpy()] = ra.numpy()
        greedy = q.argmax(dim=2).numpy()
        replay = np.where(mask.numpy()[:, None], rand_actions, greedy).astype(np.float32)
        assert np.array_equal(replay, action.numpy()), "RNG replay mismatch"
        res[tag] = dict(obs=obs.numpy(), hidden=hid.numpy(), epsilon=np.float32(eps), u=u.numpy(),
                        rand_actions=rand_actions, action=action.numpy(), q=q.numpy(),
                        next_hidden=h2.numpy(), **sd_arrays("p.", net))
    for tag, d in res.items():
        np.savez_compressed(os.path.join(OUT, f"sample_action_{tag}.npz"), **d)


# ---------------------------------------------------------------- cal_td_error
def gen_td_error():
    sys.path.insert(0, os.path.join(REF, "vdn"))
    sys.modules.pop("_utils", None)
    utils = importlib.import_module("_utils")
    sys.path.pop(0)
    g = torch.Generator().manual_seed(3)
    cases = []
    for k in range(16):
        n, a = (2, 5) if k % 2 == 0 else (8, 5)
        action = torch.randint(0, a, (n,), generator=g).float()
        reward = [float(x) for x in (torch.randn(n, generator=g) * 3).tolist()]
        done = int(k % 3 == 0)
        bq = torch.randn(1, n, a, generator=g)
        tq = torch.randn(1, n, a, generator=g)
        td = utils.cal_td_error(action=action, reward=reward, done=done, behavior_q=bq,
                                target_q=tq, gamma=0.99)
        cases.append((n, action.numpy(), np.array(reward, np.float64), done, bq.numpy(), tq.numpy(), td))
    d = {}
    for i, (n, act, rew, done, bq, tq, td) in enumerate(cases):
        d[f"c{i}.action"] = act
        d[f"c{i}.reward"] = rew
        d[f"c{i}.done"] = np.int32(done)
        d[f"c{i}.behavior_q"] = bq
        d[f"c{i}.target_q"] = tq
        d[f"c{i}.td"] = np.float64(td)
    d["n_cases"] = np.int32(len(cases))
    d["gamma"] = np.float64(0.99)
    np.savez_compressed(os.path.join(OUT, "td_error.npz"), **d)


# ---------------------------------------------------------------- Mix_Net
def gen_mixnet(qm):
    seed_all(42)
    n, d, b = 8, 47, 32
    obs_sp, _ = spaces(n, d, 5)
    args = types.SimpleNamespace(use_recurrent=True)
    mix = qm.network.Mix_Net(obs_sp, args)
    g = torch.Generator().manual_seed(5)
    q = torch.randn(b, n, generator=g)
    obs = torch.rand(b, n, d, generator=g)
    hid = torch.randn(b, 32, generator=g) * 0.5
    with torch.no_grad():
        qt, h2 = mix(q, obs, hid)
    np.savez_compressed(os.path.join(OUT, "mixnet.npz"), q=q.numpy(), obs=obs.numpy(), hidden=hid.numpy(),
                        q_tot=qt.numpy(), next_hidden=h2.numpy(), **sd_arrays("p.", mix))


# ---------------------------------------------------------------- PER / SumTree
def per_args(pkg, cap):
    if pkg == "vdn":
        return types.SimpleNamespace(use_step_weight=True, buffer_limit=cap, step_weight=0.99, eps=1e-6,
                                     alpha=0.4, beta=0.4, update_alpha_beta=True, max_episodes=30000,
                                     update_iter=10)
    return types.SimpleNamespace(buffer_limit=cap, eps=1e-6, alpha=0.8, beta=0.2, update_alpha_beta=True,
                                 max_episodes=100000, update_iter=10)


class UniformRecorder:
    """Record the fractions behind ``random.uniform`` (CPython: a + (b-a)*random())."""

    def __enter__(self):
        self.orig = random.uniform
        self.fracs = []

        def uniform(a, b):
            f = random.random()
            self.fracs.append(f)
            return a + (b - a) * f

        random.uniform = uniform
        return self

    def __exit__(self, *exc):
        random.uniform = self.orig


def gen_per(mods, pkg):
    """A scripted op sequence (add / sample / update); every op's tree is recorded."""
    cap, n, d, c, b = 10, 2, 3, 2, 4            # non power of two capacity on purpose
    random.seed(99)
    rng = np.random.default_rng(17)
    per = mods.per.Prioritized_Experience_Replay(per_args(pkg, cap))
    rec = {"capacity": np.int32(cap), "batch": np.int32(b), "chunk": np.int32(c)}
    k = 0
    chunk_id = 0
    for step in range(26):
        if step in (12, 19, 25):
            with UniformRecorder() as ur:
                outs = per.sample(b, c)
            rec[f"op{k}.kind"] = np.int32(1)
            rec[f"op{k}.fracs"] = np.array(ur.fracs, np.float64)
            rec[f"op{k}.idx"] = np.array(outs[5], np.int64)
            rec[f"op{k}.is_weight"] = outs[6].numpy()
            rec[f"op{k}.chunk_ids"] = outs[0].numpy()[:, 0, 0, 0].astype(np.int64)
            rec[f"op{k}.alpha"] = np.float64(per.alpha)
            rec[f"op{k}.beta"] = np.float64(per.beta)
            rec[f"op{k}.tree"] = np.array(per.sum_tree.priority_tree, np.float64)
            k += 1
            new_td = np.abs(rng.standard_normal(b)).astype(np.float32)
            for i, idx in enumerate(outs[5]):
                per.update(idx, torch.tensor([new_td[i]]))
            rec[f"op{k}.kind"] = np.int32(2)
            rec[f"op{k}.idx"] = np.array(outs[5], np.int64)
            rec[f"op{k}.td"] = new_td
            rec[f"op{k}.tree"] = np.array(per.sum_tree.priority_tree, np.float64)
            k += 1
        else:
            td = float(abs(rng.standard_normal()) * 2)
            # payload: the chunk id is written into every state entry so samples can be traced
            s = np.full((c, n, d), float(chunk_id))
            a = rng.integers(0, 5, (c, 1, n)).astype(np.float64)
            r = rng.standard_normal((c, n)).round(3)
            s2 = np.full((c, n, d), float(chunk_id))
            dn = rng.integers(0, 2, (c,))
            per.collect_sample([s.tolist(), a.tolist(), r.tolist(), s2.tolist(), dn.tolist()], td, warm_up=True)
            rec[f"op{k}.kind"] = np.int32(0)
            rec[f"op{k}.td"] = np.float64(td)
            rec[f"op{k}.chunk_id"] = np.int32(chunk_id)
            rec[f"op{k}.tree"] = np.array(per.sum_tree.priority_tree, np.float64)
            rec[f"op{k}.alpha"] = np.float64(per.alpha)
            k += 1
            chunk_id += 1
    rec["n_ops"] = np.int32(k)
    np.savez_compressed(os.path.join(OUT, f"per_{pkg}.npz"), **rec)


# ---------------------------------------------------------------- learners
class CapturePER:
    """Wraps a reference PER to record what sample() returned and what update() got."""

    def __init__(self, per):
        self.per = per
        self.samples = []
        self.updates = []

    def sample(self, b, c):
        out = self.per.sample(b, c)
        self.samples.append(out)
        return out

    def update(self, idx, td):
        self.updates.append((int(idx), float(td)))
        self.per.update(idx, td)

    def __getattr__(self, k):
        return getattr(self.per, k)


def fill_per(per, n_chunks, c, n, d, rng):
    for i in range(n_chunks):
        s = rng.random((c, n, d)).astype(np.float32)
        a = rng.integers(0, 5, (c, 1, n)).astype(np.float32)
        r = (rng.standard_normal((c, n)) * 0.5).astype(np.float32)
        s2 = rng.random((c, n, d)).astype(np.float32)
        dn = (rng.random(c) < 0.15).astype(np.int64)
        per.collect_sample([s.tolist(), a.tolist(), r.tolist(), s2.tolist(), dn.tolist()],
                           float(rng.random() * 2), warm_up=True)


def grads_capture(optimizer):
    store = {}
    orig = optimizer.step

    def step(*a, **k):
        for gi, group in enumerate(optimizer.param_groups):
            for pi, p in enumerate(group["params"]):
                store[f"g{gi}.{pi}"] = p.grad.detach().numpy().copy()
        return orig(*a, **k)

    optimizer.step = step
    return store


def gen_vdn_train(vm):
    n, d, a, b, c = 2, 94, 5, 32, 10
    seed_all(42)
    obs_sp, act_sp = spaces(n, d, a)
    args = types.SimpleNamespace(use_recurrent=True, use_cuda=False, batch_size=b, update_iter=1, chunk_size=c,
                                 gamma=0.99, grad_clip_norm=5, lr=1e-3)
    target = vm.network.Q_Net(obs_sp, act_sp, args)
    behavior = vm.network.Q_Net(obs_sp, act_sp, args)
    target.load_state_dict(behavior.state_dict())
    # perturb target so that target != behavior (a mid-training snapshot)
    with torch.no_grad():
        for p in target.parameters():
            p.add_(torch.randn_like(p) * 0.05)
    per = vm.per.Prioritized_Experience_Replay(per_args("vdn", 64))
    fill_per(per, 48, c, n, d, np.random.default_rng(31))
    cap = CapturePER(per)
    opt = torch.optim.Adam(params=behavior.parameters(), lr=1e-3)
    before = sd_arrays("before.", behavior)
    tgt = sd_arrays("target.", target)
    grads = grads_capture(opt)
    random.seed(777)
    tree0 = np.array(per.sum_tree.priority_tree, np.float64)
    module = vm.train.Target_Dqn(cap, behavior, target, args, torch.device("cpu"))
    with UniformRecorder() as ur:
        loss = module.train(target_network=target, optimizer=opt, epsilon=0.1)
    s, act, r, s2, dn, idx, w = cap.samples[0]
    after = sd_arrays("after.", behavior)
    np.savez_compressed(os.path.join(OUT, "vdn_train.npz"), states=s.numpy(), actions=act.numpy(),
                        rewards=r.numpy(), next_states=s2.numpy(), dones=dn.numpy(), idx=np.array(idx),
                        is_weight=w.numpy(), loss=np.float32(loss.item()),
                        new_td=np.array([u[1] for u in cap.updates]), upd_idx=np.array([u[0] for u in cap.updates]),
                        gamma=np.float32(0.99), lr=np.float32(1e-3), grad_clip=np.float32(5.0),
                        tree_before=tree0, tree_after=np.array(per.sum_tree.priority_tree, np.float64),
                        fracs=np.array(ur.fracs), **before, **tgt, **after, **grads)


def gen_qmix_train(qm):
    n, d, a, b, c = 4, 47, 5, 32, 10
    seed_all(42)
    obs_sp, act_sp = spaces(n, d, a)
    args = types.SimpleNamespace(use_recurrent=True, use_cuda=False, batch_size=b, update_iter=1, chunk_size=c,
                                 gamma=0.99, grad_clip_norm=5, lr=1e-3)
    tq = qm.network.Q_Net(obs_sp, act_sp, args)
    tm = qm.network.Mix_Net(obs_sp, args)
    bq = qm.network.Q_Net(obs_sp, act_sp, args)
    bm = qm.network.Mix_Net(obs_sp, args)
    tq.load_state_dict(bq.state_dict())
    tm.load_state_dict(bm.state_dict())
    with torch.no_grad():
        for p in list(tq.parameters()) + list(tm.parameters()):
            p.add_(torch.randn_like(p) * 0.05)
    per = qm.per.Prioritized_Experience_Replay(per_args("qmix", 64))
    fill_per(per, 48, c, n, d, np.random.default_rng(37))
    cap = CapturePER(per)
    opt = torch.optim.Adam([{"params": bq.parameters()}, {"params": bm.parameters()}], lr=1e-3)
    data = {}
    data.update(sd_arrays("before_q.", bq))
    data.update(sd_arrays("before_m.", bm))
    data.update(sd_arrays("target_q.", tq))
    data.update(sd_arrays("target_m.", tm))
    grads = grads_capture(opt)
    # record the loss by wrapping F.mse_loss accumulation: recompute via a hook on backward
    losses = []
    orig_backward = torch.Tensor.backward

    def bw(self, *a, **k):
        losses.append(float(self.detach()))
        return orig_backward(self, *a, **k)

    torch.Tensor.backward = bw
    try:
        random.seed(778)
        tree0 = np.array(per.sum_tree.priority_tree, np.float64)
        module = qm.train.Train_dqn(args, torch.device("cpu"))
        with UniformRecorder() as ur:
            module.train(cap, bq, bm, tq, tm, opt, 0.1)
    finally:
        torch.Tensor.backward = orig_backward
    s, act, r, s2, dn, idx, w = cap.samples[0]
    data.update(sd_arrays("after_q.", bq))
    data.update(sd_arrays("after_m.", bm))
    np.savez_compressed(os.path.join(OUT, "qmix_train.npz"), states=s.numpy(), actions=act.numpy(),
                        rewards=r.numpy(), next_states=s2.numpy(), dones=dn.numpy(), idx=np.array(idx),
                        is_weight=w.numpy(), loss=np.float32(losses[0]),
                        new_td=np.array([u[1] for u in cap.updates]), upd_idx=np.array([u[0] for u in cap.updates]),
                        gamma=np.float32(0.99), lr=np.float32(1e-3), grad_clip=np.float32(5.0),
                        tree_before=tree0, tree_after=np.array(per.sum_tree.priority_tree, np.float64),
                        fracs=np.array(ur.fracs), **data, **grads)


def main():
    torch.set_num_threads(1)
    qm = load_pkg("qmix")
    gen_qnet_q = qm
    vm = load_pkg("vdn")
    gen_qnet(gen_qnet_q, vm)
    gen_sample_action(qm, vm)
    gen_td_error()
    gen_mixnet(qm)
    gen_per(vm, "vdn")
    gen_per(qm, "qmix")
    gen_vdn_train(vm)
    gen_qmix_train(qm)
    print("fixtures written to", OUT)


if __name__ == "__main__":
    main()
