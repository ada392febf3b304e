"""Golden vectors for the episode-level recurrent QMix / VDN trainer of ``offpolicy/`` (SURVEY §8f
rank 3): ``QMix.train_policy_on_batch`` (offpolicy/algorithms/qmix/qmix.py:80-210) with the
shared ``QMixPolicy`` (algorithm/QMixPolicy.py:51-195: AgentQFunction = LN -> [Linear, ReLU, LN]
x 2 -> GRU -> LN -> Linear, agent_q_function.py / utils/algorithm_utils/{mlp,rnn,act}.py) and the
2-layer-hypernet ``QMixer`` (algorithm/q_mixer.py:6-94) or ``VDNMixer``.

Runs ONLY in the build container (imports /root/reference, read-only); the GPU box reads the
``offq_*.npz`` fixtures only. ``utils/util.py`` imports ``gym`` / ``gym.spaces`` (Box, Discrete,
Tuple; class names and ``.shape`` / ``.n`` only), so an in-memory stand-in is inserted.

One fixture per variant, each ONE train_policy_on_batch call on a fixed synthetic episode batch
(layout of PrioritizedRecReplayBuffer.sample, rec_buffer.py:192-240,278-304):
  offq_qmix.npz  QMixer, use_double_q, use_per (R2D2 priorities, qmix.py:178-191), MSE
  offq_vdn.npz   VDNMixer, max-Q target (no double Q), no PER, Huber (delta 10)
Recorded: behavior params before, gradients after clip_grad_norm_, params after Adam, the new
priorities, loss / grad_norm / Q_tot. The target nets are the behavior nets plus a seeded
perturbation that the tests rebuild from ``target_seed`` (numpy default_rng, f32), so target and
behavior paths are checked independently without storing a second parameter set.

Usage (from /root/repo):  python tests/golden/make_golden_offq.py
"""
import importlib
import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = "/root/reference/offpolicy"
OUT = os.path.dirname(os.path.abspath(__file__))


class Box:
    def __init__(self, low=None, high=None, shape=None, dtype=None):
        self.shape = tuple(shape) if shape is not None else np.asarray(low).shape


class Discrete:
    def __init__(self, n):
        self.n = n


class Tuple:
    pass


class Space:
    pass


def install_gym():
    gym = types.ModuleType("gym")
    sp = types.ModuleType("gym.spaces")
    sp.Box, sp.Discrete, sp.Tuple = Box, Discrete, Tuple
    gym.spaces, gym.Space = sp, Space
    sys.modules.update({"gym": gym, "gym.spaces": sp})


def load():
    install_gym()
    sys.path.insert(0, REF)
    try:
        m = types.SimpleNamespace()
        m.config = importlib.import_module("config")
        m.qmix = importlib.import_module("algorithms.qmix.qmix")
        m.policy = importlib.import_module("algorithms.qmix.algorithm.QMixPolicy")
    finally:
        sys.path.pop(0)
    return m


def target_perturbation(shapes, seed, scale=0.02):
    """The seeded target offsets (rebuilt identically by the tests)."""
    rng = np.random.default_rng(seed)
    return {k: (rng.standard_normal(s) * scale).astype(np.float32) for k, s in shapes}


# the synthetic batch generator lives in the package (bench.py uses it too); same draws as before
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mini-marl_amd"))
from minimarl.synth import gen_obs  # noqa: E402,F401
from minimarl.synth import offq_episode_batch as make_batch  # noqa: E402


def run_variant(m, name, mixer, double_q, use_per, huber, N=2, T=12, B=4, D=47, A=5, seed=5):
    torch.manual_seed(seed)
    args = m.config.get_config().parse_known_args([])[0]
    args.use_double_q, args.use_per, args.use_huber_loss = double_q, use_per, huber
    args.episode_length, args.batch_size = T, B
    cfg = {"args": args, "device": torch.device("cpu"), "num_agents": N}
    pcfg = {"obs_space": Box(shape=(D,)), "act_space": Discrete(A), "cent_obs_dim": N * D}
    policy = m.policy.QMixPolicy(args, cfg, pcfg)
    trainer = m.qmix.QMix(args, N, B, {"policy_0": policy}, lambda a: "policy_0", device=torch.device("cpu"),
                          episode_length=T, vdn=(mixer == "vdn"))
    out = {}
    q_sd = policy.q_network.state_dict()
    m_sd = trainer.mixer.state_dict()
    for k, v in q_sd.items():
        out["q." + k] = v.numpy().copy()
    for k, v in m_sd.items():
        out["m." + k] = v.numpy().copy()
    # perturbed target nets (seeded)
    tseed = seed + 1000
    shapes = [("q." + k, tuple(v.shape)) for k, v in q_sd.items()] + [("m." + k, tuple(v.shape))
                                                                      for k, v in m_sd.items()]
    pert = target_perturbation(shapes, tseed)
    with torch.no_grad():
        tq = trainer.target_policies["policy_0"].q_network
        for k, p in tq.state_dict().items():
            p.add_(torch.from_numpy(pert["q." + k]))
        for k, p in trainer.target_mixer.state_dict().items():
            p.add_(torch.from_numpy(pert["m." + k]))
    rng = np.random.default_rng(seed + 7)
    obs, share, acts, rew, dones, dones_env = make_batch(rng, N, T, B, D, A)
    isw = (0.5 + rng.random(B)).astype(np.float32) if use_per else None
    idx = np.arange(B)
    batch = ({"policy_0": obs}, {"policy_0": share}, {"policy_0": acts}, {"policy_0": rew}, {"policy_0": dones},
             {"policy_0": dones_env}, {"policy_0": None}, isw, idx)
    info, prios, _ = trainer.train_policy_on_batch(batch)
    for k, p in policy.q_network.named_parameters():
        out["grad.q." + k] = (p.grad.numpy().copy() if p.grad is not None else np.zeros(p.shape, np.float32))
        out["post.q." + k] = p.detach().numpy().copy()
    for k, p in trainer.mixer.named_parameters():
        out["grad.m." + k] = p.grad.numpy().copy()
        out["post.m." + k] = p.detach().numpy().copy()
    out.update({"obs": obs, "share_obs": share, "acts": acts, "rewards": rew, "dones": dones,
                "dones_env": dones_env, "loss": np.float32(info["loss"].item()),
                "grad_norm": np.float32(float(info["grad_norm"])), "q_tot": np.float32(info["Q_tot"].item()),
                "meta": np.array([N, T, B, D, A, int(double_q), int(use_per), int(huber), tseed], np.int64),
                "hyper": np.array([args.gamma, args.lr, args.opti_eps, args.max_grad_norm, args.huber_delta,
                                   args.per_nu, args.per_eps], np.float64),
                "mixer_dims": np.array([args.mixer_hidden_dim, args.hypernet_hidden_dim], np.int64)})
    if isw is not None:
        out["is_weight"] = isw
        out["new_priorities"] = np.asarray(prios, np.float64)
    np.savez_compressed(os.path.join(OUT, f"offq_{name}.npz"), **out)
    print(f"wrote offq_{name}.npz: loss {out['loss']:.6f} grad_norm {out['grad_norm']:.6f} "
          f"dones_env steps {dones_env[:, :, 0].sum(0)}")


def main():
    torch.set_num_threads(1)
    m = load()
    run_variant(m, "qmix", "qmix", True, True, False)
    run_variant(m, "vdn", "vdn", False, False, True, seed=6)


if __name__ == "__main__":
    main()
