"""Measure the fp32 spread that tests/test_gpu_mappo.py derives its MAPPO training bars from (CPU only).

For the golden fixture (E = 4, N = 2, T = 10) and a synthetic cfg3-shaped rollout (E envs x 8 agents x T = 100
on the oracle env, random actions / hiddens / values), runs the oracle's PPO epoch-0 gradients three times
(fp32 chunk order, fp32 permuted chunk order, float64) and prints, per tensor, the spread relative to the
tensor's max |g|. Usage: python tools/mappo_tol.py [E]   (default 512, the GPU scale test's E)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from oracle import mappo as om  # noqa: E402
from oracle.env import EnvSpec, VecEnvOracle  # noqa: E402
import test_gpu_mappo as t  # noqa: E402


def report(tag, g64, sp):
    rel = {k: sp[k] / max(np.abs(g64[k]).max(), 1e-30) for k in sp}
    worst = max(rel, key=rel.get)
    print(f"{tag}: spread / max|g| median {np.median(list(rel.values())):.2e}, max {rel[worst]:.2e} ({worst})")


def synthetic(E, N=8, T=100, D=47, H=32, seed=0):
    rng = np.random.default_rng(seed)
    ora = VecEnvOracle(EnvSpec(N, 100), E)
    obs, masks, acts, rew = [ora.observe()], [np.ones((E, N))], [], []
    for _ in range(T):
        a = rng.integers(0, 5, (E, N))
        _, r, d = ora.step(a)
        ora.reset_envs(d)
        obs.append(ora.observe())
        masks.append(np.repeat((~d)[:, None], N, 1))
        acts.append(a)
        rew.append(r)
    f = lambda x: np.asarray(x, np.float32)  # noqa: E731
    data = {"obs": f(obs), "masks": f(masks)[..., None], "active_masks": np.ones((T + 1, E, N, 1), np.float32),
            "actions": f(acts)[..., None], "rewards": f(rew)[..., None],
            "rnn_states": f(rng.normal(0, 0.3, (T + 1, E, N, 1, H))),
            "rnn_states_critic": f(rng.normal(0, 0.3, (T + 1, E, N, 1, H))),
            "action_log_probs": f(np.log(rng.uniform(0.1, 0.3, (T, E, N, 1)))),
            "value_preds": f(rng.normal(0, 1, (T + 1, E, N, 1))), "returns": f(rng.normal(0, 1, (T + 1, E, N, 1)))}
    g = torch.Generator().manual_seed(seed)

    def net(O):
        r = lambda *s: torch.randn(*s, generator=g) * 0.2  # noqa: E731
        return dict(ln0_w=torch.ones(D), ln0_b=torch.zeros(D), W1=r(H, D), b1=torch.zeros(H), ln1_w=torch.ones(H),
                    ln1_b=torch.zeros(H), W2=r(H, H), b2=torch.zeros(H), ln2_w=torch.ones(H), ln2_b=torch.zeros(H),
                    Wih=r(3 * H, H), Whh=r(3 * H, H), bih=torch.zeros(3 * H), bhh=torch.zeros(3 * H),
                    lnr_w=torch.ones(H), lnr_b=torch.zeros(H), Wo=r(O, H) * 0.5, bo=torch.zeros(O))
    return net(5), net(1), data, (0.1, 0.5, 0.9), T * E * N // 5


def main():
    fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "mappo_train.npz")))
    PA, PC, data, vn0, nch = t._golden_oracle_inputs(fx)
    L = int(fx["L"])
    report("golden epoch-0 gradients", *t._fp32_spread(
        lambda dt, pm: t._unclipped_grads(t._ppo_oracle(PA, PC, data, vn0, 1, L, dt, pm)[0]), nch))
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    PA, PC, data, vn0, nch = synthetic(E)
    report(f"synthetic {E} x 8 x 100 epoch-0 gradients", *t._fp32_spread(
        lambda dt, pm: t._unclipped_grads(t._ppo_oracle(PA, PC, data, vn0, 1, 5, dt, pm)[0]), nch))
    _ = om


if __name__ == "__main__":
    main()
