"""Switch corridor env on the GPU (csrc/switch.hip, minimarl.env.SwitchVecEnv) vs its restatement
oracle/switch.py: obs, rewards, per-agent and env dones bit-exact, with auto-reset, for 2-4 agents,
partial / full observation, clock on / off. (ma-gym parity itself is unpinned: it is absent.)"""
import numpy as np
import pytest
import torch

from oracle.switch import SwitchOracle, SwitchSpec

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,full,clock,max_steps", [(2, False, True, 100), (2, True, True, 9), (3, False, False, 25),
                                                    (4, True, True, 40)])
def test_switch_matches_oracle(N, full, clock, max_steps):
    from minimarl.env import SwitchVecEnv
    E = 384
    env = SwitchVecEnv(E, N, max_steps=max_steps, step_cost=-0.1, full_observable=full, clock=clock)
    ora = SwitchOracle(SwitchSpec(N, max_steps, -0.1, full, clock), E)
    np.testing.assert_array_equal(env.reset().cpu().numpy(), ora.reset_all())
    rng = np.random.default_rng(N * 10 + max_steps)
    D, L, U, R, NO = 0, 1, 2, 3, 4
    plan = [(D, NO)] + [(R, NO)] * 5 + [(U, NO)] + [(NO, D)] + [(NO, L)] * 5 + [(NO, U)]
    arrivals = 0
    for t in range(120):
        act = rng.integers(0, 5, (E, N)).astype(np.int32)
        if N == 2 and t < len(plan):
            act[0] = plan[t]                                  # env 0: both agents swap rooms
        nxt, rew, adone, done, cur = env.step(torch.as_tensor(act).cuda(), autoreset=True)
        o, r, ad, dn = ora.step(act)
        np.testing.assert_array_equal(nxt.cpu().numpy(), o, err_msg=f"obs t={t}")
        np.testing.assert_array_equal(rew.cpu().numpy(), r, err_msg=f"rew t={t}")
        np.testing.assert_array_equal(adone.cpu().numpy().astype(bool), ad, err_msg=f"agent_done t={t}")
        np.testing.assert_array_equal(done.cpu().numpy().astype(bool), dn, err_msg=f"done t={t}")
        arrivals += int((r == 5).sum())
        ora.reset_envs(dn)
        np.testing.assert_array_equal(cur.cpu().numpy(), ora.obs(), err_msg=f"obs_cur t={t}")
    pos, ad, steps = env.get_state()
    np.testing.assert_array_equal(pos, ora.pos)
    np.testing.assert_array_equal(steps, ora.steps)
    if N == 2 and max_steps == 100:
        assert arrivals >= 2
