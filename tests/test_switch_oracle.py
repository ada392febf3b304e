"""CPU checks of the Switch corridor restatement (oracle/switch.py). ma-gym is absent and the
reference holds no Switch outputs, so these pin the restated rules, not ma-gym itself (parity
unpinned): the two agents must pass each other through the one-cell corridor."""
import numpy as np

from oracle.switch import FINAL, INIT, SwitchOracle, SwitchSpec, open_cells


def test_grid_and_initial_obs():
    g = open_cells()
    assert g.sum() == 7 + 2 * 4                 # middle row + four side columns in rows 0 and 2
    ora = SwitchOracle(SwitchSpec(2, max_steps=100), 3)
    o = ora.reset_all()
    assert o.shape == (3, 2, 3)
    np.testing.assert_array_equal(o[0], np.array([[0, 0.17, 0], [0, 0.83, 0]], np.float32))


def test_scripted_swap_reaches_both_targets():
    """agent 0: (0,1) -> (1,1) -> (1,2..6) -> (0,6); agent 1 waits in its room, then (0,5) -> (0,...0)."""
    ora = SwitchOracle(SwitchSpec(2, max_steps=100, step_cost=-0.1), 1)
    ora.reset_all()
    D, L, U, R, NO = 0, 1, 2, 3, 4
    plan = [(D, NO)] + [(R, NO)] * 5 + [(U, NO)] + [(NO, D)] + [(NO, L)] * 5 + [(NO, U)]
    total = np.zeros(2, np.float32)
    for t, (a0, a1) in enumerate(plan):
        o, r, ad, done = ora.step(np.array([[a0, a1]]))
        total += r[0]
    assert ad[0].all() and done[0]
    np.testing.assert_array_equal(ora.pos[0], FINAL[:2])
    # every agent pays step_cost on every step except its arrival step (+5), also after it finished
    assert np.allclose(total, 5 - 0.1 * (len(plan) - 1))


def test_blocking_and_timeout():
    ora = SwitchOracle(SwitchSpec(2, max_steps=3), 1)
    ora.reset_all()
    ora.pos[0, 0] = (1, 3)
    ora.pos[0, 1] = (1, 4)
    ora.step(np.array([[3, 1]]))                 # both try to enter each other's cell: blocked
    np.testing.assert_array_equal(ora.pos[0], [[1, 3], [1, 4]])
    ora.step(np.array([[2, 2]]))                 # up from the corridor is wall
    np.testing.assert_array_equal(ora.pos[0], [[1, 3], [1, 4]])
    o, r, ad, done = ora.step(np.array([[4, 4]]))
    assert done[0] and ad[0].all() and np.isclose(o[0, 0, 2], 1.0)
    assert INIT.shape == (4, 2)
