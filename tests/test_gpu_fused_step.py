"""GPU: the fused one-launch rollout step (mm_rollout_step, RolloutEngine(fused=True)) against the two-launch
step (env kernel + dual forward) and against the oracle env.

The fused kernel runs the same restated Checkers dynamics and the same fp16x3 / exact-f32 forward bodies, so
every stored transition, hidden state, chunk priority, PER tree and env state must be BIT-identical to the
two-launch engine with the same seed, through chunk starts (slot-0 writes), chunk ends (PER insert with the
TD fold), auto-resets, flush_td and graph replay; the env side is also checked bit-exact against
oracle/env.py step by step."""
import numpy as np
import pytest
import torch

from oracle.env import EnvSpec, VecEnvOracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _state(e):
    torch.cuda.synchronize()
    st = [e.store.obs, e.store.act, e.store.rew, e.store.done, e.h, e.ht, e.chunk_td, e.cur_row, e.staging,
          e.per.tree(), e.per.slot_rows(), e.act, e.last_rew, e.last_done, e.counter_dev[e.t % 2 if e.fused else 0]]
    return [x.detach().clone().cpu() for x in st] + [torch.as_tensor(v) for v in e.env.get_state()]


def _pair(E, f1, g, h, seed, guard=False, n=8):
    from minimarl.engine import RolloutEngine
    kw = dict(f1=f1, g=g, h=h, chunk=10, capacity=4 * E, seed=seed, device=DEV)
    a = RolloutEngine(E, n, fused=False, **kw)
    b = RolloutEngine(E, n, fused=True, **kw)
    assert b.fused and not a.fused and b.graph_steps() == 30
    if guard:   # agent 3 beyond the fp16 range: both engines run it on the exact-f32 image
        for eng in (a, b):
            with torch.no_grad():
                eng.behavior.view("W1")[3, 0, :] = 3.0e3
            eng.behavior.mark_dirty()
            eng.sync_target()
    return a, b


@pytest.mark.parametrize("E,f1,g,h,guard,n", [(2048, 64, 64, 64, False, 8), (2200, 64, 32, 32, False, 8),
                                              (2048, 64, 64, 64, True, 8), (2304, 64, 32, 32, False, 4),
                                              (2048, 128, 32, 32, False, 8), (2048, 64, 32, 64, False, 8),
                                              (2100, 64, 64, 64, True, 4)])
def test_fused_step_bit_identical_to_two_launch(E, f1, g, h, guard, n):
    a, b = _pair(E, f1, g, h, seed=21, guard=guard, n=n)
    spec = EnvSpec(n, 100)
    ora = VecEnvOracle(spec, E)
    for t in range(34):
        rows = b.staging.cpu().numpy()
        a.step(0.3)
        b.step(0.3)
        if t == 14:
            a.flush_td()
            b.flush_td()
        c = t % 10
        act = b.act.cpu().numpy().astype(np.int64)
        nxt, rew, done = ora.step(act)
        np.testing.assert_array_equal(b.store.obs[rows, c + 1].cpu().numpy(), nxt)
        if c == 0:
            np.testing.assert_array_equal(b.store.obs[rows, 0].cpu().numpy(), a.store.obs[rows, 0].cpu().numpy())
        np.testing.assert_array_equal(b.last_rew.cpu().numpy(), rew)
        np.testing.assert_array_equal(b.last_done.cpu().numpy().astype(bool), done)
        ora.reset_envs(done)
        if c == 9 or t == 14:
            for i, (x, y) in enumerate(zip(_state(a), _state(b))):
                assert torch.equal(x, y), (t, i)
    a.flush_td()
    b.flush_td()
    for i, (x, y) in enumerate(zip(_state(a), _state(b))):
        assert torch.equal(x, y), ("end", i)
    pos, prev, grid, steps, apples = b.env.get_state()
    np.testing.assert_array_equal(pos, ora.pos)
    np.testing.assert_array_equal(prev, ora.prev)
    np.testing.assert_array_equal(grid, ora.grid)
    np.testing.assert_array_equal(steps, ora.steps)
    np.testing.assert_array_equal(apples, ora.apples)


def test_fused_region_graphs_match_eager():
    """bench.py's timed regions on the fused engine (30-step graph cycle): region graphs from several phases,
    chunk graphs and single-step graphs replay bit-identically to eager fused steps."""
    from minimarl.engine import RolloutEngine
    kw = dict(f1=64, g=64, h=64, chunk=10, capacity=2 * 2048, seed=23, device=DEV)
    a = RolloutEngine(2048, 8, fused=True, **kw)
    b = RolloutEngine(2048, 8, fused=True, **kw)
    for _ in range(77):
        a.step(0.3)
    a.flush_td()
    b.run_steps(3, 0.3)
    b.capture_region(20)
    b.run_steps(20, 0.3)                      # region graph, phase 3
    b.capture_region(20, start=b.t + 20)
    b.run_steps(20, 0.3)                      # phase 23
    b.run_steps(20, 0.3)                      # phase 13: chunk / single-step graphs
    b.run_steps(14, 0.3)
    b.flush_td()
    assert a.t == b.t == 77
    for i, (x, y) in enumerate(zip(_state(a), _state(b))):
        assert torch.equal(x, y), i


def test_learner_repacks_f32_image_and_rollout_refreshes_fp16x3_image():
    """After an Adam step the learner's graph repacks only the exact-f32 image (mm_qnet_pack_f32, what its own
    forward reads); the rollout's next full pack then refreshes the fp16x3 image and flags, so the packed buffer
    is bit-identical to a fresh full pack of the updated parameters."""
    from minimarl.engine import RolloutEngine
    from minimarl.learner import Mixer, QLearner
    from minimarl.qnet import AgentQNet
    eng = RolloutEngine(2048, 8, f1=64, g=64, h=64, chunk=10, capacity=4096, seed=3, device=DEV)
    for _ in range(2):
        eng.run_graph(0.5)
    N, D = eng.N, eng.D
    mix, tmix = Mixer(N, N * D, 64, 32, DEV, seed=7), Mixer(N, N * D, 64, 32, DEV, seed=7)
    lrn = QLearner(eng.behavior, eng.target, mix, tmix, batch=32, chunk=10, mode="qmix", device=DEV)
    lrn.capture_update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=1)
    before = eng.behavior.packed.clone()
    lrn.replay_update()
    lrn.replay_update()
    assert eng.behavior._h3_stale and not eng.behavior._dirty
    torch.cuda.synchronize()
    ref = AgentQNet(N, D, 5, 64, 64, 64, DEV)
    ref.flat.copy_(eng.behavior.flat)
    ref.mark_dirty()
    ref.pack()
    f32_len = (ref.packed.numel() - 64) // 2   # [f32 image | fp16x3 image | flags (padded to 64)]
    assert torch.equal(ref.packed[:f32_len], eng.behavior.packed[:f32_len])        # f32 image current
    assert not torch.equal(before[:f32_len], eng.behavior.packed[:f32_len])        # ... and it did change
    eng.step(0.1)                                                                   # the rollout's full pack
    torch.cuda.synchronize()
    assert not eng.behavior._h3_stale
    assert torch.equal(ref.packed, eng.behavior.packed)


def test_fused_step_not_taken_for_odd_band_counts():
    """2 or 6 agents give an odd row count (3 rows per band): no whole 16-byte grid pieces per env, so the engine
    keeps the two-launch step there (and refuses fused=True)."""
    from minimarl.engine import RolloutEngine
    for n in (2, 6):
        eng = RolloutEngine(2048, n, f1=64, g=32, h=32, chunk=10, capacity=4096, device=DEV)
        assert not eng.fused
        with pytest.raises(ValueError):
            RolloutEngine(2048, n, f1=64, g=32, h=32, chunk=10, capacity=4096, fused=True, device=DEV)


def test_fused_step_skips_corrupt_staging_row():
    """Guard rail: a staging row outside the chunk store (a corrupt PER slot map) is never written through by the
    fused step (obs store, chunk-start slot 0, the folded TD / act / rew / done store) and sets the engine's sticky
    error bit 0, which check_errors() raises; every other env's stores match an uncorrupted twin bit for bit."""
    from minimarl.engine import RolloutEngine
    kw = dict(f1=64, g=64, h=64, chunk=10, capacity=2 * 2048, seed=31, device=DEV)
    a = RolloutEngine(2048, 8, fused=True, **kw)
    b = RolloutEngine(2048, 8, fused=True, **kw)
    for _ in range(3):
        a.step(0.3)
        b.step(0.3)
    a.check_errors()
    bad = [5, 700, 2047]
    good_rows = b.staging.clone()
    with torch.no_grad():
        b.staging[5] = b.store.rows + 100
        b.staging[700] = -3
        b.staging[2047] = b.store.rows
    for _ in range(4):
        a.step(0.3)
        b.step(0.3)
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="corrupt staging row"):
        b.check_errors()
    b.check_errors()                                    # cleared
    keep = torch.ones(2048, dtype=torch.bool)
    keep[bad] = False
    rows = good_rows.cpu()[keep]
    for x, y in ((a.store.obs, b.store.obs), (a.store.act, b.store.act), (a.store.rew, b.store.rew),
                 (a.store.done, b.store.done)):
        assert torch.equal(x.cpu()[rows], y.cpu()[rows])
    assert torch.equal(a.chunk_td.cpu()[keep], b.chunk_td.cpu()[keep])
    # corrupt rows are never handed on as cur_row
    assert not (b.cur_row.cpu()[bad] >= b.store.rows).any() and not (b.cur_row.cpu()[bad] < -1).any()
