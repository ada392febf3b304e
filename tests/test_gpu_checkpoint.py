"""GPU: checkpoint / resume (minimarl.checkpoint) — a learner restored from a checkpoint continues
bit-identically to the one that kept running (QMIX QLearner, offpolicy OffQMix, MAPPO trainer)."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
pytestmark = pytest.mark.gpu
DEV = "cuda"


def _qlearner(seed_off=0):
    from minimarl.learner import Mixer, QLearner
    from minimarl.qnet import AgentQNet
    N, D, A, B, C = 4, 47, 5, 16, 5
    beh = AgentQNet(N, D, A, 64, 64, 64, DEV, seed=1 + seed_off)
    tgt = AgentQNet(N, D, A, 64, 64, 64, DEV, seed=2 + seed_off)
    mix = Mixer(N, N * D, 64, 32, DEV, seed=3 + seed_off)
    tmix = Mixer(N, N * D, 64, 32, DEV, seed=4 + seed_off)
    return QLearner(beh, tgt, mix, tmix, batch=B, chunk=C, mode="qmix", device=DEV), (N, D, A, B, C)


def _q_batch(dims, seed):
    N, D, A, B, C = dims
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(B, C, N, D, generator=g), torch.randint(0, A, (B, C, N), generator=g).float(),
            torch.randn(B, C, N, generator=g) * 0.5, torch.rand(B, C, N, D, generator=g),
            (torch.rand(B, C, 1, generator=g) < 0.2).float(), torch.rand(B, 1, generator=g) * 0.5 + 0.5)


def test_qlearner_resume_is_bit_identical(tmp_path):
    from minimarl.checkpoint import load_checkpoint, save_checkpoint
    a, dims = _qlearner()
    for it in range(2):
        a.load_batch(*_q_batch(dims, it))
        a.train_step(a._obs_buf, a._obs_buf)
    path = str(tmp_path / "q.safetensors")
    save_checkpoint(path, learner=a)
    b, _ = _qlearner(seed_off=10)                 # different init: everything must come from the file
    meta = load_checkpoint(path, learner=b)
    assert meta["learner"]["scalars"]["mode"] == "qmix"
    for L in (a, b):
        L.load_batch(*_q_batch(dims, 7))
        L.train_step(L._obs_buf, L._obs_buf)
    torch.cuda.synchronize()
    assert torch.equal(a.P, b.P) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v)
    assert torch.equal(a.loss, b.loss)


def test_offq_resume_is_bit_identical(tmp_path):
    from minimarl.synth import offq_episode_batch as make_batch
    from minimarl.checkpoint import load_checkpoint, save_checkpoint
    from minimarl.offq import OffQMix
    N, T, B, D, A = 2, 9, 6, 47, 5
    a = OffQMix(N, D, A, T, B, seed=1)
    rng = np.random.default_rng(3)
    pid = "policy_0"

    def batch():
        obs, share, acts, rew, dones, dn = make_batch(rng, N, T, B, D, A)
        w = (0.5 + rng.random(B)).astype(np.float32)
        return ({pid: obs}, {pid: share}, {pid: acts}, {pid: rew}, {pid: dones}, {pid: dn}, {pid: None}, w, None)

    for _ in range(2):
        a.train_policy_on_batch(batch())
        a.soft_target_updates()
    path = str(tmp_path / "o.safetensors")
    save_checkpoint(path, offq=a)
    b = OffQMix(N, D, A, T, B, seed=99)
    load_checkpoint(path, offq=b)
    bt = batch()
    for tr in (a, b):
        tr.train_policy_on_batch(bt)
        tr.soft_target_updates()
    torch.cuda.synchronize()
    for k in ("P", "PT", "m", "v", "step"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k


def test_mappo_resume_is_bit_identical(tmp_path):
    from minimarl.checkpoint import load_checkpoint, save_checkpoint
    from minimarl.env import VecEnv
    from minimarl.mappo import MappoPolicy, MappoRunner
    runs = []
    for seed in (5, 6):
        env = VecEnv(64, 2, max_steps=20, device=DEV)
        pol = MappoPolicy(env.obs_dim, 5, 32, DEV, seed=seed)
        runs.append(MappoRunner(env, pol, T=20, L=5, ppo_epoch=2, seed=0))
    a, b = runs
    a.warmup()
    a.run_episode()
    path = str(tmp_path / "m.safetensors")
    save_checkpoint(path, mappo=a.trainer)
    load_checkpoint(path, mappo=b.trainer)
    # same data for both: train b's trainer on a copy of a's next buffer
    a.rollout()
    a.compute()
    for k in ("obs", "rnn_states", "rnn_states_critic", "value_preds", "returns", "actions", "action_log_probs",
              "rewards", "masks", "active_masks"):
        getattr(b.buf, k).copy_(getattr(a.buf, k))
    a.trainer.train(a.buf)
    b.trainer.train(b.buf)
    torch.cuda.synchronize()
    assert torch.equal(a.p.actor.flat, b.p.actor.flat)
    assert torch.equal(a.p.critic.flat, b.p.critic.flat)
    assert torch.equal(a.trainer.vn, b.trainer.vn)


def test_trainer_resume_bit_identical(tmp_path):
    """QTrainer checkpoint = learner + replay (tree, slot map, annealed alpha / beta, sample counter) +
    engine hiddens / RNG counters + env state + chunk store: a resumed trainer's next episodes (rollout,
    PER sampling, updates, reprioritisation) are bit-identical to the uninterrupted run."""
    from minimarl.checkpoint import load_checkpoint, save_checkpoint
    from minimarl.config import QTrainConfig
    from minimarl.train import QTrainer
    cfg = QTrainConfig(algo="qmix", n_envs=64, n_agents=4, full_observable=False, buffer_limit=512, max_step=20,
                       update_iter=3, update_target_interval=2, test_interval=0, test_envs=0,
                       epsilon_anneal_episode=10, seed=9)
    a = QTrainer(cfg, device=DEV)
    for _ in range(3):
        a.train_episode()
    path = str(tmp_path / "trainer.safetensors")
    save_checkpoint(path, trainer=a)
    alpha_saved = a.eng.per.alpha
    for _ in range(2):
        a.train_episode()
    b = QTrainer(cfg, device=DEV)
    load_checkpoint(path, trainer=b)
    assert b.episode == 3 and b.eng.t == a.eng.t - 40 and abs(b.eng.per.alpha - alpha_saved) < 1e-15
    for _ in range(2):
        b.train_episode()
    torch.cuda.synchronize()
    for x, y in [(a.learner.P, b.learner.P), (a.learner.m, b.learner.m), (a.eng.target.flat, b.eng.target.flat),
                 (a.eng.per.tree(), b.eng.per.tree()), (a.eng.per.slot_rows(), b.eng.per.slot_rows()),
                 (a.eng.store.obs, b.eng.store.obs), (a.eng.store.act, b.eng.store.act), (a.eng.h, b.eng.h),
                 (a.score_acc, b.score_acc)]:
        assert torch.equal(x, y)
    assert a.eng.per.alpha == b.eng.per.alpha and a.eng.per.alpha > cfg.alpha


def test_trainer_resume_bit_identical_fused_odd_step(tmp_path):
    """The same at the fused one-launch step's geometry (E = 2048, 4 agents, local obs), checkpointed at an ODD
    step count: the fused step double-buffers the env state by step parity, so the restore must write the state
    into the buffer the next step reads (the restore used to run before the step count was set)."""
    from minimarl.checkpoint import load_checkpoint, save_checkpoint
    from minimarl.config import QTrainConfig
    from minimarl.train import QTrainer
    cfg = QTrainConfig(algo="qmix", n_envs=2048, n_agents=4, full_observable=False, buffer_limit=4096, max_step=13,
                       update_iter=2, update_target_interval=2, test_interval=0, test_envs=0,
                       epsilon_anneal_episode=10, seed=11, persistent=False)
    a = QTrainer(cfg, device=DEV)
    assert a.eng.fused
    a.train_episode()
    assert a.eng.t % 2 == 1
    path = str(tmp_path / "trainer_fused.safetensors")
    save_checkpoint(path, trainer=a)
    for _ in range(2):
        a.train_episode()
    b = QTrainer(cfg, device=DEV)
    load_checkpoint(path, trainer=b)
    assert b.eng.t == a.eng.t - 26 and b.eng.t % 2 == 1
    for _ in range(2):
        b.train_episode()
    torch.cuda.synchronize()
    for x, y in [(a.learner.P, b.learner.P), (a.eng.per.tree(), b.eng.per.tree()),
                 (a.eng.per.slot_rows(), b.eng.per.slot_rows()), (a.eng.store.obs, b.eng.store.obs),
                 (a.eng.store.act, b.eng.store.act), (a.eng.h, b.eng.h), (a.eng.ht, b.eng.ht),
                 (a.score_acc, b.score_acc)]:
        assert torch.equal(x, y)
    for x, y in zip(a.eng.env.get_state(), b.eng.env.get_state()):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("src_persistent", [True, False])
def test_trainer_resume_across_step_modes(tmp_path, src_persistent):
    """the engine state a checkpoint holds depends on the rollout step mode picked for the device (chunk
    rings vs fused ping-pong buffers). A file saved at a chunk boundary also carries the mode-independent step state
    (act / Q(a) of step t, done of step t - 1, RNG counter), so a trainer running the OTHER mode resumes it and
    continues bit-identically to the uninterrupted run (the two modes are bit-identical step for step); a file saved
    mid-chunk names both modes in its error."""
    from minimarl.checkpoint import load_checkpoint, save_checkpoint
    from minimarl.config import QTrainConfig
    from minimarl.train import QTrainer
    kw = dict(algo="qmix", n_envs=2048, n_agents=4, full_observable=False, buffer_limit=4096, max_step=20,
              update_iter=2, update_target_interval=2, test_interval=0, test_envs=0, epsilon_anneal_episode=10, seed=13)
    a = QTrainer(QTrainConfig(persistent=src_persistent, **kw), device=DEV)
    assert a.eng.chunked == src_persistent
    a.train_episode()
    assert a.eng.t % 10 == 0
    path = str(tmp_path / "trainer_mode.safetensors")
    save_checkpoint(path, trainer=a)
    for _ in range(2):
        a.train_episode()
    b = QTrainer(QTrainConfig(persistent=not src_persistent, **kw), device=DEV)
    assert b.eng.step_mode != a.eng.step_mode
    b.train_episode()   # a different history before the restore
    load_checkpoint(path, trainer=b)
    assert b.eng.t == a.eng.t - 40
    for _ in range(2):
        b.train_episode()
    torch.cuda.synchronize()
    # (the modes place chunks in different physical store rows — chunk mode rotates its staging sets — so the PER's
    # chunks are compared through the slot maps)
    ra, rb = a.eng.per.slot_rows().long(), b.eng.per.slot_rows().long()
    for x, y in [(a.learner.P, b.learner.P), (a.eng.per.tree(), b.eng.per.tree()),
                 (a.eng.store.obs[ra], b.eng.store.obs[rb]), (a.eng.store.act[ra], b.eng.store.act[rb]),
                 (a.eng.store.rew[ra], b.eng.store.rew[rb]), (a.eng.h, b.eng.h), (a.eng.ht, b.eng.ht),
                 (a.eng.chunk_td, b.eng.chunk_td), (a.score_acc, b.score_acc)]:
        assert torch.equal(x, y)
    for x, y in zip(a.eng.env.get_state(), b.eng.env.get_state()):
        assert np.array_equal(x, y)
    # mid-chunk: the other mode refuses with both modes named
    a.eng.run_steps(3, 0.1)
    save_checkpoint(path, trainer=a)
    with pytest.raises(ValueError, match="step mode"):
        load_checkpoint(path, trainer=b)
