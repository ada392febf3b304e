"""Integrated QMIX / VDN rollout-and-learn trainer on lockstep device envs.

Maps the reference's training loops (vdn/main.py:80-198, qmix/main.py:100-277) onto the device
engine:

* warm-up (vdn/main.py:80-125): epsilon = 1 rollout until the prioritized replay holds
  ``buffer_limit`` chunks;
* training episode ``ep`` (vdn/main.py:127-186): epsilon = max(min, max - (max - min) * ep / anneal)
  (:133-134); ``max_step`` lockstep steps of all ``n_envs`` envs (rollout + TD priorities + chunk
  inserts, HIP-graph replays); then ``update_iter`` learner updates (``Target_Dqn.train`` /
  ``Train_dqn.train``, :179-180, each = PER sample -> BPTT -> clip/Adam -> reprioritize, replayed
  HIP graphs); every ``update_target_interval`` episodes (at episode 0 too) the target AGENT net
  is hard-synced (:184-186; QMIX keeps its target mixer, qmix/main.py:255-256); every
  ``test_interval`` episodes greedy test episodes (``Test.execute``, :188-190) on separate envs.

One lockstep "episode" advances every env by ``max_step`` steps (envs whose episode ended early
auto-reset, so env episodes are not aligned; chunks span episode boundaries like the reference's
global ``count_step``, :151-167). The update-to-data ratio is the reference's: ``update_iter``
updates of ``batch_size`` chunks per ``max_step`` steps — per env-shard and rank.

Data parallel: one trainer per rank on its own env shard and replay; the flat
gradient is all-reduced (``grad_allreduce``) between the captured backward and the clip/Adam graph,
so the replicas stay identical (rank 0's initial parameters are broadcast by the caller).
"""
import os
import time

import torch

from ._lib import check, lib
from .config import QTrainConfig
from .engine import RolloutEngine
from .evaluate import QEvaluator
from .learner import Mixer, QLearner
from .qnet import ptr, stream_handle


def _ranks_share_device(world):
    """True when this node runs more ranks than it has GPUs (LOCAL_WORLD_SIZE from the launcher, else WORLD_SIZE)."""
    local = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    return local > max(1, torch.cuda.device_count())


class QTrainer:
    def __init__(self, cfg: QTrainConfig, device="cuda", rank=0, grad_allreduce=None, world=1, track_score=True):
        self.cfg = c = cfg
        self.device = torch.device(device)
        assert c.n_actions == 5, "the gridworld / switch envs have 5 actions"
        assert c.algo in ("vdn", "vdn_double", "qmix", "qmix_min")
        if c.buffer_limit < c.n_envs:
            raise ValueError(f"buffer_limit ({c.buffer_limit} chunks) must hold one chunk per env ({c.n_envs})")
        persistent = c.persistent
        if persistent is None and world > 1 and _ranks_share_device(world):
            # several ranks on one GPU: their kernels run beside each other, and the chunk-persistent launch needs
            # every CU for its own blocks (its hand-off waits would expire: include/minimarl.h, co-residency)
            persistent = False
        per_kwargs = dict(alpha=c.alpha, beta=c.beta, eps=c.eps, step_weight=c.step_weight,
                          use_step_weight=c.use_step_weight and c.per_flavor == "vdn",
                          update_alpha_beta=c.update_alpha_beta, max_episodes=c.max_episodes,
                          update_iter=c.update_iter)
        self.eng = RolloutEngine(c.n_envs, c.n_agents, n_actions=c.n_actions, f1=c.f1, g=c.g, h=c.h,
                                 chunk=c.chunk_size, capacity=c.buffer_limit, gamma=c.gamma, max_steps=c.max_step,
                                 step_cost=c.step_cost, full_observable=c.full_observable,
                                 per_flavor=c.per_flavor, per_kwargs=per_kwargs, seed=c.seed + 7919 * rank,
                                 env=c.env, persistent=persistent, device=self.device)
        eng = self.eng
        # the behavior net's init does not depend on the rank (same seed): replicas start identical
        eng.behavior.init_default(c.seed)
        eng.sync_target()
        self.mix = self.tmix = None
        if c.algo in ("qmix", "qmix_min"):
            S = c.n_agents * eng.D
            self.mix = Mixer(c.n_agents, S, c.mixer_hidden, c.mixer_k1, self.device, seed=c.seed + 1)
            self.tmix = Mixer(c.n_agents, S, c.mixer_hidden, c.mixer_k1, self.device)
            self.tmix.flat.copy_(self.mix.flat)          # qmix/_utils.py:40-41 init sync
        self.learner = QLearner(eng.behavior, eng.target, self.mix, self.tmix, batch=c.batch_size,
                                chunk=c.chunk_size, gamma=c.gamma, lr=c.lr, grad_clip=c.grad_clip_norm, mode=c.algo,
                                device=self.device, reference_compat=c.reference_compat)
        self.allreduce = grad_allreduce
        if grad_allreduce is not None:
            self.learner._graph_scale = 1.0 / world
        self.rank, self.world = rank, world
        self.evaluator = None
        if c.test_interval and c.test_envs > 0:
            self.evaluator = QEvaluator(c.test_envs, c.n_agents, c.max_step, c.step_cost, c.full_observable,
                                        c.gamma, env=c.env, device=self.device)
        self.track_score = track_score
        self.ep_ret = torch.zeros(c.n_envs, device=self.device)
        self.score_acc = torch.zeros(2, dtype=torch.float64, device=self.device)
        self._rows = torch.empty(c.n_envs, dtype=torch.int64, device=self.device)
        self.episode = 0
        self.warmed = False
        self.updates_captured = False
        self.history = []

    # ------------------------------------------------------------------ rollout
    def _rollout(self, n_steps, epsilon):
        """n_steps lockstep steps; whole chunks are replayed one graph at a time so each stored chunk's
        rewards feed the training score (mm_chunk_score)."""
        eng, C = self.eng, self.eng.C
        eng.set_epsilon(epsilon)
        G = eng.graph_steps()
        left = int(n_steps)
        while left > 0:
            if eng.t % C == 0 and left >= C and self.track_score:
                self._rows.copy_(eng.staging)            # rows this chunk is written into
                if G == C:
                    eng.run_graph()
                else:                                    # graph cycle of several chunks: one region graph per chunk
                    eng.run_region(C)
                check(lib().mm_chunk_score(eng.E, C, eng.N, ptr(eng.store.rew), ptr(eng.store.done),
                                           ptr(self._rows), ptr(self.ep_ret), ptr(self.score_acc),
                                           stream_handle(self.device)), "chunk_score")
                left -= C
            else:
                k = G if (eng.t % G == 0 and left >= G) else 1
                eng.run_steps(k)
                left -= k

    def warmup(self):
        """vdn/main.py:80-125: epsilon = 1 until the replay holds buffer_limit chunks."""
        eng = self.eng
        while len(eng.per) < eng.capacity:
            self._rollout(eng.graph_steps(), 1.0)
        self.score_acc.zero_()                          # the train score counts training episodes only
        self.warmed = True

    # ------------------------------------------------------------------ learning
    def _capture(self):
        eng = self.eng
        self.learner.capture_update(eng.per, eng.store, eng.env.reset_obs_ptr(), seed=self.cfg.seed + 104729 * self.rank,
                                    per_replay=self.cfg.update_iter if self.allreduce is None else 1)
        self.updates_captured = True

    def learn(self, epsilon):
        """``update_iter`` learner updates (Target_Dqn.train / Train_dqn.train, vdn/_train.py:56-101)."""
        if not self.updates_captured:
            self._capture()
        if self.cfg.algo == "vdn_double":
            self.learner.double_eps = epsilon if self.cfg.double_epsilon else 0.0
        self.learner.replay_updates(self.cfg.update_iter, self.allreduce)

    def train_episode(self):
        """One training episode (vdn/main.py:127-196), no host sync."""
        c, ep = self.cfg, self.episode
        if not self.warmed:
            self.warmup()
        eps = c.epsilon(ep)
        self._rollout(c.max_step, eps)
        self.learn(eps)
        if ep % c.update_target_interval == 0:
            self.learner.sync_target(mixer=False)
        self.episode += 1
        return eps

    def check_device_errors(self):
        """Raise if a device-side sticky error bit is set (the PER's out-of-range priority-update nodes, skipped on
        the device where the reference's tree write would raise); polled at the host syncs train() already has."""
        self.eng.per.check_errors()
        self.eng.check_errors()

    def train(self, n_episodes, log=None):
        """Run n_episodes training episodes; greedy tests every test_interval episodes (host sync); the device
        error words are polled at every test and at the end."""
        for _ in range(int(n_episodes)):
            eps = self.train_episode()
            ep = self.episode - 1
            if self.evaluator is not None and (ep + 1) % self.cfg.test_interval == 0:
                self.check_device_errors()
                rec = self.test()
                rec.update(episode=ep + 1, epsilon=eps, train_score=self.train_score(reset=True),
                           loss=float(self.learner.loss.item()), alpha=self.eng.per.alpha, beta=self.eng.per.beta)
                self.history.append(rec)
                if log is not None:
                    log(rec)
        self.check_device_errors()
        return self.history

    # ------------------------------------------------------------------ scores
    def train_score(self, reset=False):
        """Mean return of the training episodes finished since the last reset (None if none)."""
        s, n = (float(x) for x in self.score_acc.cpu())
        if reset:
            self.score_acc.zero_()
        return s / n if n > 0 else None

    def test(self):
        """Greedy test episodes (vdn/_test.py:22-50 score + TD^2 loss; qmix/_test.py:19-36 score)."""
        tgt = self.eng.target if self.cfg.algo.startswith("vdn") else None
        score, loss, _, _ = self.evaluator.run(self.eng.behavior, tgt)
        return {"test_score": score, "test_loss": loss}

    # ------------------------------------------------------------------ checkpoint (minimarl.checkpoint)
    def checkpoint_tensors(self, include_replay=True):
        """Learner (params, targets, Adam), replay (tree, slot map, annealed alpha / beta, sample counter),
        engine (hiddens, RNG step counter, current-obs rows, staging rows), env integer state and, with
        ``include_replay``, the chunk store itself — a resumed trainer continues bit-identically."""
        torch.cuda.synchronize(self.device)
        eng = self.eng
        ts, sc = self.learner.checkpoint_tensors()
        out = {"learner/" + k: v for k, v in ts.items()}
        pts, _ = eng.per.checkpoint_tensors()
        out.update({"per/" + k: v for k, v in pts.items()})
        ets, _ = eng.env.checkpoint_tensors()
        out.update({"env/" + k: v for k, v in ets.items()})
        for k, v in eng.state_buffers().items():
            out["engine/" + k] = v
        carry = eng.carry_state()   # (at a chunk boundary: lets another step mode resume the file)
        for k, v in (carry or {}).items():
            out["carry/" + k] = v
        if include_replay:
            for k in ("obs", "act", "rew", "done"):
                out["store/" + k] = getattr(eng.store, k)
        out["trainer/ep_ret"] = self.ep_ret
        out["trainer/score_acc"] = self.score_acc
        scalars = {"learner": sc, "t": eng.t, "chunks_inserted": eng.chunks_inserted, "primed": eng._primed,
                   "step_mode": eng.step_mode,
                   "td_pending": eng._td_pending, "episode": self.episode, "warmed": self.warmed,
                   "replay_saved": bool(include_replay)}
        return out, scalars

    def restore_tensors(self, ts, scalars):
        from .checkpoint import copy_into
        eng = self.eng
        # the step mode the file was written in (files before round 6 carry none: the chunk rings name chunk mode);
        # another mode can resume it only from the mode-independent carry of a chunk boundary
        saved_mode = scalars.get("step_mode") or ("chunk" if "engine/act_r" in ts else "fused or two-launch")
        if saved_mode != eng.step_mode and "carry/act" not in ts:
            raise ValueError(f"checkpoint was written by the {saved_mode!r} rollout step mode mid-chunk "
                             f"(t = {scalars['t']}); this engine runs {eng.step_mode!r}. Resume it with the same mode "
                             f"(QTrainConfig.persistent=True for 'chunk', False for the others) or save at a chunk "
                             f"boundary, where any mode can resume it")
        self.learner.restore_tensors({k[8:]: v for k, v in ts.items() if k.startswith("learner/")}, scalars["learner"])
        eng.per.restore_tensors({k[4:]: v for k, v in ts.items() if k.startswith("per/")})
        # the step count first: the fused step double-buffers the env state by step parity (env.state_buffer()
        # = t % 2), so the restored state must land in the buffer the next step reads
        eng.t, eng.chunks_inserted = int(scalars["t"]), int(scalars["chunks_inserted"])
        eng.env.restore_tensors({k[4:]: v for k, v in ts.items() if k.startswith("env/")})
        if saved_mode == eng.step_mode:
            for k, v in eng.state_buffers().items():
                if "engine/" + k not in ts:
                    raise ValueError(f"checkpoint lacks engine/{k}")
                copy_into(v, ts["engine/" + k], k)
        else:   # another step mode, saved at a chunk boundary: the shared buffers plus the mode-independent carry
            for k in eng.COMMON_STATE:
                if k != "staging_all":
                    copy_into(getattr(eng, k), ts["engine/" + k], k)
            src_set = (eng.t // eng.C) % eng.S if saved_mode == "chunk" else 0
            eng.load_carry({k[6:]: v for k, v in ts.items() if k.startswith("carry/")}, copy_into,
                           ts["engine/staging_all"], src_set)
        if scalars.get("replay_saved"):
            for k in ("obs", "act", "rew", "done"):
                copy_into(getattr(eng.store, k), ts["store/" + k], k)
        copy_into(self.ep_ret, ts["trainer/ep_ret"], "ep_ret")
        copy_into(self.score_acc, ts["trainer/score_acc"], "score_acc")
        eng._primed = bool(scalars["primed"])
        eng._td_pending = bool(scalars["td_pending"]) and saved_mode == eng.step_mode
        eng._eps_host = None
        eng.behavior.mark_dirty()
        eng.target.mark_dirty()
        self.episode, self.warmed = int(scalars["episode"]), bool(scalars["warmed"])
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ throughput
    def timed(self, n_episodes):
        """Wall time of n_episodes training episodes (rollout + learner), synchronised."""
        torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        for _ in range(int(n_episodes)):
            self.train_episode()
        torch.cuda.synchronize(self.device)
        return time.perf_counter() - t0
