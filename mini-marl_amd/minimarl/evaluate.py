"""Greedy evaluation episodes on device.

Replaces the reference's test loops, one env stepped serially per episode:
  * ``Test.execute`` of VDN (vdn/_test.py:22-50): greedy actions (epsilon 0) from the behavior
    net, score = mean episode return, loss = mean over episodes of sum_t td_t^2 with td from
    ``cal_td_error`` against the target net (vdn/_utils.py:44-52);
  * ``Test.execute`` of QMIX (qmix/_test.py:19-36): the score only;
  * ``MAGYM_Runner.eval`` (mappo/runner/shared/magym_runner.py:198-241): deterministic actions
    (Categorical mode) of the shared actor, the episode's summed reward.
Here E test envs run one episode each in lockstep (one episode per env instead of
``test_episodes`` sequential episodes); each env stops accumulating at its own ``done``.
"""
import ctypes

import torch

from ._lib import MM_MAPPO_ROLLOUT, MappoFwdArgs, check, lib
from .env import VecEnv, make_env
from .qnet import ptr, stream_handle


class QEvaluator:
    """Greedy episodes of a VDN / QMIX agent net (AgentQNet) on a dedicated test VecEnv."""

    def __init__(self, n_envs, n_agents, max_steps=100, step_cost=-0.01, full_observable=False, gamma=0.99,
                 env="checkers", device="cuda"):
        self.env = make_env(env, n_envs, n_agents, max_steps, step_cost, full_observable, device=device)
        self.switch = env == "switch"
        self.E, self.N, self.max_steps, self.gamma = int(n_envs), int(n_agents), int(max_steps), float(gamma)
        self.device = torch.device(device)

    @torch.no_grad()
    def run(self, behavior, target=None):
        """-> (mean score, mean sum of td^2 or None, per-env scores [E], per-env losses [E] or None)."""
        E, dev = self.E, self.device
        obs = self.env.reset()
        h = torch.zeros(E, self.N, behavior.H, device=dev)
        ht = torch.zeros(E, self.N, target.H, device=dev) if target is not None else None
        active = torch.ones(E, dtype=torch.uint8, device=dev)
        score = torch.zeros(E, device=dev)
        loss = torch.zeros(E, device=dev) if target is not None else None
        for _ in range(self.max_steps):        # every env is done by max_steps
            act, qsel, h, _ = behavior.act(obs, h, 0.0)
            out = self.env.step(act)
            nxt, rew, done = (out[0], out[1], out[3]) if self.switch else out   # switch: all(agent done)
            maxq = None
            if target is not None:
                maxq, ht = target.max_q(nxt, ht)
            check(lib().mm_eval_accum(E, self.N, self.gamma, ptr(rew), ptr(done),
                                      ptr(qsel) if target is not None else None, ptr(maxq), ptr(active), ptr(score),
                                      ptr(loss), stream_handle(dev)), "eval_accum")
            obs = nxt
        return (float(score.mean()), None if loss is None else float(loss.mean()), score,
                loss)


class MappoEvaluator:
    """Deterministic episodes of the shared MAPPO actor (MAGYM_Runner.eval)."""

    def __init__(self, n_envs, n_agents, max_steps=100, step_cost=-0.01, device="cuda"):
        self.env = VecEnv(n_envs, n_agents, max_steps, step_cost, False, device=device)
        self.E, self.N, self.max_steps = int(n_envs), int(n_agents), int(max_steps)
        self.device = torch.device(device)

    @torch.no_grad()
    def run(self, policy):
        """-> (mean episode reward, per-env episode rewards [E])."""
        E, N, dev, H = self.E, self.N, self.device, policy.H
        R = E * N
        obs = self.env.reset().reshape(R, -1).contiguous()
        ha = torch.zeros(R, H, device=dev)
        ha2 = torch.empty_like(ha)
        hc = torch.zeros(R, H, device=dev)   # the critic runs alongside in the fused launch; unused
        hc2 = torch.empty_like(hc)
        lp = torch.empty(R, device=dev)
        v = torch.empty(R, device=dev)
        act = torch.empty(R, dtype=torch.int32, device=dev)
        active = torch.ones(E, dtype=torch.uint8, device=dev)
        score = torch.zeros(E, device=dev)
        for _ in range(self.max_steps):
            a = policy.rollout_args(obs, ha, hc, None, ha2, hc2, lp, v, act_out=act)
            a.mode, a.deterministic = MM_MAPPO_ROLLOUT, 1
            check(lib().mm_mappo_fwd(ctypes.byref(policy.dims), ctypes.byref(a), stream_handle(dev)), "mappo_fwd")
            nxt, rew, done = self.env.step(act.view(E, N))
            check(lib().mm_eval_accum(E, N, 0.0, ptr(rew), ptr(done), None, None, ptr(active), ptr(score), None,
                                      stream_handle(dev)), "eval_accum")
            obs = nxt.reshape(R, -1).contiguous()
            ha, ha2 = ha2, ha
            hc, hc2 = hc2, hc
        return float(score.mean()), score

