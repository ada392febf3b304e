"""Greedy evaluation episodes vs oracle loops of the reference's test code.

QEvaluator: vdn/_test.py Test.execute (score + sum of cal_td_error^2 against the target net) and
qmix/_test.py Test.execute (score); MappoEvaluator: magym_runner.py eval (deterministic actor,
summed episode reward). E test envs run one episode each. Small E keeps the exact-f32 forward,
so the greedy trajectories match the oracle's; scores are sums of exactly representable
rewards (rtol 1e-6), td^2 sums rtol 1e-4.
"""
import numpy as np
import pytest
import torch

from oracle import mappo as om
from oracle import nets
from oracle.env import EnvSpec, VecEnvOracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _oracle_q_episode(P, T, E, N, gamma, max_steps=100):
    ora = VecEnvOracle(EnvSpec(N, max_steps), E)
    obs = torch.tensor(ora.observe())
    H = P["Whh"].shape[2]
    h, ht = torch.zeros(E, N, H), torch.zeros(E, N, H)
    active = np.ones(E, bool)
    score, loss = np.zeros(E, np.float32), np.zeros(E, np.float32)
    for _ in range(max_steps):
        q, h = nets.agent_forward(P, obs, h)
        act = q.argmax(2)
        nxt, rew, done = ora.step(act.numpy())
        tq, ht = nets.agent_forward(T, torch.tensor(nxt), ht)
        qs = q.gather(2, act.unsqueeze(-1)).squeeze(-1).sum(1)
        sr = torch.tensor(rew).sum(1)
        td = (sr + (1 - torch.tensor(done, dtype=torch.float32)) * gamma * tq.max(2)[0].sum(1) - qs).abs()
        score[active] += sr.numpy()[active]
        loss[active] += (td * td).numpy()[active]
        active &= ~done
        obs = torch.tensor(nxt)
    return score, loss


@pytest.mark.parametrize("n_agents", [2, 8])
def test_q_greedy_eval_vs_oracle(n_agents):
    from minimarl.evaluate import QEvaluator
    from minimarl.qnet import AgentQNet
    E = 96
    beh = AgentQNet(n_agents, 47, 5, 64, 32, 32, DEV, seed=11)
    tgt = AgentQNet(n_agents, 47, 5, 64, 32, 32, DEV, seed=12)
    ev = QEvaluator(E, n_agents, 100, device=DEV)
    mean_s, mean_l, score, loss = ev.run(beh, tgt)
    P = {k: v.detach().cpu().clone() for k, v in beh.params().items()}
    T = {k: v.detach().cpu().clone() for k, v in tgt.params().items()}
    os_, ol = _oracle_q_episode(P, T, E, n_agents, 0.99)
    np.testing.assert_allclose(score.cpu().numpy(), os_, rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(loss.cpu().numpy(), ol, rtol=1e-4, atol=1e-4)
    assert abs(mean_s - os_.mean()) < 1e-3
    # QMIX's Test.execute: the score only
    s2, l2, _, _ = QEvaluator(E, n_agents, 100, device=DEV).run(beh)
    assert l2 is None and abs(s2 - mean_s) < 1e-4


def test_mappo_deterministic_eval_vs_oracle():
    from minimarl.evaluate import MappoEvaluator
    from minimarl.mappo import MappoPolicy
    E, N = 64, 8
    pol = MappoPolicy(47, 5, 32, DEV, seed=4)
    mean, score = MappoEvaluator(E, N, 100, device=DEV).run(pol)
    PA = om.net_from_state({k: v.numpy() for k, v in pol.actor.state_dict().items()}, "", "actor")
    ora = VecEnvOracle(EnvSpec(N, 100), E)
    obs = torch.tensor(ora.observe()).reshape(E * N, -1)
    h = torch.zeros(E * N, 32)
    active = np.ones(E, bool)
    sc = np.zeros(E, np.float32)
    for _ in range(100):
        logits, h = om.net_step(PA, obs, h, torch.ones(E * N, 1))
        act = logits.argmax(-1).view(E, N)
        nxt, rew, done = ora.step(act.numpy())
        sc[active] += rew.sum(1)[active]
        active &= ~done
        obs = torch.tensor(nxt).reshape(E * N, -1)
    np.testing.assert_allclose(score.cpu().numpy(), sc, rtol=1e-6, atol=1e-5)
    assert abs(mean - sc.mean()) < 1e-3
