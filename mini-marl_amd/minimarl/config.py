"""Typed configuration of the QMIX / VDN trainer and presets for BASELINE.json's five configs.

Field names and defaults follow the reference's argparse flags (vdn/_config.py, qmix/_config.py;
``buffer_limit`` counts chunks, ``max_episodes`` / ``epsilon_anneal_episode`` count training
iterations = reference episodes). The reference's ``type=bool`` flags become
real booleans here. Lockstep-specific fields: ``n_envs`` (envs stepped together; one training
iteration = ``max_step`` lockstep steps of all of them) and ``test_envs`` (greedy test episodes run
in parallel, the reference's ``test_episodes``).
"""
from dataclasses import dataclass, field, replace
from typing import Optional


@dataclass
class QTrainConfig:
    algo: str = "vdn"                   # "vdn" | "vdn_double" | "qmix" | "qmix_min"
    # --env_name (vdn/_config.py:19-24 "ma_gym:Checkers-v0"; qmix/_config.py:14-19 "ma_gym:Switch2-v0"):
    # "checkers" | "switch"
    env: str = "checkers"
    n_envs: int = 32
    n_agents: int = 2
    full_observable: bool = True        # vdn/main.py:61-62 (Checkers full obs); QMIX uses partial obs
    max_step: int = 100                 # --max_step
    step_cost: float = -0.01            # --step_cost
    n_actions: int = 5
    # rollout step mode (RolloutEngine persistent=): None = the chunk-persistent launches where they fit, False = one
    # launch per step (e.g. several processes sharing one GPU: the chunk kernel needs every CU for its own blocks)
    persistent: Optional[bool] = None
    # agent Q_Net (vdn/_network.py:14-19): D -> f1 -> g (ReLU) -> GRUCell(g, h) -> A
    f1: int = 64
    g: int = 32
    h: int = 32
    # QMIX Mix_Net (qmix/_network.py:172-197): GRUCell(state, mixer_hidden), hypernet width k1
    mixer_hidden: int = 32
    mixer_k1: int = 32
    # learner (vdn/_config.py:84-121)
    lr: float = 1e-3
    gamma: float = 0.99
    batch_size: int = 32
    chunk_size: int = 10
    update_iter: int = 10
    grad_clip_norm: float = 5.0
    # exploration / target sync (vdn/_config.py:60-80,112-116)
    max_epsilon: float = 0.8
    min_epsilon: float = 0.05
    epsilon_anneal_episode: int = 15000
    update_target_interval: int = 20
    max_episodes: int = 30000
    # prioritized replay (vdn/_config.py:155-191)
    buffer_limit: int = 10000
    eps: float = 1e-6
    alpha: float = 0.4
    beta: float = 0.4
    update_alpha_beta: bool = True
    use_step_weight: bool = True
    step_weight: float = 0.99
    # evaluation (vdn/_config.py:145-152)
    test_interval: int = 1
    test_envs: int = 1
    double_epsilon: bool = True         # vdn_double: the double net explores with the current epsilon
    # True: the reference's TD target w * (sum r + N * gamma * (1-d) * Q'_tot);
    # False: sum r + gamma * (1-d) * Q'_tot (qmix/qmix.py:215-217)
    reference_compat: bool = True
    seed: int = 42

    @property
    def per_flavor(self):
        return "vdn" if self.algo.startswith("vdn") else "qmix"

    def epsilon(self, episode):
        """vdn/main.py:133-134 (qmix/main.py:173-177): linear anneal per training episode."""
        return max(self.min_epsilon, self.max_epsilon - (self.max_epsilon - self.min_epsilon)
                   * (episode / self.epsilon_anneal_episode))


def vdn_reference():
    """vdn/_config.py defaults: Checkers 2 agents, full obs (D = 94), GRU-32, PER alpha = beta = 0.4."""
    return QTrainConfig()


def qmix_reference():
    """qmix/_config.py defaults: the Switch2 env (2 agents, partial obs), alpha 0.8, beta 0.2, buffer
    1000, eps 0.9 -> 0.05 over 60000 episodes, 10 test episodes every 10 episodes."""
    return QTrainConfig(algo="qmix", env="switch", full_observable=False, max_epsilon=0.9, epsilon_anneal_episode=60000,
                        max_episodes=100000, buffer_limit=1000, alpha=0.8, beta=0.2, use_step_weight=False,
                        test_interval=10, test_envs=10)


@dataclass
class MappoTrainConfig:
    """mappo/_config.py values on the hot path (rmappo, shared policy, recurrent, 1 minibatch)."""
    n_envs: int = 4096
    n_agents: int = 8
    episode_length: int = 100
    hidden: int = 32
    data_chunk_length: int = 5
    ppo_epoch: int = 15
    clip_param: float = 0.2
    huber_delta: float = 10.0
    entropy_coef: float = 0.01
    value_loss_coef: float = 0.5
    max_grad_norm: float = 0.5
    lr: float = 1e-4
    critic_lr: float = 1e-4
    opti_eps: float = 1e-5
    gamma: float = 0.99
    gae_lambda: float = 0.95
    seed: int = 1


@dataclass
class Preset:
    name: str
    description: str
    q: QTrainConfig = None
    mappo: MappoTrainConfig = None
    gpus: int = 1
    extra: dict = field(default_factory=dict)


def presets():
    """BASELINE.json configs[0..4] (SURVEY 8d shapes)."""
    cfg2 = replace(qmix_reference(), env="checkers", n_agents=8, n_envs=4096, g=64, h=64, mixer_hidden=64,
                   buffer_limit=65536)
    return {
        "cfg1": Preset("cfg1", "VDN on 2-agent cooperative gridworld, 32 parallel envs (D = 94 full obs, GRU-32)",
                       q=replace(vdn_reference(), n_envs=32)),
        "cfg2": Preset("cfg2", "QMIX 8-agent gridworld, 4096 envs, GRU-64 agents + Hm-64 hypernet mixer, 1 GPU",
                       q=cfg2),
        "cfg3": Preset("cfg3", "MAPPO 8-agent, 4096 envs, shared actor-critic, device GAE, 1 GPU",
                       mappo=MappoTrainConfig()),
        "cfg4": Preset("cfg4", "QMIX 8-agent, 32768 envs sharded 4096 per GPU over 8 GPUs, RCCL gradient all-reduce",
                       q=cfg2, gpus=8),
        "cfg5": Preset("cfg5", "QMIX SMAC-scale 27 agents, obs 300, 36 actions, 8192 envs, GRU-32, 8 GPUs "
                               "(no env of that shape exists: synthetic observations)",
                       q=replace(qmix_reference(), env="checkers", n_agents=27, n_envs=8192, n_actions=36, g=32, h=32,
                                 mixer_hidden=32, buffer_limit=65536),
                       gpus=8, extra={"obs_dim": 300}),
    }
