"""PyTorch custom ops of the hot path: ``torch.ops.minimarl.*`` and ``torch.classes.minimarl.*``.

Loads the in-tree op library (``lib/libminimarl_torch.so``, built from csrc/torch_ops.cpp by the
Makefile; it links libminimarl.so). The ops take caller-allocated outputs, run on the current HIP
stream without a host sync and raise RuntimeError on bad arguments:

  minimarl::qnet_pack(params, dims, packed!)
  minimarl::agent_q_fwd(packed, dims, obs, hidden, hidden_out!, q!)              Q_Net.forward
  minimarl::agent_q_act(packed, dims, obs, hidden, epsilon, u?, rand_act?, seed, counter,
                        hidden_out!, act!, q_taken!)                             Q_Net.sample_action
  minimarl::agent_q_max(packed, dims, obs, hidden, hidden_out!, max_q!)          target max_a Q
  minimarl::td_error(rew, done, q_taken, max_q_next, gamma, td!)                 cal_td_error
  minimarl::gae_scan(rewards, value_preds, masks, value_norm, gamma, lambda, returns!)
  torch.classes.minimarl.Env(n_envs, n_agents, max_steps, step_cost, full_obs, device)
      .reset(obs!) / .step(act, next_obs!, obs_cur!?, rew!, done!)
  torch.classes.minimarl.PER(capacity, flavor, alpha, beta, eps, step_weight, use_step_weight,
                             alpha_inc, beta_inc, device)
      .insert(td, slots!) / .sample(fracs?, seed, counter, nodes!, slots!, is_weight!) / .update(nodes, td)

No fallback: importing this module without the built library raises.
"""
import os

import torch

from ._lib import LIB_PATH

TORCH_LIB_PATH = os.path.join(os.path.dirname(LIB_PATH), "libminimarl_torch.so")
_loaded = False


def load():
    """Register the ops (once) and return ``torch.ops.minimarl``."""
    global _loaded
    if not _loaded:
        if not os.path.exists(TORCH_LIB_PATH):
            raise ImportError(f"minimarl: torch op library not built ({TORCH_LIB_PATH}); run `make -C mini-marl_amd`")
        torch.ops.load_library(TORCH_LIB_PATH)
        _loaded = True
    return torch.ops.minimarl


def dims(net):
    """[n_agents, obs_dim, f1, g, h, n_actions] of an AgentQNet."""
    return [net.N, net.D, net.F1, net.G, net.H, net.A]


def Env(n_envs, n_agents, max_steps=100, step_cost=-0.01, full_observable=False, device=0):
    load()
    return torch.classes.minimarl.Env(int(n_envs), int(n_agents), int(max_steps), float(step_cost),
                                      bool(full_observable), int(torch.device(device).index or 0))


def PER(capacity, flavor="vdn", alpha=0.4, beta=0.4, eps=1e-6, step_weight=0.99, use_step_weight=True,
        alpha_inc=0.0, beta_inc=0.0, device=0):
    load()
    return torch.classes.minimarl.PER(int(capacity), str(flavor), float(alpha), float(beta), float(eps),
                                      float(step_weight), bool(use_step_weight), float(alpha_inc), float(beta_inc),
                                      int(torch.device(device).index or 0))
