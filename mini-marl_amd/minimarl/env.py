"""ma_gym Checkers-v0 stepped on the GPU (csrc/env.hip), E envs in lockstep.

Stands in for ``gym.make("ma_gym:Checkers-v0", full_observable, max_steps,
step_cost)`` (vdn/main.py:61-64, qmix/main.py:66-71): E independent envs x N
agents, obs laid out [env, agent, feat] in HBM. Dynamics: the rule-by-rule restatement of
ma_gym's published checkers.py in oracle/env.py (ma-gym 0.0.14 itself is absent: parity with it
is unpinned; N > 2 is the documented band extension).
"""
import ctypes

import numpy as np
import torch

from ._lib import release, EnvCfg, c_i32, c_vp, check, lib
from .qnet import ptr, stream_handle


class VecEnv:
    def __init__(self, n_envs, n_agents=2, max_steps=100, step_cost=-0.01, full_observable=False, cols=8,
                 device="cuda"):
        self.E, self.N = int(n_envs), int(n_agents)
        self.device = torch.device(device)
        self.cfg = EnvCfg(self.N, int(max_steps), int(bool(full_observable)), int(cols), float(step_cost))
        h = c_vp()
        check(lib().mm_env_create(ctypes.byref(self.cfg), self.E, 0, ctypes.byref(h)), "env_create")
        self._h = h
        self.obs_dim = lib().mm_env_obs_dim(h)
        self.n_actions = 5
        r, c = c_i32(), c_i32()
        lib().mm_env_grid_shape(h, ctypes.byref(r), ctypes.byref(c))
        self.rows, self.cols = r.value, c.value
        # which of the two state buffers holds the live state (the fused rollout step alternates them;
        # RolloutEngine installs its step parity here)
        self.state_buffer = lambda: 0

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._h = None
            try:
                release("mm_env_destroy", h)   # deferred while a graph capture is running
            except Exception:   # interpreter shutdown: module globals already gone
                pass

    def handle(self):
        return self._h

    def reset_obs_ptr(self):
        return lib().mm_env_reset_obs(self._h)

    # the rollout engine's chunk-store row steps (mm_env_step_rows / _td, include/minimarl.h)
    def step_rows(self, *args):
        return lib().mm_env_step_rows(self._h, *args)

    def step_rows_td(self, *args):
        return lib().mm_env_step_rows_td(self._h, *args)

    def step_rows_begin(self, *args):
        return lib().mm_env_step_rows_begin(self._h, *args)

    def reset(self, out=None):
        out = out if out is not None else torch.empty(self.E, self.N, self.obs_dim, device=self.device)
        check(lib().mm_env_reset(self._h, ptr(out), stream_handle(self.device)), "env_reset")
        return out

    def step(self, actions, autoreset=False):
        """actions [E,N] (int) -> (next_obs [E,N,D] terminal, reward [E,N], done [E] uint8[, obs_cur])."""
        actions = torch.as_tensor(actions, device=self.device).to(torch.int32).contiguous()
        assert actions.shape == (self.E, self.N)
        nxt = torch.empty(self.E, self.N, self.obs_dim, device=self.device)
        rew = torch.empty(self.E, self.N, device=self.device)
        done = torch.empty(self.E, dtype=torch.uint8, device=self.device)
        cur = torch.empty_like(nxt) if autoreset else None
        check(lib().mm_env_step(self._h, ptr(actions), ptr(nxt), ptr(cur), ptr(rew), ptr(done),
                                stream_handle(self.device)), "env_step")
        if autoreset:
            return nxt, rew, done, cur
        return nxt, rew, done

    def get_state(self):
        """(pos, prev, grid, steps, apples): agent_pos / agent_prev_pos [E,N,2], _full_obs codes [E,R,C]
        (0 empty, 1 lemon, 2 apple, 3 + k agent k), _step_count [E], apples left [E]."""
        pos = np.empty((self.E, self.N, 2), np.int32)
        prev = np.empty((self.E, self.N, 2), np.int32)
        grid = np.empty((self.E, self.rows, self.cols), np.int8)
        steps = np.empty(self.E, np.int32)
        apples = np.empty(self.E, np.int32)
        check(lib().mm_env_get_state_buf(self._h, self.state_buffer(), pos.ctypes.data, prev.ctypes.data,
                                         grid.ctypes.data, steps.ctypes.data, apples.ctypes.data), "env_get_state")
        return pos, prev, grid, steps, apples

    def set_state(self, pos, prev, grid, steps, apples):
        """Restore the state returned by get_state (checkpoint resume)."""
        pos = np.ascontiguousarray(pos, np.int32)
        prev = np.ascontiguousarray(prev, np.int32)
        grid = np.ascontiguousarray(grid, np.int8)
        steps = np.ascontiguousarray(steps, np.int32)
        apples = np.ascontiguousarray(apples, np.int32)
        assert pos.shape == prev.shape == (self.E, self.N, 2) and grid.shape == (self.E, self.rows, self.cols)
        check(lib().mm_env_set_state_buf(self._h, self.state_buffer(), pos.ctypes.data, prev.ctypes.data,
                                         grid.ctypes.data, steps.ctypes.data, apples.ctypes.data), "env_set_state")

    # ------------------------------------------------------------------ checkpoint (minimarl.checkpoint)
    def checkpoint_tensors(self):
        pos, prev, grid, steps, apples = self.get_state()
        return {"pos": torch.from_numpy(pos), "prev": torch.from_numpy(prev), "grid": torch.from_numpy(grid),
                "steps": torch.from_numpy(steps), "apples": torch.from_numpy(apples)}, {}

    def restore_tensors(self, ts, scalars=None):
        self.set_state(ts["pos"].numpy(), ts["prev"].numpy(), ts["grid"].numpy(), ts["steps"].numpy(),
                       ts["apples"].numpy())


class SwitchVecEnv:
    """``gym.make("ma_gym:Switch2-v0", max_steps, step_cost)`` (qmix/_config.py:14-19, qmix/main.py:66-71)
    for E envs in lockstep on the GPU (csrc/switch.hip; dynamics spec oracle/switch.py, parity with the
    absent ma-gym unpinned). ``step`` returns the env's per-agent done list as ``agent_done`` [E, N]
    and ``all(done)`` (what the reference's loops test) as ``done`` [E]."""

    def __init__(self, n_envs, n_agents=2, max_steps=100, step_cost=-0.01, full_observable=False, clock=True,
                 device="cuda"):
        from ._lib import SwitchCfg
        self.E, self.N = int(n_envs), int(n_agents)
        self.device = torch.device(device)
        self.cfg = SwitchCfg(self.N, int(max_steps), int(bool(full_observable)), int(bool(clock)), float(step_cost))
        h = c_vp()
        with torch.cuda.device(self.device):
            check(lib().mm_switch_create(ctypes.byref(self.cfg), self.E, ctypes.byref(h)), "switch_create")
        self._h = h
        self.obs_dim = lib().mm_switch_obs_dim(h)
        self.n_actions = 5

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._h = None
            try:
                release("mm_switch_destroy", h)
            except Exception:
                pass

    def handle(self):
        return self._h

    def reset_obs_ptr(self):
        return lib().mm_switch_reset_obs(self._h)

    def step_rows(self, *args):
        return lib().mm_switch_step_rows(self._h, *args)

    def step_rows_td(self, *args):
        return lib().mm_switch_step_rows_td(self._h, *args)

    def step_rows_begin(self, *args):
        return lib().mm_switch_step_rows_begin(self._h, *args)

    def reset(self, out=None):
        out = out if out is not None else torch.empty(self.E, self.N, self.obs_dim, device=self.device)
        check(lib().mm_switch_reset(self._h, ptr(out), stream_handle(self.device)), "switch_reset")
        return out

    def step(self, actions, autoreset=False):
        """actions [E, N] -> (next_obs [E, N, D], reward [E, N], agent_done [E, N] u8, done [E] u8[, obs_cur])."""
        actions = torch.as_tensor(actions, device=self.device).to(torch.int32).contiguous()
        assert actions.shape == (self.E, self.N)
        nxt = torch.empty(self.E, self.N, self.obs_dim, device=self.device)
        rew = torch.empty(self.E, self.N, device=self.device)
        adone = torch.empty(self.E, self.N, dtype=torch.uint8, device=self.device)
        done = torch.empty(self.E, dtype=torch.uint8, device=self.device)
        cur = torch.empty_like(nxt) if autoreset else None
        check(lib().mm_switch_step(self._h, ptr(actions), ptr(nxt), ptr(cur), ptr(rew), ptr(adone), ptr(done),
                                   stream_handle(self.device)), "switch_step")
        self._keep = actions
        if autoreset:
            return nxt, rew, adone, done, cur
        return nxt, rew, adone, done

    def get_state(self):
        pos = np.empty((self.E, self.N, 2), np.int32)
        adone = np.empty((self.E, self.N), np.uint8)
        steps = np.empty(self.E, np.int32)
        check(lib().mm_switch_get_state(self._h, pos.ctypes.data, adone.ctypes.data, steps.ctypes.data),
              "switch_get_state")
        return pos, adone, steps

    def set_state(self, pos, adone, steps):
        pos = np.ascontiguousarray(pos, np.int32)
        adone = np.ascontiguousarray(adone, np.uint8)
        steps = np.ascontiguousarray(steps, np.int32)
        assert pos.shape == (self.E, self.N, 2) and adone.shape == (self.E, self.N) and steps.shape == (self.E,)
        check(lib().mm_switch_set_state(self._h, pos.ctypes.data, adone.ctypes.data, steps.ctypes.data),
              "switch_set_state")

    def checkpoint_tensors(self):
        pos, adone, steps = self.get_state()
        return {"pos": torch.from_numpy(pos), "adone": torch.from_numpy(adone), "steps": torch.from_numpy(steps)}, {}

    def restore_tensors(self, ts, scalars=None):
        self.set_state(ts["pos"].numpy(), ts["adone"].numpy(), ts["steps"].numpy())


def make_env(kind, n_envs, n_agents, max_steps=100, step_cost=-0.01, full_observable=False, device="cuda"):
    """The lockstep env behind ``gym.make(args.env_name, ...)``: "checkers" (ma_gym:Checkers-v0, the
    VDN default, vdn/_config.py:19-24) or "switch" (ma_gym:Switch2-v0, the QMIX default,
    qmix/_config.py:14-19)."""
    if kind == "checkers":
        return VecEnv(n_envs, n_agents, max_steps, step_cost, full_observable, device=device)
    if kind == "switch":
        return SwitchVecEnv(n_envs, n_agents, max_steps, step_cost, full_observable, device=device)
    raise ValueError(f"unknown env {kind!r} (checkers | switch)")
