"""Oracle (test infrastructure only): the lockstep "checkers" gridworld, vectorised over envs.

The reference steps ``gym.make("ma_gym:Checkers-v0", full_observable, max_steps,
step_cost)`` (vdn/main.py:61-64, qmix/main.py:66-71); ma_gym 0.0.14 is not in
this image, so its dynamics are PARITY UNPINNED. This module *defines* the
build's environment (described after the reference notes vdn/explain.txt:3-6):

* grid R x Cc with R = 3*ceil(N/2), Cc = 8 (N = 2 gives Checkers' 3 x 8); agents
  pair up in 3-row bands: agent k starts at row 3*(k//2) + 2*(k%2), col Cc-2.
* fruit on every cell of columns 0..Cc-3: apple where (r + c) is even, lemon
  where odd; the last two columns are empty.
* actions 0 down, 1 left, 2 up, 3 right, 4 noop. Agents move in id order; a move
  is blocked by the border or by a cell held by another agent (positions as
  updated so far this step).
* reward per agent = step_cost, plus fruit at the agent's cell after its move
  (the fruit is consumed): even agents apple +10 / lemon -10, odd agents +1 / -1.
* done (env level, all agents) when step_count >= max_steps or no apple is left.
* obs per agent (D = 47): [row/(R-1), col/(Cc-1)] then the 3x3 neighbourhood
  (row-major, centre = own cell) x 5 channels {lemon, apple, even agent,
  odd agent, wall}; off-grid cells are wall [0,0,0,0,1]. full_observable:
  every agent sees the concatenation of all N agents' obs (D = 47*N).

Integer state, so GPU parity is bit-exact (coords use f32(r) * f32(1/(R-1))).
"""
import numpy as np

OBS_LOCAL = 47
DR = np.array([1, 0, -1, 0, 0], np.int32)
DC = np.array([0, -1, 0, 1, 0], np.int32)


class EnvSpec:
    def __init__(self, n_agents=2, max_steps=100, step_cost=-0.01, full_observable=False, cols=8):
        self.n_agents = int(n_agents)
        self.rows = 3 * ((self.n_agents + 1) // 2)
        self.cols = int(cols)
        self.max_steps = int(max_steps)
        self.step_cost = np.float32(step_cost)
        self.full_observable = bool(full_observable)
        self.obs_dim = OBS_LOCAL * (self.n_agents if full_observable else 1)
        self.n_actions = 5
        self.inv_r = np.float32(1.0 / max(self.rows - 1, 1))
        self.inv_c = np.float32(1.0 / max(self.cols - 1, 1))
        self.init_pos = np.array([[3 * (k // 2) + 2 * (k % 2), self.cols - 2] for k in range(self.n_agents)],
                                 np.int32)
        grid = np.zeros((self.rows, self.cols), np.int8)        # 0 empty, 1 lemon, 2 apple
        for r in range(self.rows):
            for c in range(self.cols - 2):
                grid[r, c] = 2 if (r + c) % 2 == 0 else 1
        self.init_grid = grid
        self.init_apples = int((grid == 2).sum())


class VecEnvOracle:
    def __init__(self, spec, n_envs):
        self.spec = spec
        self.E = int(n_envs)
        self.reset_all()

    def reset_all(self):
        s = self.spec
        self.pos = np.tile(s.init_pos[None], (self.E, 1, 1)).copy()          # [E,N,2]
        self.grid = np.tile(s.init_grid[None], (self.E, 1, 1)).copy()        # [E,R,C]
        self.steps = np.zeros(self.E, np.int32)
        self.apples = np.full(self.E, s.init_apples, np.int32)

    def reset_envs(self, mask):
        s = self.spec
        self.pos[mask] = s.init_pos
        self.grid[mask] = s.init_grid
        self.steps[mask] = 0
        self.apples[mask] = s.init_apples

    def observe(self):
        """obs [E,N,D] float32 for the current state."""
        s = self.spec
        E, N = self.E, s.n_agents
        local = np.zeros((E, N, OBS_LOCAL), np.float32)
        occ = np.full((E, s.rows, s.cols), -1, np.int32)
        ar = np.arange(E)
        for k in range(N):
            occ[ar, self.pos[:, k, 0], self.pos[:, k, 1]] = k
        for k in range(N):
            r = self.pos[:, k, 0]
            c = self.pos[:, k, 1]
            local[:, k, 0] = r.astype(np.float32) * s.inv_r
            local[:, k, 1] = c.astype(np.float32) * s.inv_c
            for dr in (-1, 0, 1):
                for dc in (-1, 0, 1):
                    cell = (dr + 1) * 3 + (dc + 1)
                    base = 2 + cell * 5
                    rr = r + dr
                    cc = c + dc
                    inside = (rr >= 0) & (rr < s.rows) & (cc >= 0) & (cc < s.cols)
                    rr_c = np.clip(rr, 0, s.rows - 1)
                    cc_c = np.clip(cc, 0, s.cols - 1)
                    item = self.grid[ar, rr_c, cc_c]
                    who = occ[ar, rr_c, cc_c]
                    lemon = inside & (item == 1)
                    apple = inside & (item == 2)
                    ag = inside & (item == 0) & (who >= 0)
                    local[:, k, base + 0] = lemon
                    local[:, k, base + 1] = apple
                    local[:, k, base + 2] = ag & (who % 2 == 0)
                    local[:, k, base + 3] = ag & (who % 2 == 1)
                    local[:, k, base + 4] = ~inside
        if s.full_observable:
            full = local.reshape(E, N * OBS_LOCAL)
            return np.repeat(full[:, None, :], N, axis=1).copy()
        return local

    def step(self, actions):
        """actions [E,N] int -> (next_obs [E,N,D] terminal obs, reward [E,N] f32, done [E] bool).
        Done envs are NOT reset here (use reset_envs)."""
        s = self.spec
        E, N = self.E, s.n_agents
        ar = np.arange(E)
        actions = np.asarray(actions, np.int32)
        self.steps += 1
        rew = np.full((E, N), s.step_cost, np.float32)
        for k in range(N):
            a = actions[:, k]
            nr = self.pos[:, k, 0] + DR[a]
            nc = self.pos[:, k, 1] + DC[a]
            ok = (nr >= 0) & (nr < s.rows) & (nc >= 0) & (nc < s.cols)
            for j in range(N):
                if j == k:
                    continue
                ok &= ~((self.pos[:, j, 0] == nr) & (self.pos[:, j, 1] == nc))
            self.pos[:, k, 0] = np.where(ok, nr, self.pos[:, k, 0])
            self.pos[:, k, 1] = np.where(ok, nc, self.pos[:, k, 1])
            item = self.grid[ar, self.pos[:, k, 0], self.pos[:, k, 1]]
            big = (k % 2 == 0)
            rew[:, k] += np.where(item == 2, np.float32(10 if big else 1),
                                  np.where(item == 1, np.float32(-10 if big else -1), np.float32(0)))
            self.apples -= (item == 2).astype(np.int32)
            self.grid[ar, self.pos[:, k, 0], self.pos[:, k, 1]] = 0
        done = (self.steps >= s.max_steps) | (self.apples == 0)
        return self.observe(), rew, done
