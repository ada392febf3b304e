"""Oracle (test infrastructure only): the ``ma_gym:Switch2-v0`` corridor env, vectorised over envs.

QMIX's default env is ``gym.make("ma_gym:Switch2-v0", max_steps=args.max_step,
step_cost=args.step_cost)`` (qmix/_config.py:14-19, qmix/main.py:66-71: max_step 100, step_cost
-0.01). ma-gym 0.0.14 is not in this image and no reference file holds its outputs, so this is a
restatement of the published ma_gym ``Switch`` env (envs/switch/switch_one_corridor.py) and its
dynamics are PARITY UNPINNED. The restated algorithm:

* grid 3 x 7, every cell wall except the middle row and columns 0, 1, 5, 6 (two 3-cell rooms
  joined by a one-cell-wide corridor);
* n_agents 2..4 (Switch2: 2). Agent k starts at {0: (0,1), 1: (0,5), 2: (2,1), 3: (2,5)}[k] and must
  reach {0: (0,6), 1: (0,0), 2: (2,6), 3: (2,0)}[k] (the opposite room);
* actions 0 down, 1 left, 2 up, 3 right, 4 noop; agents move in id order; a move succeeds if the
  target cell is on the grid, not a wall and not held by another agent (positions as updated so
  far this step; finished agents keep their cell);
* reward per agent: step_cost, or +5 on the step the agent reaches its target (it is then done
  and no longer moves, but keeps receiving step_cost); at step_count >= max_steps every agent is
  done;
* obs per agent: [round(row / 2, 2), round(col / 6, 2)] (+ [step_count / max_steps] with the
  clock, ma_gym's default), as float32; full_observable: the concatenation of all agents' obs.

Integer state and a 7-entry column table make GPU parity bit-exact.
"""
import numpy as np

ROWS, COLS = 3, 7
DR = np.array([1, 0, -1, 0, 0], np.int32)
DC = np.array([0, -1, 0, 1, 0], np.int32)
INIT = np.array([[0, 1], [0, COLS - 2], [2, 1], [2, COLS - 2]], np.int32)
FINAL = np.array([[0, COLS - 1], [0, 0], [2, COLS - 1], [2, 0]], np.int32)


def open_cells():
    g = np.zeros((ROWS, COLS), bool)
    g[ROWS // 2, :] = True
    g[:, [0, 1, COLS - 2, COLS - 1]] = True
    return g


class SwitchSpec:
    def __init__(self, n_agents=2, max_steps=100, step_cost=-0.01, full_observable=False, clock=True):
        assert 2 <= n_agents <= 4
        self.n_agents, self.max_steps = int(n_agents), int(max_steps)
        self.step_cost = np.float32(step_cost)
        self.full_observable, self.clock = bool(full_observable), bool(clock)
        self.local_dim = 2 + int(self.clock)
        self.obs_dim = self.local_dim * (self.n_agents if self.full_observable else 1)
        self.n_actions = 5
        self.row_feat = np.array([round(r / (ROWS - 1), 2) for r in range(ROWS)], np.float32)
        self.col_feat = np.array([round(c / (COLS - 1), 2) for c in range(COLS)], np.float32)


class SwitchOracle:
    def __init__(self, spec, n_envs):
        self.spec, self.E = spec, int(n_envs)
        self.open = open_cells()
        self.reset_all()

    def reset_all(self):
        N = self.spec.n_agents
        self.pos = np.broadcast_to(INIT[:N], (self.E, N, 2)).copy()
        self.adone = np.zeros((self.E, N), bool)
        self.steps = np.zeros(self.E, np.int64)
        return self.obs()

    def reset_envs(self, mask):
        N = self.spec.n_agents
        self.pos[mask] = INIT[:N]
        self.adone[mask] = False
        self.steps[mask] = 0

    def obs(self):
        s, N = self.spec, self.spec.n_agents
        parts = [s.row_feat[self.pos[:, :, 0]], s.col_feat[self.pos[:, :, 1]]]
        if s.clock:
            clk = np.array([np.float32(int(k) / s.max_steps) for k in self.steps], np.float32)
            parts.append(np.broadcast_to(clk[:, None], (self.E, N)))
        local = np.stack(parts, -1).astype(np.float32)                   # [E, N, local]
        if s.full_observable:
            flat = local.reshape(self.E, 1, N * s.local_dim)
            return np.broadcast_to(flat, (self.E, N, N * s.local_dim)).copy()
        return local

    def step(self, act):
        """act [E, N] -> (obs [E, N, D], reward [E, N] f32, agent_done [E, N] bool, done [E] bool)."""
        s, N = self.spec, self.spec.n_agents
        act = np.asarray(act, np.int64)
        self.steps += 1
        rew = np.full((self.E, N), s.step_cost, np.float32)
        for e in range(self.E):
            for k in range(N):
                if self.adone[e, k]:
                    continue
                a = act[e, k]
                if a != 4:
                    r, c = self.pos[e, k, 0] + DR[a], self.pos[e, k, 1] + DC[a]
                    ok = 0 <= r < ROWS and 0 <= c < COLS and self.open[r, c]
                    if ok:
                        for j in range(N):
                            if j != k and self.pos[e, j, 0] == r and self.pos[e, j, 1] == c:
                                ok = False
                    if ok:
                        self.pos[e, k] = (r, c)
                if self.pos[e, k, 0] == FINAL[k, 0] and self.pos[e, k, 1] == FINAL[k, 1]:
                    self.adone[e, k] = True
                    rew[e, k] = np.float32(5)
        self.adone[self.steps >= s.max_steps] = True
        return self.obs(), rew, self.adone.copy(), self.adone.all(1)
