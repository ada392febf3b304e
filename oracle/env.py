"""Oracle (test infrastructure only): ma_gym's ``Checkers-v0`` restated, vectorised over envs.

The reference steps ``gym.make("ma_gym:Checkers-v0", full_observable=True, max_steps=args.max_step,
step_cost=args.step_cost)`` (vdn/main.py:61-64; max_step 100, step_cost -0.01, vdn/_config.py:19-24).
ma-gym 0.0.14 (pinned in vdn/wandb/run-20240318_214947-tw6w4mqv/files/requirements.txt:19, with gym 0.20.0)
is not in this image and no reference file holds its outputs, so this module RESTATES the published env
``ma_gym/envs/checkers/checkers.py`` (class ``Checkers``) rule by rule; its dynamics are PARITY UNPINNED
against ma_gym itself. Anchors the reference does hold: an episode without fruit scores
2 x 100 x -0.01 = -2.00 (vdn/logs/vdn-1710766189.log:42-43), and the logged scores of the first,
near-random episodes (eps 0.8) end early about 2 times in 3 — the statistics only "fruit is eaten once and
the env ends when no apple is left" reproduce (tests/test_env_checkers.py). The restated algorithm:

* ``_grid_shape = (3, 8)``, ``n_agents = 2``; ``init_agent_pos = {0: [0, 6], 1: [2, 6]}`` (column
  ``grid_shape[1] - 2``); ``agent_reward = {0: {lemon: -10, apple: 10}, 1: {lemon: -1, apple: 1}}``.
* ``__init_full_obs``: ``_full_obs`` (one entry per cell: empty / lemon / apple / agent marker) starts empty,
  every agent marker is written at its position (``__update_agent_view``), then the fruit: a flag starting at
  lemon walks the cells column by column (``for col in range(8 - 2): for row in range(3)``) and flips after
  every cell, so cell (r, c) of columns 0..5 holds a lemon where 3c + r (equivalently r + c) is even and an
  apple where it is odd: 9 lemons, 9 apples; ``_food_count`` counts them.
* ``step(actions)``: ``_step_count += 1``; every reward starts at ``step_cost``; agents act in id order:
  ``__update_agent_pos``: action 0 down (row + 1), 1 left (col - 1), 2 up (row - 1), 3 right (col + 1),
  4 no-op; the move happens when the next cell is on the grid and vacant of agents (its ``_full_obs`` entry is
  not an agent marker), and then ``agent_prev_pos = old position``. ``agent_prev_pos`` is NOT touched
  otherwise. Then, if ``agent_pos != agent_prev_pos``: the fruit in ``_full_obs`` at the agent's cell (lemon
  checked first, then apple) adds that agent's reward for it and decrements ``_food_count`` (eaten once),
  and ``__update_agent_view`` writes empty at ``agent_prev_pos`` and the agent's marker at ``agent_pos``.
  ma_gym's quirk, restated as is: after a move, ``agent_prev_pos`` stays stale, so on later no-move steps the
  view update runs again every step; it re-writes empty at the stale cell, which ERASES another agent that
  moved in there (that agent drops out of every observation, its own included, until its own next view
  update re-marks it; an agent acting later in the same step would find its cell vacant).
* done for every agent when ``_step_count >= max_steps`` or ``_food_count['apple'] == 0``.
* ``get_agent_obs``: per agent ``[round(row / 2, 2), round(col / 7, 2)]`` then the 3 x 3 neighbourhood
  (row-major, centre = own cell) x 5 channels ``ITEM_ONE_HOT_INDEX = {lemon: 0, apple: 1, A1: 2, A2: 3,
  wall: 4}`` read from ``_full_obs``; cells off the grid stay all-zero (``_agent_i_neighbour`` starts as
  zeros and only valid cells are written; Checkers has no walls, so channel 4 is always 0). Python floats
  become float32 in the reference's ``torch.Tensor(state)``. full_observable: every agent gets the
  concatenation of all agents' obs (D = 94).

Extension beyond ma_gym (documented, not restated): N > 2 agents stack N / 2 copies of the 3 x 8 board as
3-row bands (R = 3 ceil(N / 2) rows); agents 2b and 2b + 1 start at (3b, cols - 2) and (3b + 2, cols - 2),
band b's fruit follows the board's parity with band-local rows ((r - 3b) + c even = lemon), even agents score
+-10 and show in channel 2, odd agents +-1 and channel 3; coordinates are round(row / (R - 1), 2) and
round(col / (cols - 1), 2). N = 2 with 8 columns is exactly the restatement above.

Integer state, so GPU parity is bit-exact (coordinates come from the same float32 tables).
"""
import numpy as np

OBS_LOCAL = 47
EMPTY, LEMON, APPLE, AGENT0 = 0, 1, 2, 3          # _full_obs entries; agent k's marker is AGENT0 + k
DR = np.array([1, 0, -1, 0, 0], np.int32)
DC = np.array([0, -1, 0, 1, 0], np.int32)


def coord_table(n):
    """[round(i / (n - 1), 2) for i < n] as float32 (Python's round of the double, then float32)."""
    return np.array([np.float32(round(i / (n - 1), 2)) if n > 1 else np.float32(0.0) for i in range(n)], np.float32)


class EnvSpec:
    def __init__(self, n_agents=2, max_steps=100, step_cost=-0.01, full_observable=False, cols=8):
        self.n_agents = int(n_agents)
        self.bands = (self.n_agents + 1) // 2
        self.rows = 3 * self.bands
        self.cols = int(cols)
        self.max_steps = int(max_steps)
        self.step_cost = np.float32(step_cost)
        self.full_observable = bool(full_observable)
        self.obs_dim = OBS_LOCAL * (self.n_agents if full_observable else 1)
        self.n_actions = 5
        self.rtab = coord_table(self.rows)
        self.ctab = coord_table(self.cols)
        self.init_pos = np.array([[3 * (k // 2) + 2 * (k % 2), self.cols - 2] for k in range(self.n_agents)],
                                 np.int32)
        grid = np.zeros((self.rows, self.cols), np.int8)
        for k in range(self.n_agents):                      # __update_agent_view of every agent first
            grid[self.init_pos[k, 0], self.init_pos[k, 1]] = AGENT0 + k
        for b in range(self.bands):                         # then the fruit, lemon flag first
            flag = True
            for c in range(self.cols - 2):
                for lr in range(3):
                    grid[3 * b + lr, c] = LEMON if flag else APPLE
                    flag = not flag
        self.init_grid = grid
        self.init_apples = int((grid == APPLE).sum())
        big = (np.arange(self.n_agents) % 2) == 0
        self.apple_reward = np.where(big, np.float32(10), np.float32(1)).astype(np.float32)
        self.lemon_reward = np.where(big, np.float32(-10), np.float32(-1)).astype(np.float32)


class VecEnvOracle:
    """State per env: ``grid`` = _full_obs codes [E, R, C] int8, ``pos`` / ``prev`` = agent_pos /
    agent_prev_pos [E, N, 2], ``steps`` = _step_count, ``apples`` = _food_count['apple']."""

    def __init__(self, spec, n_envs):
        self.spec = spec
        self.E = int(n_envs)
        self.reset_all()

    def reset_all(self):
        s = self.spec
        self.pos = np.tile(s.init_pos[None], (self.E, 1, 1)).copy()          # [E,N,2]
        self.prev = self.pos.copy()
        self.grid = np.tile(s.init_grid[None], (self.E, 1, 1)).copy()        # [E,R,C]
        self.steps = np.zeros(self.E, np.int32)
        self.apples = np.full(self.E, s.init_apples, np.int32)

    def reset_envs(self, mask):
        s = self.spec
        self.pos[mask] = s.init_pos
        self.prev[mask] = s.init_pos
        self.grid[mask] = s.init_grid
        self.steps[mask] = 0
        self.apples[mask] = s.init_apples

    def observe(self):
        """obs [E,N,D] float32 for the current state (get_agent_obs)."""
        s = self.spec
        E, N = self.E, s.n_agents
        local = np.zeros((E, N, OBS_LOCAL), np.float32)
        ar = np.arange(E)
        for k in range(N):
            r = self.pos[:, k, 0]
            c = self.pos[:, k, 1]
            local[:, k, 0] = s.rtab[r]
            local[:, k, 1] = s.ctab[c]
            for dr in (-1, 0, 1):
                for dc in (-1, 0, 1):
                    base = 2 + ((dr + 1) * 3 + (dc + 1)) * 5
                    rr, cc = r + dr, c + dc
                    inside = (rr >= 0) & (rr < s.rows) & (cc >= 0) & (cc < s.cols)
                    item = self.grid[ar, np.clip(rr, 0, s.rows - 1), np.clip(cc, 0, s.cols - 1)].astype(np.int32)
                    item = np.where(inside, item, EMPTY)
                    who = item - AGENT0
                    local[:, k, base + 0] = item == LEMON
                    local[:, k, base + 1] = item == APPLE
                    local[:, k, base + 2] = (item >= AGENT0) & (who % 2 == 0)
                    local[:, k, base + 3] = (item >= AGENT0) & (who % 2 == 1)
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
        actions = np.asarray(actions, np.int64)
        assert actions.shape == (E, N) and ((actions >= 0) & (actions < 5)).all(), "Action Not found!"
        self.steps += 1
        rew = np.full((E, N), s.step_cost, np.float32)
        for k in range(N):
            a = actions[:, k]
            r0, c0 = self.pos[:, k, 0].copy(), self.pos[:, k, 1].copy()
            nr, nc = r0 + DR[a], c0 + DC[a]
            inside = (a != 4) & (nr >= 0) & (nr < s.rows) & (nc >= 0) & (nc < s.cols)
            tgt = self.grid[ar, np.clip(nr, 0, s.rows - 1), np.clip(nc, 0, s.cols - 1)]
            move = inside & (tgt < AGENT0)                     # _is_cell_vacant: no agent marker there
            self.prev[move, k, 0], self.prev[move, k, 1] = r0[move], c0[move]
            self.pos[move, k, 0], self.pos[move, k, 1] = nr[move], nc[move]
            moved = (self.pos[:, k, 0] != self.prev[:, k, 0]) | (self.pos[:, k, 1] != self.prev[:, k, 1])
            pr, pc = self.pos[:, k, 0], self.pos[:, k, 1]
            item = self.grid[ar, pr, pc]
            lemon = moved & (item == LEMON)
            apple = moved & (item == APPLE)
            rew[:, k] += np.where(lemon, s.lemon_reward[k], np.where(apple, s.apple_reward[k], np.float32(0)))
            self.apples -= apple.astype(np.int32)
            ix = np.nonzero(moved)[0]
            self.grid[ix, self.prev[ix, k, 0], self.prev[ix, k, 1]] = EMPTY
            self.grid[ix, pr[ix], pc[ix]] = AGENT0 + k
        done = (self.steps >= s.max_steps) | (self.apples == 0)
        return self.observe(), rew, done
