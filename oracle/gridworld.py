"""ORACLE / TEST INFRASTRUCTURE — numpy restatement of the discrete gridworld hot path:
Multistory FourRooms (`gym_po/envs/rooms/msrooms.py`) and ROOMS (`gym_po/envs/rooms/rooms.py`),
their observation builders (`rooms/observations.py`, `msrooms.py:131-254`) and action sampler
(`rooms/action_utils.py`). Pinned against golden fixtures from the reference (tests/golden).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this module.
"""
import json
import os

import numpy as np

from .draws import NumpyDraws

_MAPS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-po-taxi_amd",
                     "gym_po_amd", "data", "maps.json")


def load_maps():
    with open(_MAPS) as f:
        return json.load(f)


# action_utils.py:16-33 — N, NE, E, SE, S, SW, W, NW ; cardinal = every other
ACTIONS_ORDINAL = np.array([[-1, 0], [-1, 1], [0, 1], [1, 1], [1, 0], [1, -1], [0, -1], [-1, -1]])
ACTIONS_CARDINAL = ACTIONS_ORDINAL[::2]
ACTIONS_ORDINAL_Z = np.concatenate((np.zeros((8, 1), dtype=int), ACTIONS_ORDINAL), -1)
ACTIONS_CARDINAL_Z = ACTIONS_ORDINAL_Z[::2]


def action_probability_matrix(n, p):
    """action_utils.py:38-48: diagonal 1-p, off-diagonal p/(n-1), float64."""
    m = np.full((n, n), p / (n - 1), dtype=np.float64)
    np.fill_diagonal(m, 1 - p)
    return m


def sample_effective_action(prob_rows, u):
    """action_utils.py:84-90: a = #{j : cumsum(row)_j < u}."""
    s = prob_rows.cumsum(axis=1)
    return (s < u[:, None]).sum(axis=1)


# ------------------------------------------------------------------ observation builders ----
def hansen_obs_rooms(ayx, grid, gyx, n):
    """observations.py:44-71 — binary adjacency digits x goal multiplier (float64)."""
    a = (ACTIONS_CARDINAL if n == 4 else ACTIONS_ORDINAL)[None]
    coords = ayx[:, None] + a
    where = np.nonzero((gyx[:, None] == coords).all(-1))
    mult = np.ones(gyx.shape[0])
    mult[where[0]] = where[1] + 1
    sq = grid[tuple(coords.transpose(2, 0, 1))] + 1
    sq[sq > 0] = 1
    return sq.dot(np.array([2 ** i for i in range(a.shape[1])])) * mult


def hansen_vector_obs_rooms(ayx, grid, gyx, n):
    """observations.py:106-131 — 0 wall / 1 empty / 2 goal (goal only if gyx given)."""
    a = (ACTIONS_CARDINAL if n == 4 else ACTIONS_ORDINAL)[None]
    coords = ayx[:, None] + a
    sq = grid[tuple(coords.transpose(2, 0, 1))] + 1
    sq[sq > 0] = 1
    if gyx is not None:
        sq[(gyx[:, None] == coords).all(-1)] = 2
    return sq


def grid_obs_rooms(ayx, grid, gyx, n):
    """observations.py:74-103 — n x n window; out-of-range coordinates map to (0, 0)."""
    off = n // 2
    mg = np.mgrid[:n, :n] - off
    coords = (ayx[..., None, None] + mg[None]).swapaxes(0, 1)
    bad = (coords[0] < 0) | (coords[1] < 0) | (coords[0] >= grid.shape[0]) | (coords[1] >= grid.shape[1])
    coords[:, bad] = 0
    is_goal = (gyx.swapaxes(0, 1)[..., None, None] == coords).all(0)
    sq = grid[tuple(coords)] + 1
    sq[sq > 0] = 1
    sq[is_goal] = 2
    return sq


MAX_GR_CNST = 3  # msrooms.py:27-34 (wall 0, goal 1, stair_down 2, stair_up 3)


def hansen_obs_ms(azyx, ms, gzyx, n):
    """msrooms.py:162-189 — ternary digits (0 wall, 2 floor/stair, 1 if value > 3) x goal mult."""
    a = (ACTIONS_CARDINAL_Z if n == 4 else ACTIONS_ORDINAL_Z)[None]
    coords = azyx[:, None] + a
    where = np.nonzero((gzyx[:, None] == coords).all(-1))
    mult = np.ones(gzyx.shape[0])
    mult[where[0]] = where[1] + 1
    sq = ms[tuple(coords.transpose(2, 0, 1))]
    sq[(sq > 0) & (sq <= MAX_GR_CNST)] = 2
    sq[sq > MAX_GR_CNST] = 1
    return sq.dot(np.array([3 ** i for i in range(a.shape[1])])) * mult


def hansen_vector_obs_ms(azyx, ms, gzyx, n):
    """msrooms.py:131-159 — 0 wall / 2 floor-or-stair / 1 (>3) / 3 goal."""
    a = (ACTIONS_CARDINAL_Z if n == 4 else ACTIONS_ORDINAL_Z)[None]
    coords = azyx[:, None] + a
    sq = ms[tuple(coords.transpose(2, 0, 1))]
    sq[(sq > 0) & (sq <= MAX_GR_CNST)] = 2
    sq[sq > MAX_GR_CNST] = 1
    if gzyx is not None:
        sq[(gzyx[:, None] == coords).all(-1)] = 3
    return sq


def discrete_states(grid):
    """observations.py:16-29."""
    n = int((grid >= 0).sum())
    return n, ((grid >= 0).cumsum() - 1).reshape(grid.shape)


def rooms_obs_fn(obs_type, grid, obs_n):
    """rooms.py:15-68 (substring dispatch order: room, mdp, hansen, grid)."""
    vec = "vector" in obs_type
    goal = "goal" in obs_type
    if "room" in obs_type:
        n = len(np.unique(grid)) - 1
        if goal:
            return lambda a, g: grid[tuple(a.T)] + n * grid[tuple(g.T)]
        return lambda a, g: grid[tuple(a.T)]
    if "mdp" in obs_type:
        if vec:
            if goal:
                return lambda a, g: np.concatenate((a, g), -1)
            return lambda a, g: a.copy()
        n, sg = discrete_states(grid)
        if goal:
            return lambda a, g: sg[tuple(a.T)] + n * sg[tuple(g.T)]
        return lambda a, g: sg[tuple(a.T)]
    if "hansen" in obs_type:
        base = 8 if "8" in obs_type else 4
        if vec:
            if goal:
                return lambda a, g: hansen_vector_obs_rooms(a, grid, g, base)
            return lambda a, g: hansen_vector_obs_rooms(a, grid, None, base)
        return lambda a, g: hansen_obs_rooms(a, grid, g, base)
    if "grid" in obs_type:
        return lambda a, g: grid_obs_rooms(a, grid, g, obs_n)
    raise NotImplementedError(obs_type)


def ms_obs_fn(obs_type, ms, obs_n):
    """msrooms.py:192-254 (room obs raises in gymnasium: Discrete(n<=0))."""
    vec = "vector" in obs_type
    goal = "goal" in obs_type
    if "room" in obs_type:
        raise ValueError("msrooms 'room' obs: reference builds Discrete(n<=0) (msrooms.py:206-216)")
    if "mdp" in obs_type:
        if vec:
            if goal:
                return lambda a, g: np.concatenate((a, g), -1)
            return lambda a, g: a.copy()
        n, sg = discrete_states(ms - 1)
        if goal:
            return lambda a, g: sg[tuple(a.T)] + n * sg[tuple(g.T)]
        return lambda a, g: sg[tuple(a.T)]
    if "hansen" in obs_type:
        base = 8 if "8" in obs_type else 4
        if vec:
            if goal:
                return lambda a, g: hansen_vector_obs_ms(a, ms, g, base)
            return lambda a, g: hansen_vector_obs_ms(a, ms, None, base)
        return lambda a, g: hansen_obs_ms(a, ms, g, base)
    raise NotImplementedError(obs_type)


# ------------------------------------------------------------------------- environments ----
class _GridOracle:
    """Shared batched step (msrooms.py:390-413 / rooms.py:198-222), pure given the draws."""
    STATE_ALIASES = dict(agent="agent", goal="goal", elapsed="elapsed")

    def _finish_init(self, num_envs, time_limit, p_fail, step_reward, wall_reward, goal_reward):
        self.num_envs = num_envs
        self.time_limit = time_limit
        self.step_reward, self.wall_reward, self.goal_reward = step_reward, wall_reward, goal_reward
        self.action_matrix = action_probability_matrix(self.actions.shape[0], p_fail)

    def _sample(self, fixed, valid, b, draws, site):
        if fixed is not None:
            return np.full((b, self.grid.ndim), fixed, dtype=int)
        mask = self._pending_mask
        idx = draws.choice(valid, mask, site)
        return np.array(np.unravel_index(idx, self.grid.shape)).swapaxes(0, 1)

    def reset(self, draws):
        B = self.num_envs
        self.elapsed = np.zeros(B, int)
        self._pending_mask = np.ones(B, bool)
        self.goal = self._sample(self.fixed_goal, self.valid_goal, B, draws, "goal")
        self.agent = self._sample(self.fixed_agent, self.valid_agent, B, draws, "agent")
        return self.obs_fn(self.agent, self.goal)

    def reset_seed(self, seed):
        self.gen = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        return self.reset(NumpyDraws(self.gen))

    def _transit(self, moved):
        pass

    def step(self, action, draws):
        self.elapsed += 1
        u = draws.uniform(self.num_envs)
        a = sample_effective_action(self.action_matrix[action], u)
        prop = self.agent + self.actions[a]
        oob = self.grid[tuple(prop.T)] == self.wall_value
        self.agent[~oob] = prop[~oob]
        self._transit(~oob)
        r = np.zeros(self.num_envs, dtype=np.float32)
        d = (self.agent == self.goal).all(-1)
        r += self.step_reward
        r[oob] = self.wall_reward
        r[d] = self.goal_reward
        trunc = self.elapsed > self.time_limit
        mask = d | trunc
        if b := int(mask.sum()):
            self._pending_mask = mask
            self.elapsed[mask] = 0
            self.goal[mask] = self._sample(self.fixed_goal, self.valid_goal, b, draws, "goal")
            self.agent[mask] = self._sample(self.fixed_agent, self.valid_agent, b, draws, "agent")
        return self.obs_fn(self.agent, self.goal), r, d, trunc

    def step_seeded(self, action):
        return self.step(action, NumpyDraws(self.gen))


class FourRoomsOracle(_GridOracle):
    """MultistoryFourRoomsEnv restated (msrooms.py:257-428)."""
    END_XYZ = (9, 7, -1)
    START_XYZ = (1, 1, 0)
    UP_YX = np.array([1, 11])    # msrooms.py:23
    DOWN_YX = np.array([11, 1])  # msrooms.py:24

    def __init__(self, num_envs, grid_z=1, floor_map=None, time_limit=500, obs_type="mdp", obs_n=3,
                 action_failure_probability=1.0 / 3, action_type="cardinal", agent_xyz=None,
                 goal_xyz=END_XYZ, step_reward=0.0, wall_reward=0.0, goal_reward=1.0):
        fm = np.array(load_maps()["fourrooms_floor_map"] if floor_map is None else floor_map)
        walk = fm.copy()
        walk[fm > 0] = 1
        ms = np.stack([walk for _ in range(grid_z)], 0)
        if grid_z > 1:
            ms[1:, self.DOWN_YX[0], self.DOWN_YX[1]] = 2
            ms[:-1, self.UP_YX[0], self.UP_YX[1]] = 3
        self.grid = ms
        self.wall_value = 0
        self.obs_fn = ms_obs_fn(obs_type, ms, obs_n)
        sv = np.array(np.nonzero(ms > 0))
        self.valid_agent = np.ravel_multi_index(sv[:, sv[0] == 0], ms.shape)
        self.valid_goal = np.ravel_multi_index(sv[:, sv[0] == ms.shape[0] - 1], ms.shape)
        self.actions = ACTIONS_CARDINAL_Z if action_type == "cardinal" else ACTIONS_ORDINAL_Z
        if goal_xyz is not None:
            g = tuple(reversed(goal_xyz))
            if ms[g] <= MAX_GR_CNST:
                g = tuple(reversed(self.END_XYZ))
            g = np.array(g)
            if g[0] == -1:
                g[0] = ms.shape[0] - 1
            self.fixed_goal = g
        else:
            self.fixed_goal = None
        if agent_xyz is not None:
            # NOTE: reference indexes grid with an ndarray here (msrooms.py:356) and raises;
            # restated with the evident intent (wall -> START_XYZ). Parity unpinned.
            a = tuple(reversed(agent_xyz))
            if ms[a] == 0:
                a = tuple(reversed(self.START_XYZ))
            self.fixed_agent = np.array(a)
        else:
            self.fixed_agent = None
        self._finish_init(num_envs, time_limit, action_failure_probability, step_reward, wall_reward,
                          goal_reward)

    def _transit(self, moved):
        """msrooms.py:419-428."""
        v = self.grid[tuple(self.agent.T)]
        up = (v == 3) & moved
        down = (v == 2) & moved
        if up.any():
            self.agent[up, 0] += 1
            self.agent[up, 1:] = self.DOWN_YX
        if down.any():
            self.agent[down, 0] -= 1
            self.agent[down, 1:] = self.UP_YX


class RoomsOracle(_GridOracle):
    """RoomsEnv restated (rooms.py:71-226)."""

    def __init__(self, num_envs, layout="4", time_limit=500, obs_type="mdp", obs_n=3,
                 action_failure_probability=0.2, action_type="ordinal", agent_xy=None, goal_xy=(0, 0),
                 step_reward=0.0, wall_reward=0.0, goal_reward=1.0):
        maps = load_maps()
        grid = np.array(maps["rooms_layouts"][layout])
        key = layout[:-1] if "b" in layout else layout
        self.grid = grid
        self.wall_value = -1
        self.obs_fn = rooms_obs_fn(obs_type, grid, obs_n)
        self.valid_goal = self.valid_agent = np.flatnonzero(grid >= 0)
        self.actions = ACTIONS_CARDINAL if action_type == "cardinal" else ACTIONS_ORDINAL
        if goal_xy is not None:
            g = tuple(reversed(goal_xy))
            if grid[g] < 0:
                g = tuple(reversed(maps["rooms_ends_xy"][key]))
            self.fixed_goal = np.array(g)
        else:
            self.fixed_goal = None
        if agent_xy is not None:
            # reference raises here (ndarray index, rooms.py:166); evident intent restated
            a = tuple(reversed(agent_xy))
            if grid[a] < 0:
                a = tuple(reversed(maps["rooms_starts_xy"][key]))
            self.fixed_agent = np.array(a)
        else:
            self.fixed_agent = None
        self._finish_init(num_envs, time_limit, action_failure_probability, step_reward, wall_reward,
                          goal_reward)
