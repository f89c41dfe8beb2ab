"""ORACLE / TEST INFRASTRUCTURE — numpy restatement of batched C-ROOMS (`gym_po/envs/rooms/crooms.py`).

`dtype=np.float64` is the reference arithmetic (seed-identical with `NumpyDraws`);
`dtype=np.float32` is the per-step fp32 twin the GPU kernel is checked against: same operation
order, float32 rounding after every operation, float32 noise (the float64 draw rounded once).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this module.
"""
import numpy as np

from .draws import NumpyDraws
from .gridworld import (ACTIONS_CARDINAL, ACTIONS_ORDINAL, action_probability_matrix, discrete_states,
                        grid_obs_rooms, hansen_obs_rooms, hansen_vector_obs_rooms, load_maps,
                        sample_effective_action)


def coord_to_grid(c, cell):
    """utils.py:15-20."""
    return np.floor(c / cell).astype(int)


def grid_to_coord(g, cell=1.0):
    """utils.py:7-12."""
    return g * cell + cell / 2


def crooms_obs_fn(obs_type, grid, obs_m, cell):
    """crooms.py:16-88."""
    vec = "vector" in obs_type
    goal = "goal" in obs_type
    cg = lambda x: coord_to_grid(x, cell)  # noqa: E731
    if "room" in obs_type:
        n = len(np.unique(grid)) - 1
        if goal:
            return lambda a, g: grid[tuple(cg(a).T)] + n * grid[tuple(cg(g).T)]
        return lambda a, g: grid[tuple(cg(a).T)]
    if "mdp" in obs_type:
        if vec:
            if goal:
                return lambda a, g: np.concatenate((a, g), -1)
            return lambda a, g: a.copy()
        n, sg = discrete_states(grid)
        if goal:
            return lambda a, g: sg[tuple(cg(a).T)] + n * sg[tuple(cg(g).T)]
        return lambda a, g: sg[tuple(cg(a).T)]
    if "hansen" in obs_type:
        base = 8 if "8" in obs_type else 4
        if vec:
            if goal:
                return lambda a, g: hansen_vector_obs_rooms(cg(a), grid, cg(g), base)
            return lambda a, g: hansen_vector_obs_rooms(cg(a), grid, None, base)
        return lambda a, g: hansen_obs_rooms(cg(a), grid, cg(g), base)
    if "grid" in obs_type:
        return lambda a, g: grid_obs_rooms(cg(a), grid, cg(g), obs_m)
    raise NotImplementedError(obs_type)


class CRoomsOracle:
    """CRoomsEnv restated (crooms.py:91-338)."""
    STATE_ALIASES = dict(agent="agent", goal="goal", elapsed="elapsed", velocity="velocity")

    def __init__(self, num_envs, layout="4", time_limit=500, use_velocity=False, cell_size=1.0,
                 obs_type="mdp", obs_m=3, action_failure_probability=0.2, action_type="yx", action_std=0.2,
                 action_power=1.0, agent_xy=None, goal_xy=(0, 0), step_reward=0.0, wall_reward=0.0,
                 goal_reward=1.0, goal_threshold=0.5, dtype=np.float64):
        maps = load_maps()
        grid = np.array(maps["rooms_layouts"][layout])
        key = layout[:-1] if "b" in layout else layout
        self.f = dtype
        self.grid = grid
        self.gridshape = np.array(grid.shape)
        self.obs_fn = crooms_obs_fn(obs_type, grid, obs_m, cell_size)
        self.valid = np.flatnonzero(grid >= 0)
        self.max_velocity = 5.0
        self.yx = action_type == "yx"
        self.action_std = action_std
        if not self.yx:
            self.actions = ACTIONS_CARDINAL if action_type == "cardinal" else ACTIONS_ORDINAL
            self.action_matrix = action_probability_matrix(self.actions.shape[0], action_failure_probability)
        self.use_velocity = use_velocity
        self.num_envs = num_envs
        self.time_limit = time_limit
        self.step_reward, self.goal_reward, self.wall_reward = step_reward, goal_reward, wall_reward
        self.goal_threshold = goal_threshold
        self.cell = cell_size
        self.action_power = action_power
        if goal_xy is not None:
            g = tuple(reversed(goal_xy))
            if grid[g] < 0:
                g = tuple(reversed(maps["rooms_ends_xy"][key]))
            self.fixed_goal = np.array(g)
        else:
            self.fixed_goal = None
        if agent_xy is not None:
            # reference raises here (ndarray index, crooms.py:234); evident intent restated
            a = tuple(reversed(agent_xy))
            if grid[a] < 0:
                a = tuple(reversed(maps["rooms_starts_xy"][key]))
            self.fixed_agent = np.array(a)
        else:
            self.fixed_agent = None

    # crooms.py:217-244 — NOTE goal (fixed or random) and random agent ignore cell_size
    def _sample_goal(self, mask, draws):
        b = int(mask.sum())
        if self.fixed_goal is not None:
            return grid_to_coord(np.full((b, 2), self.fixed_goal, dtype=int)).astype(self.f)
        idx = draws.choice(self.valid, mask, "goal")
        return grid_to_coord(np.array(np.unravel_index(idx, self.grid.shape)).swapaxes(0, 1)).astype(self.f)

    def _sample_agent(self, mask, draws):
        b = int(mask.sum())
        if self.fixed_agent is not None:
            return grid_to_coord(np.full((b, 2), self.fixed_agent, dtype=int), self.cell).astype(self.f)
        idx = draws.choice(self.valid, mask, "agent")
        return grid_to_coord(np.array(np.unravel_index(idx, self.grid.shape)).swapaxes(0, 1)).astype(self.f)

    def reset_seed(self, seed):
        self.gen = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        return self.reset(NumpyDraws(self.gen))

    def reset(self, draws):
        B = self.num_envs
        mask = np.ones(B, bool)
        self.elapsed = np.zeros(B, int)
        self.goal = self._sample_goal(mask, draws)
        self.agent = self._sample_agent(mask, draws)
        self.velocity = np.zeros((B, 2), dtype=self.f)
        return self.obs_fn(self.agent, self.goal)

    def step_seeded(self, action):
        return self.step(action, NumpyDraws(self.gen))

    def _normal(self, draws, scale, mask, site):
        if isinstance(draws, NumpyDraws):
            v = draws.normal(scale, int(mask.sum()), site)
            hook = getattr(draws, "record_normal", None)  # tests: capture the stream's values per env
            if hook is not None:
                hook(site, mask, v)
            return v.astype(self.f)
        return draws.normal_masked(mask, site).astype(self.f)

    def _sample_action(self, a, draws):
        """crooms.py:175-198."""
        B = self.num_envs
        allm = np.ones(B, bool)
        if self.yx:
            return a.astype(self.f) + self._normal(draws, self.action_std, allm, "noise")
        u = draws.uniform(B)
        eff = sample_effective_action(self.action_matrix[a], u)
        mv = self.actions[eff]
        if self.action_std:
            return mv + self._normal(draws, self.action_std, allm, "noise")
        return mv.astype(self.f)

    def step(self, action, draws):
        """crooms.py:276-298."""
        f = self.f
        self.elapsed += 1
        a = self._sample_action(action, draws) * f(self.action_power)
        oob = self._apply_action(a, draws)
        r = np.zeros(self.num_envs, dtype=np.float32)
        d = np.linalg.norm(self.agent - self.goal, 2, -1) <= f(self.goal_threshold)
        r += self.step_reward
        r[oob] = self.wall_reward
        r[d] = self.goal_reward
        trunc = self.elapsed > self.time_limit
        mask = d | trunc
        if mask.sum():
            self.elapsed[mask] = 0
            self.goal[mask] = self._sample_goal(mask, draws)
            self.agent[mask] = self._sample_agent(mask, draws)
            self.velocity[mask] = 0.0
        return self.obs_fn(self.agent, self.goal), r, d, trunc

    def _apply_action(self, a, draws):
        """crooms.py:300-331."""
        f = self.f
        if self.use_velocity:
            self.velocity += a
            self.velocity.clip(-self.max_velocity, self.max_velocity, self.velocity)
            prop = self.agent + self.velocity
        else:
            prop = self.agent + a
        hi = (self.gridshape - 1 - 1e-6).astype(f)
        prop = prop.clip(f(0), hi)
        oob = self.grid[tuple(coord_to_grid(prop, f(self.cell)).T)] == -1
        self.agent[~oob] = prop[~oob]
        if oob.any():
            c = grid_to_coord(coord_to_grid(self.agent[oob], f(self.cell)), f(self.cell)).astype(f)
            n = self._normal(draws, 0.5, oob, "wall_noise")
            self.agent[oob] = np.clip(c + n, c - f(self.cell / 2), (c + f(self.cell / 2)) - f(1e-8))
            self.velocity[oob] = 0.0
        return oob
