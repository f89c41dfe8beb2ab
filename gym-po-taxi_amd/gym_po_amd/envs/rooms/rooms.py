"""ROOMS — drop-in for `gym_po.envs.rooms.rooms.RoomsEnv` (rooms.py:71-226)."""
import numpy as np

from ... import _lib
from ...maps import ENDS, LAYOUTS, STARTS, layout_grid
from ...spaces import Box, Discrete, batch_space
from ._grid import (ACTIONS_CARDINAL, ACTIONS_ORDINAL, GridEnvBase, GridObsSpec, create_action_probability_matrix,
                    discrete_state_grid)


def get_number_abstract_states(grid):
    """observations.py:32-41."""
    return len(np.unique(grid)) - 1


def get_observation_space_and_spec(obs_type, grid, obs_n):
    """rooms.py:15-68 lowered to a GridObsSpec."""
    is_vector = "vector" in obs_type
    has_goal = "goal" in obs_type
    a_max = np.array(grid.shape) - 2
    if "room" in obs_type:
        n = get_number_abstract_states(grid)
        if has_goal:
            return Discrete(int(n ** 2)), GridObsSpec(_lib.GP_OBS_TABLE, t1=grid, t2=n * grid)
        return Discrete(int(n)), GridObsSpec(_lib.GP_OBS_TABLE, t1=grid)
    if "mdp" in obs_type:
        if is_vector:
            if has_goal:
                return Box(1, np.tile(a_max, 2), (4,), dtype=int), GridObsSpec(_lib.GP_OBS_COORDS, goal=True)
            return Box(1, a_max, (2,), dtype=int), GridObsSpec(_lib.GP_OBS_COORDS)
        n, state_grid = discrete_state_grid(grid)
        if has_goal:
            return Discrete(int(n ** 2)), GridObsSpec(_lib.GP_OBS_TABLE, t1=state_grid, t2=n * state_grid)
        return Discrete(int(n)), GridObsSpec(_lib.GP_OBS_TABLE, t1=state_grid)
    if "hansen" in obs_type:
        base_n = 8 if "8" in obs_type else 4
        if is_vector:
            if has_goal:
                return Box(0, 2, (base_n,), dtype=int), GridObsSpec(_lib.GP_OBS_HANSEN_VEC, base_n, goal=True)
            return Box(0, 1, (base_n,), dtype=int), GridObsSpec(_lib.GP_OBS_HANSEN_VEC, base_n)
        return Discrete(int(2 ** base_n * (base_n + 1))), GridObsSpec(_lib.GP_OBS_HANSEN, base_n, goal=True)
    if "grid" in obs_type:
        return Box(0, 2, (obs_n, obs_n), dtype=int), GridObsSpec(_lib.GP_OBS_WINDOW, n=obs_n)
    raise NotImplementedError("Observation type not recognized")


class RoomsEnv(GridEnvBase):
    """Vectorized ROOMS (rooms.py:71) on MI355X. Extra kwargs: `device`, `rng_mode`."""
    metadata = {"name": "Rooms", "render_modes": ["human", "rgb_array"], "render_fps": 10}
    _ndim = 2

    def __init__(self, num_envs, layout="4", time_limit=500, obs_type="mdp", obs_n=3, action_failure_probability=0.2,
                 action_type="ordinal", agent_xy=None, goal_xy=(0, 0), step_reward=0.0, wall_reward=0.0,
                 goal_reward=1.0, render_mode=None, device=None, rng_mode="numpy", obs_dtype=None,
                 **kwargs):
        assert layout in LAYOUTS
        self.metadata = dict(self.metadata)
        self.metadata["name"] += f"__{layout}__{action_type}__{obs_type}"
        grid = layout_grid(layout)
        if "b" in layout:
            layout = layout[:-1]
        self.grid = grid
        self.gridshape = np.array(grid.shape)
        self.single_observation_space, spec = get_observation_space_and_spec(obs_type, grid, obs_n)
        self.valid_states = np.flatnonzero(grid >= 0)
        self.actions = ACTIONS_CARDINAL if action_type == "cardinal" else ACTIONS_ORDINAL
        self.num_envs = num_envs
        self.single_action_space = Discrete(self.actions.shape[0])
        self.action_space = batch_space(self.single_action_space, num_envs)
        self.observation_space = batch_space(self.single_observation_space, num_envs)
        self.time_limit = time_limit
        self.step_reward, self.goal_reward, self.wall_reward = step_reward, goal_reward, wall_reward
        self.render_mode = render_mode
        H, W = grid.shape
        fixed_goal = -1
        if goal_xy is not None:  # rooms.py:153-158
            goal_yx = tuple(reversed(goal_xy))
            if grid[goal_yx] < 0:
                goal_yx = tuple(reversed(ENDS[layout]))
            # ENDS["32"] lies outside its 25x49 grid: an unreachable goal (flat index >= cells)
            fixed_goal = int(goal_yx[0] * W + goal_yx[1])
            self._goal_yx_fixed = np.array(goal_yx)
        fixed_agent = -1
        if agent_xy is not None:
            # rooms.py:166 indexes the grid with an ndarray and raises; evident intent implemented
            agent_yx = tuple(reversed(agent_xy))
            if grid[agent_yx] < 0:
                agent_yx = tuple(reversed(STARTS[layout]))
            fixed_agent = int(agent_yx[0] * W + agent_yx[1])
        self.action_matrix = create_action_probability_matrix(self.actions.shape[0], action_failure_probability)
        if spec.kind == _lib.GP_OBS_COORDS and spec.goal and fixed_goal >= H * W:
            pass  # coordinates of an off-grid goal are reported as-is (no indexing)
        self._create_grid(_lib.GP_FLAVOR_ROOMS, grid, self.actions.shape[0], action_failure_probability, spec,
                          fixed_goal, fixed_agent, time_limit, (step_reward, wall_reward, goal_reward), num_envs,
                          device, rng_mode, obs_dtype)
        self._fixed_goal_yx = (goal_yx[0], goal_yx[1]) if goal_xy is not None else None

    def reset(self, *, seed=None, options=None):
        """Reset all environments, set seed if given (rooms.py:177-189). Returns obs only."""
        return self._reset_impl(seed)

    @property
    def agent_yx(self):
        return self._cells_to_coords(self.get_state()[0].long())

    @property
    def goal_yx(self):
        g = self.get_state()[1].long()
        if self._fixed_goal_yx is not None:
            torch = __import__("torch")
            return torch.tensor(self._fixed_goal_yx, device=self.device).expand(self.num_envs, 2).clone()
        return self._cells_to_coords(g)
