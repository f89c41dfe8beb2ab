"""Multistory FourRooms — drop-in for `gym_po.envs.rooms.msrooms.MultistoryFourRoomsEnv`
(msrooms.py:257-432): same constructor, spaces, reset/step semantics; the batched step runs in
the HIP kernels of libgympo_amd.so and returns torch-ROCm tensors.
"""
from enum import IntEnum

import numpy as np

from ... import _lib
from ...maps import FR_MAP
from ...spaces import Box, Discrete, batch_space
from ._grid import (ACTIONS_CARDINAL_Z, ACTIONS_ORDINAL_Z, GridEnvBase, GridObsSpec, create_action_probability_matrix,
                    discrete_state_grid)

END_XYZ = (9, 7, -1)      # msrooms.py:17 east hallway
START_XYZ = (1, 1, 0)     # msrooms.py:18
UPSTAIRS_YX = np.array([1, 11])    # msrooms.py:23
DOWNSTAIRS_YX = np.array([11, 1])  # msrooms.py:24


class GR_CNST(IntEnum):  # msrooms.py:27-31
    wall = 0
    goal = 1
    stair_down = 2
    stair_up = 3


MAX_GR_CNST = int(max(GR_CNST))


def rooms_map_to_multistory(map=FR_MAP, num_floors=1):
    """msrooms.py:69-90: walk map (rooms aliased to 1, stairs 2/3) and room map."""
    walk = np.array(map).copy()
    walk[np.array(map) > 0] = 1
    ms = np.stack([walk for _ in range(num_floors)], 0)
    n_rooms = np.array(map).max() - 1
    ms_rooms = np.stack([np.array(map)[np.array(map) > 0] + i * n_rooms for i in range(num_floors)], 0)
    if num_floors > 1:
        ms[1:, DOWNSTAIRS_YX[0], DOWNSTAIRS_YX[1]] = GR_CNST.stair_down
        ms[:-1, UPSTAIRS_YX[0], UPSTAIRS_YX[1]] = GR_CNST.stair_up
    return ms, ms_rooms


def get_observation_space_and_spec(obs_type, ms_grid, obs_n=3):
    """msrooms.py:192-254 lowered to a GridObsSpec (the obs function runs on the GPU)."""
    is_vector = "vector" in obs_type
    has_goal = "goal" in obs_type
    a_max = np.array(ms_grid.shape) - 2
    a_max[0] += 1
    a_min = np.array([0, 1, 1])
    if "room" in obs_type:
        assert not is_vector
        offset = len(GR_CNST)
        n = int(ms_grid.max() - offset)
        if has_goal:
            space = Discrete(int(n ** 2))
            return space, GridObsSpec(_lib.GP_OBS_TABLE, t1=ms_grid - offset, t2=n * (ms_grid - offset))
        space = Discrete(int(n))  # n <= 0: raises, as gymnasium does for the reference
        return space, GridObsSpec(_lib.GP_OBS_TABLE, t1=ms_grid)
    if "mdp" in obs_type:
        if is_vector:
            if has_goal:
                return (Box(np.tile(a_min, 2), np.tile(a_max, 2), (6,), dtype=int),
                        GridObsSpec(_lib.GP_OBS_COORDS, goal=True))
            return Box(a_min, a_max, (3,), dtype=int), GridObsSpec(_lib.GP_OBS_COORDS)
        n, state_grid = discrete_state_grid(ms_grid - 1)
        if has_goal:
            return Discrete(int(n ** 2)), GridObsSpec(_lib.GP_OBS_TABLE, t1=state_grid, t2=n * state_grid)
        return Discrete(int(n)), GridObsSpec(_lib.GP_OBS_TABLE, t1=state_grid)
    if "hansen" in obs_type:
        base_n = 8 if "8" in obs_type else 4
        if is_vector:
            if has_goal:
                return Box(0, 3, (base_n,), dtype=int), GridObsSpec(_lib.GP_OBS_HANSEN_VEC, base_n, goal=True)
            return Box(0, 2, (base_n,), dtype=int), GridObsSpec(_lib.GP_OBS_HANSEN_VEC, base_n)
        return Discrete(int(3 ** base_n * (base_n + 1))), GridObsSpec(_lib.GP_OBS_HANSEN, base_n, goal=True)
    raise NotImplementedError("Observation type not recognized")


class MultistoryFourRoomsEnv(GridEnvBase):
    """Vectorized Multistory FourRooms (msrooms.py:257) on MI355X.

    Extra keyword arguments beyond the reference: `device` (torch device, default current),
    `rng_mode` ("numpy": seed-identical to the reference; "philox": counter-based, fusable
    rollouts; "replay": pre-decided draws).
    """
    metadata = {"name": "MultistoryFourRoomsV2", "render_modes": ["human", "rgb_array"], "render_fps": 10}
    _ndim = 3

    def __init__(self, num_envs, grid_z=1, floor_map=FR_MAP, time_limit=500, obs_type="mdp", obs_n=3,
                 action_failure_probability=1.0 / 3, action_type="cardinal", agent_xyz=None, goal_xyz=END_XYZ,
                 step_reward=0.0, wall_reward=0.0, goal_reward=1.0, render_mode=None, device=None,
                 rng_mode="numpy", obs_dtype=None, **kwargs):
        self.grid, self.room_grid = rooms_map_to_multistory(floor_map, grid_z)
        self.metadata = dict(self.metadata)
        self.metadata["name"] += f"{grid_z}__{action_type}__{obs_type}"
        self.gridshape = np.array(self.grid.shape)
        self.single_observation_space, spec = get_observation_space_and_spec(obs_type, self.grid, obs_n)
        spawn_vs = np.array(np.nonzero(self.grid > GR_CNST.wall))
        self.valid_states = np.flatnonzero(self.grid > GR_CNST.wall)
        self.valid_agent_states = np.ravel_multi_index(spawn_vs[:, spawn_vs[0] == 0], self.grid.shape)
        self.valid_goal_states = np.ravel_multi_index(spawn_vs[:, spawn_vs[0] == self.gridshape[0] - 1],
                                                      self.grid.shape)
        self.render_mode = render_mode
        self.actions = ACTIONS_CARDINAL_Z if action_type == "cardinal" else ACTIONS_ORDINAL_Z
        self.num_envs = num_envs
        self.single_action_space = Discrete(self.actions.shape[0])
        self.action_space = batch_space(self.single_action_space, num_envs)
        self.observation_space = batch_space(self.single_observation_space, num_envs)
        self.time_limit = time_limit
        self.step_reward, self.goal_reward, self.wall_reward = step_reward, goal_reward, wall_reward
        # msrooms.py:341-364
        fixed_goal = -1
        if goal_xyz is not None:
            goal_zyx = tuple(reversed(goal_xyz))
            if self.grid[goal_zyx] <= MAX_GR_CNST:
                goal_zyx = tuple(reversed(END_XYZ))
            goal_zyx = np.array(goal_zyx)
            if goal_zyx[0] == -1:
                goal_zyx[0] = self.gridshape[0] - 1
            fixed_goal = int(np.ravel_multi_index(tuple(goal_zyx), self.grid.shape))
        fixed_agent = -1
        if agent_xyz is not None:
            # The reference indexes the grid with an ndarray here (msrooms.py:356) and raises;
            # we implement the evident intent (a wall spawn falls back to START_XYZ).
            agent_zyx = tuple(reversed(agent_xyz))
            if self.grid[agent_zyx] == GR_CNST.wall:
                agent_zyx = tuple(reversed(START_XYZ))
            fixed_agent = int(np.ravel_multi_index(tuple(agent_zyx), self.grid.shape))
        self.action_matrix = create_action_probability_matrix(self.actions.shape[0], action_failure_probability)
        self._create_grid(_lib.GP_FLAVOR_MULTISTORY, self.grid, self.actions.shape[0], action_failure_probability,
                          spec, fixed_goal, fixed_agent, time_limit, (step_reward, wall_reward, goal_reward),
                          num_envs, device, rng_mode, obs_dtype)

    def reset(self, *, seed=None, options=None):
        """Reset all environments, set seed if given (msrooms.py:369-381). Returns (obs, {})."""
        return self._reset_impl(seed), {}

    @property
    def agent_zyx(self):
        return self._cells_to_coords(self.get_state()[0].long())

    @property
    def goal_zyx(self):
        return self._cells_to_coords(self.get_state()[1].long())
