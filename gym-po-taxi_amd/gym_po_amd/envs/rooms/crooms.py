"""C-ROOMS — drop-in for `gym_po.envs.rooms.crooms.CRoomsEnv` (crooms.py:91-338).

Same constructor, spaces and reset/step semantics; the continuous step (action noise, velocity,
wall bounce with in-cell resampling, goal test, resets, observation functions) runs in the HIP
kernels of libgympo_amd.so (csrc/crooms.hip) in float64, operation for operation as the reference,
with float32 (default) or float64 I/O.

RNG: `"philox"` (default) draws the reference's laws from a counter-based generator (every env-step
independent, full-chip kernels); `"numpy"` draws the reference's own PCG64 stream word for word (numpy's
ziggurat normals and buffered Lemire choices, seed-identical with the reference; up to 1,024 envs one
workgroup resolves the data-dependent word counts, above that every draw call is resolved over all of its
stream positions by grid-wide kernels, at any size: 7.0-7.3e9 env-steps/s at 2^21 envs (286-299 us per
step), ~20x below philox's 14 us, profiles/r05_crooms_numpy_rate.txt);
`"replay"` takes the reference stream's values per env (bit-exact parity tests).

Philox-mode normals are Box-Muller on float32 hardware log2 / sqrt / sin / cos (a 53-bit u1, so the radius
reaches 8.57 sigma), scaled in float64: the noise has float32 precision (~1e-7 relative) while the state is
float64 -- the reference's law, not its values (csrc/crooms.hip box_muller_pair).

Extra keyword arguments beyond the reference: `device`, `rng_mode`, `dtype` (torch.float32 (default)
or torch.float64 for the continuous actions and observations).
"""
import numpy as np

from ... import _lib
from ...core import NativeVecEnv, _torch
from ...maps import ENDS, LAYOUTS, STARTS, layout_grid
from ...spaces import Box, Discrete, batch_space
from ._grid import ACTIONS_CARDINAL, ACTIONS_ORDINAL, _i32ptr, create_action_probability_matrix, discrete_state_grid
from .rooms import get_number_abstract_states


def coord_to_grid(coord_yx, cell_size=1.0):
    """utils.py:15-20."""
    return np.floor(np.asarray(coord_yx) / cell_size).astype(int)


def grid_to_coord(grid_yx, cell_size=1.0):
    """utils.py:7-12."""
    return (np.asarray(grid_yx) * cell_size) + (cell_size / 2)


def get_observation_space_and_spec(obs_type, grid, obs_m):
    """crooms.py:16-88: (space, (obs_kind, dirs, goal, n, t1, t2))."""
    is_vector = "vector" in obs_type
    has_goal = "goal" in obs_type
    a_max = np.array(grid.shape) - 1 - 1e-6
    if "room" in obs_type:
        n = get_number_abstract_states(grid)
        if has_goal:
            return Discrete(int(n ** 2)), (_lib.GP_OBS_TABLE, 4, False, 3, grid, n * grid)
        return Discrete(int(n)), (_lib.GP_OBS_TABLE, 4, False, 3, grid, None)
    if "mdp" in obs_type:
        if is_vector:
            if has_goal:
                return Box(1.0, np.tile(a_max, 2), (4,)), (_lib.GP_OBS_F32, 4, True, 3, None, None)
            return Box(1.0, a_max, (2,)), (_lib.GP_OBS_F32, 4, False, 3, None, None)
        n, sg = discrete_state_grid(grid)
        if has_goal:
            return Discrete(int(n ** 2)), (_lib.GP_OBS_TABLE, 4, False, 3, sg, n * sg)
        return Discrete(int(n)), (_lib.GP_OBS_TABLE, 4, False, 3, sg, None)
    if "hansen" in obs_type:
        base_n = 8 if "8" in obs_type else 4
        if is_vector:
            if has_goal:
                return Box(0, 2, (base_n,), dtype=int), (_lib.GP_OBS_HANSEN_VEC, base_n, True, 3, None, None)
            return Box(0, 1, (base_n,), dtype=int), (_lib.GP_OBS_HANSEN_VEC, base_n, False, 3, None, None)
        return Discrete(int(2 ** base_n * (base_n + 1))), (_lib.GP_OBS_HANSEN, base_n, True, 3, None, None)
    if "grid" in obs_type:
        return Box(0, 2, (obs_m, obs_m), dtype=int), (_lib.GP_OBS_WINDOW, 4, True, obs_m, None, None)
    raise NotImplementedError("Observation type not recognized")


class CRoomsEnv(NativeVecEnv):
    """Vectorized C-ROOMS (crooms.py:91) on MI355X."""
    metadata = {"name": "CRooms", "render.modes": ["human", "rgb_array"], "video.frames_per_second": 10}

    def __init__(self, num_envs, layout="4", time_limit=500, use_velocity=False, cell_size=1.0, obs_type="mdp",
                 obs_m=3, action_failure_probability=0.2, action_type="yx", action_std=0.2, action_power=1.0,
                 agent_xy=None, goal_xy=(0, 0), step_reward=0.0, wall_reward=0.0, goal_reward=1.0,
                 goal_threshold=0.5, render_mode=None, device=None, rng_mode="philox", dtype=None, **kwargs):
        torch = _torch()
        assert layout in LAYOUTS
        self.metadata = dict(self.metadata)
        self.metadata["name"] += f"__{layout}__{action_type}__{obs_type}"
        grid = layout_grid(layout)
        if "b" in layout:
            layout = layout[:-1]
        self.grid = grid
        self.gridshape = np.array(grid.shape)
        self.single_observation_space, spec = get_observation_space_and_spec(obs_type, grid, obs_m)
        self.valid_states = np.flatnonzero(grid >= 0)
        self.max_velocity = 5.0
        self.dtype = torch.float32 if dtype is None else dtype
        if self.dtype not in (torch.float32, torch.float64):
            raise ValueError("dtype must be torch.float32 or torch.float64")
        f64 = self.dtype == torch.float64
        if action_type == "yx":
            self.single_action_space = Box(-1.0, 1.0, (2,))
            self._action_dtype, self._action_tail = ("float64" if f64 else "float32"), (2,)
            action_kind = 0
        else:
            self.actions = ACTIONS_CARDINAL if action_type == "cardinal" else ACTIONS_ORDINAL
            self.action_matrix = create_action_probability_matrix(self.actions.shape[0], action_failure_probability)
            self.single_action_space = Discrete(self.actions.shape[0])
            action_kind = self.actions.shape[0]
        self.use_velocity = use_velocity
        self.num_envs = num_envs
        self.is_vector_env = True
        self.action_space = batch_space(self.single_action_space, num_envs)
        self.observation_space = batch_space(self.single_observation_space, num_envs)
        self.time_limit = time_limit
        self.step_reward, self.goal_reward, self.wall_reward = step_reward, goal_reward, wall_reward
        self.goal_threshold = goal_threshold
        self.cell_size = cell_size
        self.action_power = action_power
        self.render_mode = render_mode
        cfg = _lib.CRoomsConfig()
        self._cells_keep = np.ascontiguousarray(grid, dtype=np.int32)
        cfg.height, cfg.width = grid.shape
        cfg.cells = _i32ptr(self._cells_keep)
        cfg.use_velocity = int(bool(use_velocity))
        cfg.cell_size = float(cell_size)
        cfg.action_kind = action_kind
        cfg.action_f64 = int(f64)
        cfg.action_failure_probability = float(action_failure_probability)
        cfg.action_std = float(action_std or 0.0)
        cfg.action_power = float(action_power)
        kind, dirs, goal, n, t1, t2 = spec
        self._t1 = None if t1 is None else np.ascontiguousarray(t1, dtype=np.int32).ravel()
        self._t2 = None if t2 is None else np.ascontiguousarray(t2, dtype=np.int32).ravel()
        cfg.obs_kind, cfg.obs_f64, cfg.obs_dirs, cfg.obs_goal, cfg.obs_n = kind, int(f64), dirs, int(goal), n
        cfg.obs_table, cfg.obs_table2 = _i32ptr(self._t1), _i32ptr(self._t2)
        self._goal_yx_fixed = None
        if goal_xy is not None:  # crooms.py:217-224
            goal_yx = tuple(reversed(goal_xy))
            if grid[goal_yx] < 0:
                goal_yx = tuple(reversed(ENDS[layout]))
            cfg.goal_fixed, cfg.goal_y, cfg.goal_x = 1, int(goal_yx[0]), int(goal_yx[1])
            self._goal_yx_fixed = (int(goal_yx[0]), int(goal_yx[1]))
        if agent_xy is not None:
            # crooms.py:231-236 indexes the grid with an ndarray and raises; evident intent implemented
            agent_yx = tuple(reversed(agent_xy))
            if grid[agent_yx] < 0:
                agent_yx = tuple(reversed(STARTS[layout]))
            cfg.agent_fixed, cfg.agent_y, cfg.agent_x = 1, int(agent_yx[0]), int(agent_yx[1])
        cfg.time_limit = int(time_limit)
        cfg.step_reward, cfg.wall_reward, cfg.goal_reward = float(step_reward), float(wall_reward), float(goal_reward)
        cfg.goal_threshold = float(goal_threshold)
        self._obs_window = n if kind == _lib.GP_OBS_WINDOW else None
        self._create(_lib.GP_KIND_CROOMS, cfg, num_envs, device, rng_mode)

    def _obs_shape(self):
        if self._obs_window:
            return (self.num_envs, self._obs_window, self._obs_window)
        return super()._obs_shape()

    def seed(self, seed=None, spawn_key=()):
        """crooms.py:246-249: re-seed the env's generator (None -> fresh OS entropy)."""
        return super().seed(seed, spawn_key)

    def reset(self, *, seed=None, return_info=False, options=None):
        """Reset all environments, set seed if given (crooms.py:251-266). Returns obs only."""
        return self._reset_impl(seed)

    # ---- state ----
    def get_state(self):
        """(agent yx f64 [B,2], goal cell yx i32 [B,2], velocity f64 [B,2], elapsed i32 [B])."""
        torch = _torch()
        a = torch.empty((self.num_envs, 2), dtype=torch.float64, device=self.device)
        g = torch.empty((self.num_envs, 2), dtype=torch.int32, device=self.device)
        v = torch.empty((self.num_envs, 2), dtype=torch.float64, device=self.device)
        e = torch.empty(self.num_envs, dtype=torch.int32, device=self.device)
        self._get_state_raw([a, g, v, e])
        return a, g, v, e

    def set_state(self, agent_yx=None, goal_cell_yx=None, velocity=None, elapsed=None):
        torch = _torch()

        def conv(x, dt):
            if x is None:
                return None
            return torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x,
                                   device=self.device).to(dt).contiguous()
        self._set_state_raw([conv(agent_yx, torch.float64), conv(goal_cell_yx, torch.int32),
                             conv(velocity, torch.float64), conv(elapsed, torch.int32)])
        torch.cuda.current_stream(self.device).synchronize()

    @property
    def agent_yx(self):
        return self.get_state()[0]

    @property
    def goal_yx(self):
        return grid_to_coord(self.get_state()[1].cpu().numpy())

    @property
    def agent_yx_velocity(self):
        return self.get_state()[2]

    @property
    def elapsed(self):
        return self.get_state()[3].to(_torch().int64)

    def set_replay(self, u=None, goal_idx=None, agent_idx=None, noise=None, wall_noise=None):
        """rng_mode='replay': the next step's draws, per env — u: uint64 k53 action-failure uniforms
        (u = k * 2^-53) [B]; goal_idx / agent_idx: indices into valid_states [B]; noise: action noise
        f64 [B,2]; wall_noise: f64 [B,2] (the values numpy's normal() returned)."""
        torch = _torch()

        def conv(x, dt):
            if x is None:
                return None
            if isinstance(x, torch.Tensor):
                return x.to(device=self.device, dtype=dt).contiguous()
            a = np.ascontiguousarray(x)
            if dt == torch.int64:
                a = a.astype(np.uint64).view(np.int64)
            return torch.as_tensor(a, device=self.device).to(dt).contiguous()
        super().set_replay(u=conv(u, torch.int64), i0=conv(goal_idx, torch.int32), i1=conv(agent_idx, torch.int32),
                           f0=conv(noise, torch.float64), f1=conv(wall_noise, torch.float64))
