"""Lowering of the reference's grid-env constructor kwargs to the C ABI's gp_grid_config."""
import ctypes

import numpy as np

from ... import _lib
from ...core import NativeVecEnv, _torch

# action_utils.py:16-33 (N, NE, E, SE, S, SW, W, NW; cardinal = every other)
ACTIONS_ORDINAL = np.array([[-1, 0], [-1, 1], [0, 1], [1, 1], [1, 0], [1, -1], [0, -1], [-1, -1]])
ACTIONS_CARDINAL = ACTIONS_ORDINAL[::2]
ACTIONS_ORDINAL_Z = np.concatenate((np.zeros((8, 1), dtype=int), ACTIONS_ORDINAL), -1)
ACTIONS_CARDINAL_Z = ACTIONS_ORDINAL_Z[::2]
ACTION_NAMES_ORDINAL = ["N", "NE", "E", "SE", "S", "SW", "W", "NW"]
ACTION_NAMES_CARDINAL = ACTION_NAMES_ORDINAL[::2]


def create_action_probability_matrix(action_n=8, action_failure_probability=0.2):
    """action_utils.py:38-48."""
    probs = np.full((action_n, action_n), action_failure_probability / (action_n - 1), dtype=np.float64)
    np.fill_diagonal(probs, 1 - action_failure_probability)
    return probs


def discrete_state_grid(grid):
    """observations.py:16-29: (n_states, state index per cell)."""
    n = int((grid >= 0).sum())
    return n, ((grid >= 0).cumsum() - 1).reshape(grid.shape)


class GridObsSpec:
    """obs_kind + tables for gp_grid_config (obs_table arrays must outlive gp_create)."""

    def __init__(self, kind, dirs=4, goal=False, n=3, t1=None, t2=None):
        self.kind, self.dirs, self.goal, self.n = kind, dirs, goal, n
        self.t1 = None if t1 is None else np.ascontiguousarray(t1, dtype=np.int32).ravel()
        self.t2 = None if t2 is None else np.ascontiguousarray(t2, dtype=np.int32).ravel()


def _i32ptr(a):
    if a is None:
        return ctypes.POINTER(ctypes.c_int32)()
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


class GridEnvBase(NativeVecEnv):
    """A GP_KIND_GRID env (ROOMS / multistory FourRooms)."""
    _ndim = 2

    def _set_obs_dtype(self, obs_dtype, spec):
        """obs_dtype: None / "native" (int32 scalars, uint8 vectors / windows: the compact layout the kernels
        write), "reference" (the reference's own arrays: float64 for the scalar Hansen obs, whose goal multiplier
        is a float array (msrooms.py:180-189, observations.py:62-71), int64 for every other obs), or an
        explicit torch dtype / name. The cast runs on the device after the step."""
        torch = _torch()
        if obs_dtype is None or obs_dtype == "native":
            self._obs_cast = None
        elif obs_dtype == "reference":
            self._obs_cast = torch.float64 if spec.kind == _lib.GP_OBS_HANSEN else torch.int64
        elif isinstance(obs_dtype, torch.dtype):
            self._obs_cast = obs_dtype
        elif isinstance(obs_dtype, str) and isinstance(getattr(torch, obs_dtype, None), torch.dtype):
            self._obs_cast = getattr(torch, obs_dtype)
        else:
            raise ValueError(f"obs_dtype must be None, 'native', 'reference' or a torch dtype, got {obs_dtype!r}")

    def _create_grid(self, flavor, cells, n_actions, p_fail, spec, fixed_goal, fixed_agent, time_limit, rewards,
                     num_envs, device, rng_mode, obs_dtype=None):
        cells = np.ascontiguousarray(cells, dtype=np.int32)
        shape = cells.shape if cells.ndim == 3 else (1,) + cells.shape
        self._cells_keep = cells
        self._spec_keep = spec
        cfg = _lib.GridConfig()
        cfg.flavor = flavor
        cfg.depth, cfg.height, cfg.width = shape
        cfg.cells = _i32ptr(cells)
        cfg.n_actions = n_actions
        cfg.action_failure_probability = float(p_fail)
        cfg.obs_kind = spec.kind
        cfg.obs_dirs = spec.dirs
        cfg.obs_goal = int(bool(spec.goal))
        cfg.obs_n = spec.n
        cfg.obs_table = _i32ptr(spec.t1)
        cfg.obs_table2 = _i32ptr(spec.t2)
        cfg.fixed_goal = fixed_goal
        cfg.fixed_agent = fixed_agent
        cfg.time_limit = int(time_limit)
        cfg.step_reward, cfg.wall_reward, cfg.goal_reward = (float(r) for r in rewards)
        self._shape3 = shape
        self._create(_lib.GP_KIND_GRID, cfg, num_envs, device, rng_mode)
        self._obs_window = spec.n if spec.kind == _lib.GP_OBS_WINDOW else None
        self._set_obs_dtype(obs_dtype, spec)

    def _obs_shape(self):
        if self._obs_window:
            return (self.num_envs, self._obs_window, self._obs_window)
        return super()._obs_shape()

    # ---- state as coordinates (agent_zyx / goal_zyx / elapsed of the reference) ----
    def _cells_to_coords(self, c):
        D, H, W = self._shape3
        z, y, x = c // (H * W), (c // W) % H, c % W
        out = _torch().stack((z, y, x), -1)
        return out if self._ndim == 3 else out[:, 1:]

    def _coords_to_cells(self, zyx):
        D, H, W = self._shape3
        t = _torch().as_tensor(np.asarray(zyx) if not isinstance(zyx, _torch().Tensor) else zyx,
                               device=self.device).to(_torch().int64)
        if self._ndim == 2:
            return (t[:, 0] * W + t[:, 1]).to(_torch().int32)
        return ((t[:, 0] * H + t[:, 1]) * W + t[:, 2]).to(_torch().int32)

    def get_state(self):
        """(agent cells, goal cells, elapsed) as int32 device tensors [B]."""
        torch = _torch()
        a, g, e = (torch.empty(self.num_envs, dtype=torch.int32, device=self.device) for _ in range(3))
        self._get_state_raw([a, g, e])
        return a, g, e

    def set_state(self, agent_cells=None, goal_cells=None, elapsed=None):
        torch = _torch()
        conv = lambda x: None if x is None else torch.as_tensor(x, device=self.device).to(torch.int32).contiguous()  # noqa: E731
        bufs = [conv(agent_cells), conv(goal_cells), conv(elapsed)]
        self._set_state_raw(bufs)
        torch.cuda.current_stream(self.device).synchronize()

    @property
    def elapsed(self):
        return self.get_state()[2].to(_torch().int64)
