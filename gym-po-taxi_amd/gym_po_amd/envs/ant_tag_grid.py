"""Grid Ant-Tag — a build-defined grid restatement of the tag task of `gym_po.envs.ant_tag.AntTagEnv`
(ant_tag.py:88-157; the reference env is a MuJoCo ant, registered with max_episode_steps=500).

Rules (csrc/anttag.hip header): size x size arena of 1 m cells; the agent moves N/E/S/W or
stays; the target then moves away / orthogonally left / orthogonally right / not at all (uniform),
rounded to one grid step and kept inside the cage; a tag (distance <= tag_radius) pays tag_reward and
terminates; the target is observed only within visible_radius; resets put the target farther than
min_distance from the agent; truncation at time_limit steps (gymnasium TimeLimit).
Observation: int32 [ant y, ant x, target y, target x], target (-1, -1) when not visible.
"""
import math

import numpy as np

from .. import _lib
from ..core import NativeVecEnv, _torch
from ..spaces import Box, Discrete, batch_space

ACTION_NAMES = ["N", "E", "S", "W", "stay"]


class AntTagGridEnv(NativeVecEnv):
    metadata = {"render_modes": [], "name": "AntTagGrid"}

    def __init__(self, num_envs, size=10, tag_radius=1.5, visible_radius=3.0, min_distance=5.0, time_limit=500,
                 tag_reward=1.0, step_reward=0.0, device=None, rng_mode="philox"):
        self.num_envs = num_envs
        self.is_vector_env = True
        self.size = size
        self.single_action_space = Discrete(len(ACTION_NAMES))
        self.action_space = batch_space(self.single_action_space, num_envs)
        self.single_observation_space = Box(-1, size - 1, (4,), dtype=np.int32)
        self.observation_space = batch_space(self.single_observation_space, num_envs)
        self.time_limit = time_limit
        cfg = _lib.AntTagConfig()
        cfg.size = int(size)
        cfg.tag_radius2 = int(math.floor(tag_radius ** 2 + 1e-9))            # d^2 <= r^2, d^2 integer
        cfg.visible_radius2 = int(math.ceil(visible_radius ** 2 - 1e-9))     # d^2 <  r^2
        cfg.min_start_dist2 = int(math.floor(min_distance ** 2 + 1e-9))      # d^2 >  r^2
        cfg.time_limit = int(time_limit)
        cfg.tag_reward, cfg.step_reward = float(tag_reward), float(step_reward)
        self.tag_radius2, self.visible_radius2, self.min_start_dist2 = (cfg.tag_radius2, cfg.visible_radius2,
                                                                        cfg.min_start_dist2)
        if rng_mode == "numpy":
            raise _lib.GymPoError("AntTagGridEnv is build-defined: rng_mode 'philox' or 'replay'")
        self._create(_lib.GP_KIND_ANTTAG, cfg, num_envs, device, rng_mode)

    def reset(self, *, seed=None, options=None):
        return self._reset_impl(seed), {}

    def get_state(self):
        """(ant cell, target cell, elapsed) int32 [B] (cell = y * size + x)."""
        torch = _torch()
        a, t, e = (torch.empty(self.num_envs, dtype=torch.int32, device=self.device) for _ in range(3))
        self._get_state_raw([a, t, e])
        return a, t, e

    def set_state(self, ant=None, target=None, elapsed=None):
        torch = _torch()
        conv = lambda x: None if x is None else torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x, device=self.device).to(torch.int32).contiguous()  # noqa: E731
        self._set_state_raw([conv(ant), conv(target), conv(elapsed)])
        torch.cuda.current_stream(self.device).synchronize()

    def set_replay(self, choose=None, ant=None, target_idx=None):
        """rng_mode='replay': per-env target-move choice (0..3), reset ant cell and reset target index
        into the ant cell's list of admissible start cells (ascending)."""
        torch = _torch()
        conv = lambda x: None if x is None else torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x, device=self.device).to(torch.int32).contiguous()  # noqa: E731
        super().set_replay(u=conv(choose), i0=conv(ant), i1=conv(target_idx))
