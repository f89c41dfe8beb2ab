"""(PO-)Taxi — drop-in for `gym_po.envs.extended_taxi` (extended_taxi.py:149-377).

Same constructor, attributes, spaces and reset/step semantics as `TaxiVecEnv`; the batched step,
the task/episode resets and the observation builder run in the HIP kernels of libgympo_amd.so
(csrc/taxi.hip) and return torch-ROCm tensors.

RNG: `"philox"` (default, the fast path) draws from the *exact* law of the reference's reset
(`multinomial(ns, p, b).argmax(-1)`, :344-352; `reset_distribution`, computed in closed form) and from the
exact passenger/destination law of :354-364, counter-based per (env, step). `"numpy"` follows the
reference's own PCG64 stream draw for draw (the transitions and the reset ranking grid-wide above 1,024
envs; the buffered Lemire `integers` calls across a workgroup by stream position, and numpy's
random_multinomial / random_binomial_inversion reset rows evaluated grid-wide at speculated stream offsets
and chained in order, csrc/taxi.hip), so a seeded run reproduces the reference's trajectories and final
`np_random` state (4M envs: 835 us/step, ~3.3x the philox step).
`"replay"` takes caller-decided draws. The step itself uses no randomness.

Extra keyword arguments beyond the reference: `device`, `rng_mode`, `one_hot` (emit the observation
index one-hot as uint8 [B, n_obs], a build-side encoding).
"""
import ctypes
from functools import partial

import numpy as np

from .. import _lib
from ..core import NativeVecEnv, _torch
from ..maps import EXTENDED_TAXI_MAP, TAXI_MAP
from ..spaces import Box, Discrete, batch_space
from .._lib import check, lib


def convert_str_map_to_walled_np_str(map):
    """extended_taxi.py:55-69: bordered char map, navigation grid, reduced->bordered coordinates."""
    bordered = np.pad(np.asarray(map, dtype="c").astype(str), 1, constant_values="|")
    if (bordered == ":").any():
        return bordered, bordered[1:-1, 1:-1:2], (lambda r, c: (r + 1, 2 * c + 1))
    return bordered, bordered[1:-1, 1:-1], (lambda r, c: (r + 1, c + 1))


def compute_obs_space(tgrid, n_locs=4, hansen=False):
    """extended_taxi.py:72-81."""
    n_t = 2 ** 4 if hansen else tgrid.shape[0] * tgrid.shape[1]
    return int(n_t * n_locs * (n_locs + 1))


def decode_state(states, y=5, n_locs=4):
    """extended_taxi.py:84-94."""
    d = states % n_locs
    tmp = states // n_locs
    p = tmp % (n_locs + 1)
    tmp = tmp // (n_locs + 1)
    return tmp // y, tmp % y, p, d


def encode_state(r, c, p, d, y=5, n_locs=4):
    """extended_taxi.py:97-99."""
    return ((r * y + c) * (n_locs + 1) + p) * n_locs + d


def generate_hansen_map(bordered_map, tgrid, cc):
    """extended_taxi.py:102-114: wall bits N=1, S=2, W=4, E=8."""
    h = np.zeros(tgrid.shape, dtype=int)
    w = (bordered_map == "|").astype(int)
    for r in range(h.shape[0]):
        for c in range(h.shape[1]):
            br, bc = cc(r, c)
            h[r, c] = w[br - 1, bc] + 2 * w[br + 1, bc] + 4 * w[br, bc - 1] + 8 * w[br, bc + 1]
    return h


def get_locations_from_np_str_map(map):
    """extended_taxi.py:117-118."""
    return np.nonzero((map != "|") & (map != " ") & (map != ":"))


class TaxiVecEnv(NativeVecEnv):
    """Vectorized Taxi environment (extended_taxi.py:149) on MI355X."""
    metadata = {"render_modes": ["human", "rgb_array"], "render_fps": 5, "name": "Taxi"}
    ACTIONS_YX = np.array([[-1, 0], [1, 0], [0, -1], [0, 1], [0, 0]], dtype=int)
    ACTION_NAMES = ["North", "South", "West", "East", "Pickup/Dropoff"]
    ACTION_DICT = {i: n for i, n in enumerate(ACTION_NAMES)}

    def __init__(self, num_envs=1, time_limit=200, num_passengers=1, map=TAXI_MAP, hansen_obs=False,
                 reward_goal=1.0, reward_bad=-0.5, reward_any=-0.05, render_mode=None, device=None,
                 rng_mode="philox", one_hot=False):
        self.render_mode = render_mode
        self.is_vector_env = True
        self.num_envs = num_envs
        self.GOAL_MOVE, self.BAD_MOVE, self.ANY_MOVE = reward_goal, reward_bad, reward_any
        self.desc, self.tgrid, self.cc = convert_str_map_to_walled_np_str(map)
        self.contains_pseudo_walls = bool((self.desc == ":").any())
        self.hansen_encodings = generate_hansen_map(self.desc, self.tgrid, self.cc)
        self.rows, self.cols = self.tgrid.shape
        self.locs = get_locations_from_np_str_map(self.tgrid)
        self.np_locs = np.array(self.locs).T
        self.nlocs = self.np_locs.shape[0]
        self.np_locs = np.concatenate((self.np_locs, [[-1, -1]]))
        self.time_limit = time_limit
        self.last_action = None
        self.single_action_space = Discrete(len(self.ACTIONS_YX))
        self.action_space = batch_space(self.single_action_space, num_envs)
        self.na = self.single_action_space.n
        self.ns = compute_obs_space(self.tgrid, self.nlocs, False)
        self.no = compute_obs_space(self.tgrid, self.nlocs, hansen_obs)
        self.one_hot = bool(one_hot)
        if self.one_hot:
            self.single_observation_space = Box(0, 1, (self.no,), dtype=np.uint8)
        else:
            self.single_observation_space = Discrete(self.no)
        self.observation_space = batch_space(self.single_observation_space, num_envs)
        self.encode = partial(encode_state, y=self.cols, n_locs=self.nlocs)
        self.decode = partial(decode_state, y=self.cols, n_locs=self.nlocs)
        self.state_distribution = np.zeros(self.ns)
        valid = np.array([self.encode(r, c, p, d) for r in range(self.rows) for c in range(self.cols)
                          if self.tgrid[r, c] != "|" for p in range(self.nlocs) for d in range(self.nlocs) if d != p])
        self.valid_states = valid
        self.state_distribution[valid] += 1
        self.state_distribution /= self.state_distribution.sum()
        self.hansen = bool(hansen_obs)
        if hansen_obs:
            self.name = "HansenTaxi-v4"
        self.n_dropoffs = num_passengers
        # lower to the C ABI (gp_taxi_config)
        desc_bytes = "".join("".join(row) for row in self.desc).encode("ascii")
        self._desc_keep = ctypes.create_string_buffer(desc_bytes, len(desc_bytes))
        self._locs_keep = np.ascontiguousarray(np.array(self.locs).T, dtype=np.int32).ravel()
        cfg = _lib.TaxiConfig()
        cfg.rows, cfg.cols = self.rows, self.cols
        cfg.desc_rows, cfg.desc_cols = self.desc.shape
        cfg.desc = ctypes.cast(self._desc_keep, ctypes.c_char_p)
        cfg.pseudo_walls = int(self.contains_pseudo_walls)
        cfg.n_locs = self.nlocs
        cfg.locs = self._locs_keep.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        cfg.num_passengers = int(num_passengers)
        cfg.time_limit = int(time_limit)
        cfg.obs_kind = _lib.GP_OBS_HANSEN if self.hansen else _lib.GP_OBS_TABLE
        cfg.one_hot = int(self.one_hot)
        cfg.reward_goal, cfg.reward_bad, cfg.reward_any = float(reward_goal), float(reward_bad), float(reward_any)
        self._create(_lib.GP_KIND_TAXI, cfg, num_envs, device, rng_mode)

    # ---- reference surface ----
    def reset(self, *, seed=None, options=None):
        """Fully reset all environments (extended_taxi.py:232-242). Returns (obs, {})."""
        self.lastaction = None
        return self._reset_impl(seed), {}

    @property
    def reset_distribution(self):
        """P(start state = valid_states[k]): the exact law of multinomial(ns, state_distribution).argmax()."""
        out = (ctypes.c_double * len(self.valid_states))()
        n = lib().gp_taxi_reset_distribution(self._handle, out, len(self.valid_states))
        if n < 0:
            check(n, "gp_taxi_reset_distribution")
        return np.array(out[:n])

    def get_state(self):
        """(s, elapsed, n_dropoffs_completed) as int32 device tensors [B]."""
        torch = _torch()
        s, e, n = (torch.empty(self.num_envs, dtype=torch.int32, device=self.device) for _ in range(3))
        self._get_state_raw([s, e, n])
        return s, e, n

    def set_state(self, s=None, elapsed=None, n_dropoffs=None):
        torch = _torch()
        conv = lambda x: None if x is None else torch.as_tensor(x, device=self.device).to(torch.int32).contiguous()  # noqa: E731
        self._set_state_raw([conv(s), conv(elapsed), conv(n_dropoffs)])
        torch.cuda.current_stream(self.device).synchronize()

    @property
    def s(self):
        return self.get_state()[0].to(_torch().int64)

    @property
    def elapsed(self):
        return self.get_state()[1].to(_torch().int64)

    @property
    def n_dropoffs_completed(self):
        return self.get_state()[2].to(_torch().float64)

    def render(self, idx=None):
        """rgb_array of envs idx = arange(n) (default: env 0), rendered on the device (extended_taxi.py:289-331):
        the bordered char map coloured with the shared palette (+64 on the taxi's neighbours for Hansen
        envs), frames tiled by tile_images, resized like cv2.resize(img, (h*16, w*16), INTER_AREA) with (h, w)
        the bordered map's shape, and a 20-column black text band. Returns a uint8 [w*16, h*16 + 20, 3] device
        tensor. The reference indexes its frame stack with the env ids, so only idx = arange(n) is meaningful
        there; other idx raise ValueError. Not drawn: the last-action caption (cv2.putText). The resize
        restates OpenCV's INTER_AREA (cv2 is absent: parity unpinned; the tiled frame is pinned)."""
        torch = _torch()
        n = 1 if idx is None else len(idx)
        if idx is not None and not np.array_equal(np.asarray(idx), np.arange(n)):
            raise ValueError("render(idx): the reference's frame indexing only works for idx = arange(n)")
        dims = (ctypes.c_int32 * 4)()
        check(lib().gp_taxi_render(self._handle, n, int(self.hansen), None, dims, None), "gp_taxi_render")
        rows, cols, fr, fc = dims
        tiled = torch.empty((rows, cols, 3), dtype=torch.uint8, device=self.device)
        stream = self._stream()
        check(lib().gp_taxi_render(self._handle, n, int(self.hansen), ctypes.c_void_p(tiled.data_ptr()), dims,
                                   stream), "gp_taxi_render")
        dh, dw = fc * 16, fr * 16   # cv2 dsize = (width, height) = (frame_rows*16, frame_cols*16)
        out = torch.zeros((dh, dw + 20, 3), dtype=torch.uint8, device=self.device)
        check(lib().gp_resize_area_u8(ctypes.c_void_p(tiled.data_ptr()), rows, cols, 3,
                                      ctypes.c_void_p(out.data_ptr()), dh, dw, (dw + 20) * 3, stream),
              "gp_resize_area_u8")
        self._last_tiled = tiled
        return out

    def set_replay(self, reset_states=None, pd=None):
        """rng_mode='replay': per-env start states (int32 [B]) and passenger*nlocs+destination pairs
        (int32 [B]) used by the next reset/step wherever an env resets / completes a task."""
        torch = _torch()
        conv = lambda x: None if x is None else torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x, device=self.device).to(torch.int32).contiguous()  # noqa: E731
        super().set_replay(i0=conv(reset_states), i1=conv(pd))


HansenTaxiVecEnv = partial(TaxiVecEnv, hansen_obs=True)
ExtendedTaxiVecEnv = partial(TaxiVecEnv, map=EXTENDED_TAXI_MAP)
ExtendedHansenTaxiVecEnv = partial(HansenTaxiVecEnv, map=EXTENDED_TAXI_MAP)
