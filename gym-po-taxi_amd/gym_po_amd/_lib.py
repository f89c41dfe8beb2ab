"""ctypes binding of libgympo_amd.so (the C ABI declared in include/gym_po_amd.h).

The library is built in-tree (gym-po-taxi_amd/build.py -> gym_po_amd/libgympo_amd.so). There is
no CPU fallback: if the shared library is missing or fails to load, importing an env raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GYM_PO_AMD_LIB", os.path.join(_HERE, "libgympo_amd.so"))

GP_OK = 0
GP_E_DEVICE = -5
GP_KIND_GRID, GP_KIND_TAXI, GP_KIND_CROOMS, GP_KIND_ANTTAG = 1, 2, 3, 4
GP_RNG_NUMPY, GP_RNG_PHILOX, GP_RNG_REPLAY = 0, 1, 2
RNG_MODES = {"numpy": GP_RNG_NUMPY, "philox": GP_RNG_PHILOX, "replay": GP_RNG_REPLAY}
GP_DTYPE_I32, GP_DTYPE_U8, GP_DTYPE_F32, GP_DTYPE_F64 = 0, 1, 2, 3
GP_FLAVOR_ROOMS, GP_FLAVOR_MULTISTORY = 0, 1
(GP_OBS_HANSEN, GP_OBS_HANSEN_VEC, GP_OBS_TABLE, GP_OBS_COORDS, GP_OBS_WINDOW, GP_OBS_ONEHOT,
 GP_OBS_F32) = range(7)

_i32p = ctypes.POINTER(ctypes.c_int32)
_vp = ctypes.c_void_p


class GridConfig(ctypes.Structure):
    _fields_ = [("flavor", ctypes.c_int32), ("depth", ctypes.c_int32), ("height", ctypes.c_int32),
                ("width", ctypes.c_int32), ("cells", _i32p), ("n_actions", ctypes.c_int32),
                ("action_failure_probability", ctypes.c_double), ("obs_kind", ctypes.c_int32),
                ("obs_dirs", ctypes.c_int32), ("obs_goal", ctypes.c_int32), ("obs_n", ctypes.c_int32),
                ("obs_table", _i32p), ("obs_table2", _i32p), ("fixed_goal", ctypes.c_int32),
                ("fixed_agent", ctypes.c_int32), ("time_limit", ctypes.c_int32), ("step_reward", ctypes.c_float),
                ("wall_reward", ctypes.c_float), ("goal_reward", ctypes.c_float)]


class TaxiConfig(ctypes.Structure):
    _fields_ = [("rows", ctypes.c_int32), ("cols", ctypes.c_int32), ("desc_rows", ctypes.c_int32),
                ("desc_cols", ctypes.c_int32), ("desc", ctypes.c_char_p), ("pseudo_walls", ctypes.c_int32),
                ("n_locs", ctypes.c_int32), ("locs", _i32p), ("num_passengers", ctypes.c_int32),
                ("time_limit", ctypes.c_int32), ("obs_kind", ctypes.c_int32), ("one_hot", ctypes.c_int32),
                ("reward_goal", ctypes.c_float),
                ("reward_bad", ctypes.c_float), ("reward_any", ctypes.c_float)]


class CRoomsConfig(ctypes.Structure):
    _fields_ = [("height", ctypes.c_int32), ("width", ctypes.c_int32), ("cells", _i32p),
                ("use_velocity", ctypes.c_int32), ("cell_size", ctypes.c_double), ("action_kind", ctypes.c_int32),
                ("action_f64", ctypes.c_int32), ("action_failure_probability", ctypes.c_double),
                ("action_std", ctypes.c_double), ("action_power", ctypes.c_double), ("obs_kind", ctypes.c_int32),
                ("obs_f64", ctypes.c_int32), ("obs_dirs", ctypes.c_int32), ("obs_goal", ctypes.c_int32),
                ("obs_n", ctypes.c_int32), ("obs_table", _i32p), ("obs_table2", _i32p),
                ("goal_fixed", ctypes.c_int32), ("goal_y", ctypes.c_int32), ("goal_x", ctypes.c_int32),
                ("agent_fixed", ctypes.c_int32), ("agent_y", ctypes.c_int32), ("agent_x", ctypes.c_int32),
                ("time_limit", ctypes.c_int32), ("step_reward", ctypes.c_float), ("wall_reward", ctypes.c_float),
                ("goal_reward", ctypes.c_float), ("goal_threshold", ctypes.c_double)]


class AntTagConfig(ctypes.Structure):
    _fields_ = [("size", ctypes.c_int32), ("tag_radius2", ctypes.c_int32), ("visible_radius2", ctypes.c_int32),
                ("min_start_dist2", ctypes.c_int32), ("time_limit", ctypes.c_int32),
                ("tag_reward", ctypes.c_float), ("step_reward", ctypes.c_float)]


# every symbol include/gym_po_amd.h declares: name -> (restype, argtypes)
SIGNATURES = {
    "gp_last_error": (ctypes.c_char_p, []),
    "gp_abi_version": (ctypes.c_int, []),
    "gp_create": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                 ctypes.POINTER(_vp)]),
    "gp_destroy": (None, [_vp]),
    "gp_obs_info": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "gp_num_envs": (ctypes.c_int64, [_vp]),
    "gp_seed_words": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]),
    "gp_seed": (ctypes.c_int, [_vp, ctypes.c_uint64]),
    "gp_set_rng_state": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint64)]),
    "gp_get_rng_state": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint64)]),
    "gp_reset": (ctypes.c_int, [_vp, _vp, _vp]),
    "gp_step": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gp_rollout": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gp_plan_create": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(_vp)]),
    "gp_plan_run": (ctypes.c_int, [_vp]),
    "gp_plan_destroy": (None, [_vp]),
    "gp_get_state": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "gp_set_state": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "gp_set_replay": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "gp_valid_cells": (ctypes.c_int, [_vp, ctypes.c_int, _i32p, ctypes.c_int]),
    "gp_metrics": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double)]),
    "gp_check": (ctypes.c_int, [_vp]),
    "gp_autotune": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "gp_query": (ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]),
    "gp_taxi_reset_distribution": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    "gp_taxi_render": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp, ctypes.POINTER(ctypes.c_int32), _vp]),
    "gp_resize_area_u8": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, _vp]),
    "gp_set_profiling": (ctypes.c_int, [_vp, ctypes.c_int]),
    "gp_profile_read": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
    "gp_profile_read_resolver": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double),
                                                 ctypes.POINTER(ctypes.c_int64)]),
    "gp_pcg64_seed_state": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_uint32), ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_uint64)]),
    "gp_argmax_multinomial_distribution": (ctypes.c_int, [ctypes.c_int, ctypes.c_int,
                                                          ctypes.POINTER(ctypes.c_double)]),
    "gp_standard_normal_words": (ctypes.c_int, [_vp, ctypes.c_int64, _vp, ctypes.c_int64,
                                                ctypes.POINTER(ctypes.c_int64), _vp]),
    "gp_exp_libm": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                   ctypes.c_int64, ctypes.c_int]),
    "gp_exp_host_variant": (ctypes.c_int, []),
    "gp_philox_blocks": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int, ctypes.POINTER(ctypes.c_uint32),
                                        ctypes.c_int64]),
    "gp_zig_log1p_neg": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                        ctypes.c_int64]),
    "gp_debug_set": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int64]),
    "gp_debug_reset": (None, []),
    "gp_normal_tail_counts": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int64, ctypes.POINTER(ctypes.c_double),
                                             ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                             ctypes.POINTER(ctypes.c_double), _vp]),
}

_lib = None


class GymPoError(RuntimeError):
    pass


def _bind_torch_hip_runtime():
    """Make libgympo_amd.so bind to the SAME HIP runtime torch uses (torch wheels bundle their
    own libamdhip64.so.7). Device pointers and hipStream_t handles from torch are only valid in
    that runtime, so it is loaded (RTLD_GLOBAL, same soname) before our library."""
    try:
        import torch
    except Exception:  # noqa: BLE001 - pure-C users without torch use the system runtime
        return
    tl = os.path.join(os.path.dirname(torch.__file__), "lib")
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        p = os.path.join(tl, name)
        if os.path.exists(p):
            ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)


def lib():
    """Load (once) and return the shared library. Raises if it is missing — no fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise GymPoError(f"{LIB_PATH} not found: build it with `python gym-po-taxi_amd/build.py` "
                             "(gym_po_amd has no CPU fallback)")
        _bind_torch_hip_runtime()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if not hasattr(L, name) and "GYM_PO_AMD_LIB" in os.environ:
                continue  # an explicitly chosen older build (in-call A/B tooling): bind what it has
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what=""):
    if rc != GP_OK:
        msg = lib().gp_last_error()
        raise GymPoError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc


class debug_knobs:
    """Diagnostic knobs of envs created inside the block (gp_debug_set; restored to the defaults on exit):
    disable_fused, no_staging, xmode, spin_limit, fault_block. Tests and A/B tooling only."""

    def __init__(self, **knobs):
        self.knobs = knobs

    def __enter__(self):
        for k, v in self.knobs.items():
            check(lib().gp_debug_set(k.encode(), int(v)), f"gp_debug_set({k})")
        return self

    def __exit__(self, *exc):
        lib().gp_debug_reset()
        return False


def int_to_u32_words(x):
    """numpy SeedSequence's entropy convention: little-endian uint32 words of a non-negative int."""
    if x < 0:
        raise ValueError("seed must be a non-negative int")
    words = []
    while True:
        words.append(x & 0xFFFFFFFF)
        x >>= 32
        if x == 0:
            return words
