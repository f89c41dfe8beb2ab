"""Shared host-side plumbing of the drop-in vector envs: handle lifetime, seeding with the
reference's semantics, device output allocation, reset/step/rollout through the C ABI.

The reference's vector envs are `gymnasium.Env` subclasses with `is_vector_env=True` whose
`reset(*, seed, options)` re-seeds `np_random = Generator(PCG64(SeedSequence(seed)))` when a seed
is given and whose `step(actions)` returns `(obs, rew, terminated, truncated, {})` with
same-step autoreset (msrooms.py:369-413, rooms.py:177-222, extended_taxi.py:232-287,
crooms.py:251-298). Here the state and the RNG live on the GPU; outputs are torch-ROCm tensors.
"""
import ctypes
import secrets

import numpy as np

from . import _lib
from ._lib import check, lib


def _torch():
    import torch
    return torch


class _PlanKeep:
    """Owns a gp_plan (freed with the run closure) and keeps its buffers alive."""

    def __init__(self, plan, bufs):
        self.plan, self.bufs = plan, bufs

    def __del__(self):
        try:
            if self.plan is not None:
                lib().gp_plan_destroy(self.plan)
        except Exception:  # noqa: BLE001
            pass


class NativeVecEnv:
    """Base class: one C-ABI handle, one device, one stream (the torch current stream)."""
    is_vector_env = True
    metadata = {"render_modes": [], "name": "gym_po_amd"}
    _action_dtype = "int32"
    _action_tail = ()

    def _create(self, kind, cfg, num_envs, device=None, rng_mode="numpy"):
        torch = _torch()
        if not torch.cuda.is_available():
            raise _lib.GymPoError("gym_po_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
        self._handle = None
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        device = torch.device(device)
        if device.type != "cuda":
            raise ValueError("gym_po_amd envs run on a GPU device")
        self.device = torch.device("cuda", device.index if device.index is not None else torch.cuda.current_device())
        if rng_mode not in _lib.RNG_MODES:
            raise ValueError(f"rng_mode must be one of {list(_lib.RNG_MODES)}")
        self.rng_mode = rng_mode
        self.num_envs = int(num_envs)
        h = ctypes.c_void_p()
        check(lib().gp_create(kind, ctypes.byref(cfg), self.num_envs, self.device.index, _lib.RNG_MODES[rng_mode],
                              ctypes.byref(h)), "gp_create")
        self._handle = h
        dt, w = ctypes.c_int(), ctypes.c_int()
        check(lib().gp_obs_info(h, ctypes.byref(dt), ctypes.byref(w)), "gp_obs_info")
        self._obs_dtype = {0: torch.int32, 1: torch.uint8, 2: torch.float32, 3: torch.float64}[dt.value]
        self._obs_width = w.value
        self._seeded = False
        self._replay_keep = None

    # ------------------------------------------------------------------ lifetime ----
    def close(self):
        if getattr(self, "_handle", None):
            lib().gp_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    # ------------------------------------------------------------------ helpers ----
    def _stream(self):
        return ctypes.c_void_p(_torch().cuda.current_stream(self.device).cuda_stream)

    def _obs_shape(self):
        return (self.num_envs,) if self._obs_width == 1 else (self.num_envs, self._obs_width)

    def _alloc_outputs(self, K=None):
        torch = _torch()
        lead = (self.num_envs,) if K is None else (K, self.num_envs)
        oshape = self._obs_shape() if K is None else (K,) + self._obs_shape()
        obs = torch.empty(oshape, dtype=self._obs_dtype, device=self.device)
        rew = torch.empty(lead, dtype=torch.float32, device=self.device)
        term = torch.empty(lead, dtype=torch.uint8, device=self.device)
        trunc = torch.empty(lead, dtype=torch.uint8, device=self.device)
        return obs, rew, term, trunc

    def _as_actions(self, actions, K=None):
        torch = _torch()
        dt = {"int32": torch.int32, "float32": torch.float32, "float64": torch.float64}[self._action_dtype]
        shape = ((self.num_envs,) if K is None else (K, self.num_envs)) + self._action_tail
        if isinstance(actions, torch.Tensor):
            if actions.device.type == "cpu":
                self._check_host_actions(actions.numpy())
            a = actions.to(device=self.device, dtype=dt)
        else:
            an = np.asarray(actions)
            self._check_host_actions(an)
            a = torch.as_tensor(an, device=self.device).to(dt)
        if tuple(a.shape) != shape:
            a = a.reshape(shape)
        return a.contiguous()

    def _check_host_actions(self, a):
        """Host-resident discrete actions are range-checked before upload, raising the reference's own error:
        numpy's IndexError from `action_matrix[action]` (msrooms.py:400, rooms.py:208) / `ACTIONS_YX[actions]`
        (extended_taxi.py:248); negatives in [-n, 0) wrap as numpy indexing does. Device tensors are checked
        on the device instead (GP_DERR_ACTION -> GymPoError from check() / metrics()), without a sync."""
        n = getattr(getattr(self, "single_action_space", None), "n", None)
        if n is None or self._action_dtype != "int32":
            return
        if a.dtype.kind not in "iub":  # numpy refuses non-integer index arrays (before any bounds check)
            raise IndexError("arrays used as indices must be of integer (or boolean) type")
        if a.size == 0:
            return
        lo, hi = a.min(), a.max()
        if hi >= n or lo < -n:
            flat = a.reshape(-1)
            bad = int(flat[np.flatnonzero((flat >= n) | (flat < -n))[0]])  # numpy names the first in index order
            raise IndexError(f"index {bad} is out of bounds for axis 0 with size {n}")

    def _post_obs(self, obs):
        # obs_dtype="reference" (grid envs): the reference's own dtype, cast on the device after the kernel (the
        # kernels and rollout_plan's buffers keep the compact native layout)
        cast = getattr(self, "_obs_cast", None)
        return obs if cast is None else obs.to(cast)

    # ------------------------------------------------------------------ seeding ----
    def _seed(self, seed, spawn_key=()):
        words = _lib.int_to_u32_words(int(seed))
        ent = (ctypes.c_uint32 * len(words))(*words)
        sk = (ctypes.c_uint32 * max(len(spawn_key), 1))(*(list(spawn_key) or [0]))
        check(lib().gp_seed_words(self._handle, ent, len(words), sk, len(spawn_key)), "gp_seed_words")
        self._seeded = True

    def seed(self, seed=None, spawn_key=()):
        """numpy/gymnasium seeding: SeedSequence(seed[, spawn_key]); None draws fresh OS entropy."""
        if seed is None:
            seed = secrets.randbits(128)
        self._seed(seed, spawn_key)
        return seed

    @property
    def rng_state(self):
        """The device RNG state as numpy's `PCG64.state` dict (syncs)."""
        st = (ctypes.c_uint64 * 6)()
        check(lib().gp_get_rng_state(self._handle, st), "gp_get_rng_state")
        return {"bit_generator": "PCG64", "state": {"state": (st[0] << 64) | st[1], "inc": (st[2] << 64) | st[3]},
                "has_uint32": int(st[4]), "uinteger": int(st[5])}

    @rng_state.setter
    def rng_state(self, s):
        m = (1 << 64) - 1
        v = [s["state"]["state"] >> 64, s["state"]["state"] & m, s["state"]["inc"] >> 64, s["state"]["inc"] & m,
             s.get("has_uint32", 0), s.get("uinteger", 0)]
        st = (ctypes.c_uint64 * 6)(*v)
        check(lib().gp_set_rng_state(self._handle, st), "gp_set_rng_state")
        self._seeded = True

    @property
    def np_random(self):
        """A numpy Generator positioned where the device stream is (snapshot; syncs)."""
        bg = np.random.PCG64()
        bg.state = self.rng_state
        return np.random.Generator(bg)

    @np_random.setter
    def np_random(self, gen):
        self.rng_state = gen.bit_generator.state

    # ------------------------------------------------------------------ hot path ----
    def _reset_impl(self, seed=None):
        if seed is not None:
            self._seed(seed)
        elif not self._seeded:
            self.seed(None)
        obs, _, _, _ = self._alloc_outputs()
        check(lib().gp_reset(self._handle, ctypes.c_void_p(obs.data_ptr()), self._stream()), "gp_reset")
        return self._post_obs(obs)

    def _step_impl(self, actions):
        a = self._as_actions(actions)
        obs, rew, term, trunc = self._alloc_outputs()
        check(lib().gp_step(self._handle, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(obs.data_ptr()),
                            ctypes.c_void_p(rew.data_ptr()), ctypes.c_void_p(term.data_ptr()),
                            ctypes.c_void_p(trunc.data_ptr()), self._stream()), "gp_step")
        return self._post_obs(obs), rew, term.view(_torch().bool), trunc.view(_torch().bool)

    def step(self, actions):
        obs, rew, term, trunc = self._step_impl(actions)
        return obs, rew, term, trunc, {}

    def rollout(self, actions, out=None):
        """K steps in one call: actions [K, B(,2)] -> obs [K, B, ...], rew/term/trunc [K, B].

        Philox mode, and numpy mode on the grid envs (persistent kernel with a per-step grid
        exchange), run the K steps in ONE fused launch with the env state in registers; C-ROOMS
        numpy mode runs a few multi-workgroup stream kernels per step (csrc/crooms.hip xg_*), Taxi
        numpy mode one single-workgroup launch for the K steps (the stream walk); replay mode issues
        K step launches on the stream. `out` may supply preallocated buffers
        (obs, rew, term(uint8), trunc(uint8)) shaped like `_alloc_outputs(K)`: they are checked
        for shape, dtype, device and contiguity (ValueError otherwise)."""
        torch = _torch()
        K = int(actions.shape[0])
        a = self._as_actions(actions, K)
        if out is None:
            out = self._alloc_outputs(K)
        else:
            self._check_out(out, K)
        obs, rew, term, trunc = out
        check(lib().gp_rollout(self._handle, K, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(obs.data_ptr()),
                               ctypes.c_void_p(rew.data_ptr()), ctypes.c_void_p(term.data_ptr()),
                               ctypes.c_void_p(trunc.data_ptr()), self._stream()), "gp_rollout")
        return self._post_obs(obs), rew, term.view(torch.bool), trunc.view(torch.bool)

    def _check_out(self, out, K):
        torch = _torch()
        if not isinstance(out, (tuple, list)) or len(out) != 4:
            raise ValueError("out must be (obs, rew, term, trunc)")
        want = (((K,) + self._obs_shape(), self._obs_dtype), ((K, self.num_envs), torch.float32),
                ((K, self.num_envs), torch.uint8), ((K, self.num_envs), torch.uint8))
        for name, t, (shape, dt) in zip(("obs", "rew", "term", "trunc"), out, want):
            if not isinstance(t, torch.Tensor):
                raise ValueError(f"out {name}: expected a torch tensor")
            if tuple(t.shape) != shape or t.dtype != dt or t.device != self.device or not t.is_contiguous():
                raise ValueError(f"out {name}: need a contiguous {dt} tensor of shape {shape} on {self.device}, got "
                                 f"{t.dtype} {tuple(t.shape)} on {t.device} (contiguous={t.is_contiguous()})")

    def rollout_plan(self, actions, out=None):
        """A prepared K-step rollout: validates `actions` [K, B(,2)] (already the env's action dtype, on its
        device, contiguous) and the output buffers once, and returns a callable that enqueues the K steps on
        the stream current at plan time (or the hipStream_t handle it is given) with no further Python work (the agent loop's allocation-free hot path; the
        buffers are reused by every call). Returns (run, (obs, rew, term, trunc))."""
        torch = _torch()
        K = int(actions.shape[0])
        a = self._as_actions(actions, K)
        if a.data_ptr() != actions.data_ptr():
            raise ValueError("rollout_plan: actions must already be a contiguous device tensor of the action dtype")
        if out is None:
            out = self._alloc_outputs(K)
        else:
            self._check_out(out, K)
        L, h = lib(), self._handle
        args = [ctypes.c_void_p(x.data_ptr()) for x in (a,) + tuple(out)]
        stream0 = torch.cuda.current_stream(self.device).cuda_stream
        fn = L.gp_rollout
        if hasattr(L, "gp_plan_create"):
            plan = ctypes.c_void_p()
            check(L.gp_plan_create(h, K, *args, stream0, ctypes.byref(plan)), "gp_plan_create")
            keep = _PlanKeep(plan, (a, out))
            fn_plan = L.gp_plan_run
        else:  # an older library chosen through GYM_PO_AMD_LIB (in-call A/B tooling)
            keep = _PlanKeep(None, (a, out))
            fn_plan = lambda _p: fn(h, K, *args, stream0)  # noqa: E731

        def run(stream=None):
            # the bound plan: one pointer across ctypes (another stream: the plain call with its arguments)
            rc = fn_plan(keep.plan) if stream is None else fn(h, K, *args, stream)
            if rc:
                check(rc, "gp_rollout")
            return keep.bufs
        return run, (out[0], out[1], out[2].view(torch.bool), out[3].view(torch.bool))

    def autotune(self, K=20, reps=5):
        """Pick, on this device, the faster of the handle's interchangeable kernels for launches of K steps
        (numpy-mode FourRooms/ROOMS: the windowed and the fused kernel, bit-identical results) by timing `reps`
        launches of each on scratch state; the env's own state, stream position and metrics are left exactly as
        they were. Returns 1 (windowed), 0 (fused) or -1 (nothing to choose). After reset(); syncs."""
        chosen = ctypes.c_int(-1)
        check(lib().gp_autotune(self._handle, int(K), int(reps), ctypes.byref(chosen)), "gp_autotune")
        return chosen.value

    def check(self):
        """Sync and raise GymPoError if a device-side failure hit any launch since the last seed (the
        asynchronous step/rollout calls cannot report it themselves; metrics() and rng_state check too)."""
        check(lib().gp_check(self._handle), "gp_check")

    def query(self, key):
        """Handle introspection (gp_query), e.g. 'fused_blocks', 'fused_staged'."""
        v = ctypes.c_int64()
        check(lib().gp_query(self._handle, key.encode(), ctypes.byref(v)), "gp_query")
        return v.value

    def step_raw(self, a, obs, rew, term, trunc, stream=None):
        """Allocation-free step into caller buffers (all device tensors; term/trunc uint8)."""
        st = self._stream() if stream is None else ctypes.c_void_p(stream)
        check(lib().gp_step(self._handle, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(obs.data_ptr()),
                            ctypes.c_void_p(rew.data_ptr()), ctypes.c_void_p(term.data_ptr()),
                            ctypes.c_void_p(trunc.data_ptr()), st), "gp_step")

    # ------------------------------------------------------------------ state / replay ----
    def _get_state_raw(self, bufs):
        ptrs = [ctypes.c_void_p(b.data_ptr()) if b is not None else None for b in bufs]
        ptrs += [None] * (4 - len(ptrs))
        check(lib().gp_get_state(self._handle, *ptrs, self._stream()), "gp_get_state")

    def _set_state_raw(self, bufs):
        ptrs = [ctypes.c_void_p(b.data_ptr()) if b is not None else None for b in bufs]
        ptrs += [None] * (4 - len(ptrs))
        check(lib().gp_set_state(self._handle, *ptrs, self._stream()), "gp_set_state")

    def set_replay(self, u=None, i0=None, i1=None, f0=None, f1=None):
        """Pre-decided per-env draws for the next step/reset (rng_mode='replay')."""
        keep = [x for x in (u, i0, i1, f0, f1) if x is not None]
        self._replay_keep = keep  # keep the tensors alive until the step is enqueued
        ptr = lambda x: ctypes.c_void_p(x.data_ptr()) if x is not None else None  # noqa: E731
        check(lib().gp_set_replay(self._handle, ptr(u), ptr(i0), ptr(i1), ptr(f0), ptr(f1)), "gp_set_replay")

    def valid_cells(self, which):
        buf = (ctypes.c_int32 * 65536)()
        n = lib().gp_valid_cells(self._handle, which, buf, 65536)
        return np.array(buf[:n], dtype=np.int64)

    def metrics(self):
        """{episodes, return_sum, length_sum, env_steps} accumulated on device since reset (syncs; raises
        GymPoError if a device-side failure invalidated the run, see check())."""
        out = (ctypes.c_double * 4)()
        check(lib().gp_metrics(self._handle, out), "gp_metrics")
        return dict(episodes=out[0], return_sum=out[1], length_sum=out[2], env_steps=out[3])

    def set_profiling(self, enable=True):
        check(lib().gp_set_profiling(self._handle, int(bool(enable))), "gp_set_profiling")

    def profile_read(self):
        """(summed step-kernel ms, launches) since the last read (syncs)."""
        ms, n = ctypes.c_double(), ctypes.c_int64()
        check(lib().gp_profile_read(self._handle, ctypes.byref(ms), ctypes.byref(n)), "gp_profile_read")
        return ms.value, n.value

    def profile_read_resolver(self):
        """(summed reset-resolver-kernel ms, launches) since the last read (syncs; numpy mode)."""
        ms, n = ctypes.c_double(), ctypes.c_int64()
        check(lib().gp_profile_read_resolver(self._handle, ctypes.byref(ms), ctypes.byref(n)),
              "gp_profile_read_resolver")
        return ms.value, n.value

    def render(self):
        """The reference renders none of the grid / continuous envs (msrooms.py:430-432 raises, RoomsEnv and
        CRoomsEnv inherit gymnasium's NotImplementedError); TaxiVecEnv overrides this."""
        raise NotImplementedError("render() is not implemented for this env (nor in the reference)")
