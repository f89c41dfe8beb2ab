"""GPU parity of the C-ROOMS backend (csrc/crooms.hip) against the reference fixtures and the oracle.

The device computes in float64 exactly as the reference. Replay mode is fed the values the
reference's own numpy stream produced (captured from the fixture-pinned oracle run on the same seed):
with float64 I/O every output must equal the reference bit-for-bit; with float32 I/O (BASELINE
configs[4]) the observation must be the float64 reference observation rounded once to float32, i.e.
|obs - ref| <= 2^-24 |ref| (<= 1e-6 for the coordinates of every layout) — tolerance written below.
Philox mode is checked in law and for rollout/step consistency: its normals (Box-Muller on a 53-bit u1,
csrc/crooms.hip box_muller_pair) are checked for their tail mass out to 6.5 sigma over 2^36 draws. numpy's
own normal algorithm (random_standard_normal, the 256-layer ziggurat), restated on the device, is checked
bit for bit against numpy over numpy's raw words.
"""
import numpy as np
import pytest

from fixtures import digest, load_case, load_index, step_actions
from oracle.crooms import CRoomsOracle
from oracle.draws import NumpyDraws

pytestmark = pytest.mark.gpu

CASES = {k: v for k, v in load_index()["cases"].items() if v["kind"] == "crooms"}
F32_REL_TOL = 2.0 ** -24  # one float32 rounding of the float64 observation


class RecordingDraws(NumpyDraws):
    """The reference's numpy calls (NumpyDraws) + per-env capture of every value for GPU replay."""

    def __init__(self, gen, B, valid):
        super().__init__(gen)
        self.B, self.valid, self.rec = B, valid, {}

    def uniform(self, n):
        u = super().uniform(n)
        self.rec["u"] = np.round(u * 2.0 ** 53).astype(np.uint64)  # random() = k * 2^-53 exactly
        return u

    def choice(self, values, mask, site):
        v = super().choice(values, mask, site)
        idx = np.zeros(self.B, np.int32)
        idx[mask] = np.searchsorted(self.valid, v)
        self.rec[site] = idx
        return v

    def record_normal(self, site, mask, v):
        arr = np.zeros((self.B, 2), np.float64)
        arr[mask] = v
        self.rec[site] = arr


def make_env(kw, B, **extra):
    from gym_po_amd import CRoomsEnv
    kw = dict(kw)
    if "goal_xy" in kw and kw["goal_xy"] is not None:
        kw["goal_xy"] = tuple(kw["goal_xy"])
    return CRoomsEnv(B, **kw, **extra)


def make_oracle(kw, B):
    kw = dict(kw)
    if "goal_xy" in kw and kw["goal_xy"] is not None:
        kw["goal_xy"] = tuple(kw["goal_xy"])
    return CRoomsOracle(B, **kw)


def _replay_args(rec, B):
    z2 = np.zeros((B, 2))
    return dict(u=rec.get("u", np.zeros(B, np.uint64)), goal_idx=rec.get("goal", np.zeros(B, np.int32)),
                agent_idx=rec.get("agent", np.zeros(B, np.int32)), noise=rec.get("noise", z2),
                wall_noise=rec.get("wall_noise", z2))


def run_replay(kw, B, seed, acts, dtype):
    """Oracle on the reference stream and GPU on its replayed values, step by step."""
    import torch
    ora = make_oracle(kw, B)
    env = make_env(kw, B, rng_mode="replay", dtype=dtype)
    ora.gen = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
    rd = RecordingDraws(ora.gen, B, ora.valid)
    o_ref = ora.reset(rd)
    env.set_replay(**_replay_args(rd.rec, B))
    o = env.reset()
    yield -1, np.asarray(o_ref), (o.cpu().numpy(),), ora, env
    for t in range(acts.shape[0]):
        rd = RecordingDraws(ora.gen, B, ora.valid)
        ro, rr, rdn, rt = ora.step(acts[t], rd)
        env.set_replay(**_replay_args(rd.rec, B))
        a = torch.as_tensor(acts[t]).to(dtype) if acts.dtype.kind == "f" else acts[t]
        o, r, d, tr, _ = env.step(a)
        yield t, (np.asarray(ro), rr, rdn, rt), (o.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy(),
                                                 tr.cpu().numpy()), ora, env


def _acts(meta):
    a = step_actions(meta)
    return a


@pytest.mark.parametrize("name", sorted(CASES))
def test_replay_f64_bit_exact_vs_reference_fixture(name, gpu_device):
    import torch
    meta, data = load_case(name)
    acts = _acts(meta)
    for t, ref, got, ora, env in run_replay(meta["kwargs"], meta["num_envs"], meta["seed"], acts, torch.float64):
        if t < 0:
            np.testing.assert_array_equal(got[0].astype(np.float64), data["obs0"].astype(np.float64))
            continue
        o, r, d, tr = got
        np.testing.assert_array_equal(o.astype(np.float64), data["obs"][t].astype(np.float64), err_msg=f"t={t}")
        np.testing.assert_array_equal(r, data["rew"][t], err_msg=f"t={t}")
        np.testing.assert_array_equal(d.astype(bool), data["term"][t], err_msg=f"t={t}")
        np.testing.assert_array_equal(tr.astype(bool), data["trunc"][t], err_msg=f"t={t}")
        od = o.astype(np.float64) if data["obs0"].dtype.kind == "f" else o.astype(np.int64)
        assert digest(od) == data["digests"][t][0], f"obs digest t={t}"
    a, g, v, e = (x.cpu().numpy() for x in env.get_state())
    np.testing.assert_array_equal(a, data["final_agent"])
    np.testing.assert_array_equal(g + 0.5, data["final_goal"])
    np.testing.assert_array_equal(v, data["final_velocity"])
    np.testing.assert_array_equal(e, data["final_elapsed"])


@pytest.mark.parametrize("kw,B", [({"obs_type": "vector_mdp"}, 100003),
                                  ({"obs_type": "vector_goal_mdp", "use_velocity": True, "goal_xy": None,
                                    "time_limit": 60}, 30001),
                                  ({"obs_type": "hansen8", "action_type": "ordinal", "layout": "16"}, 9999),
                                  ({"obs_type": "mdp", "action_type": "cardinal", "action_std": 0.0,
                                    "action_power": 2.0, "time_limit": 40}, 4097),
                                  ({"obs_type": "goal_room", "layout": "8b", "goal_xy": None}, 2049)])
def test_replay_f32_io_vs_oracle_ragged(kw, B, gpu_device):
    """float32 actions in, float32 obs out: state math is float64, obs = f32(reference obs)."""
    import torch
    rng = np.random.default_rng(5)
    yx = kw.get("action_type", "yx") == "yx"
    if yx:
        acts = rng.uniform(-1, 1, (120, B, 2)).astype(np.float32).astype(np.float64)
    else:
        acts = rng.integers(0, 8 if kw.get("action_type") == "ordinal" else 4, (120, B))
    eps = 0
    for t, ref, got, ora, env in run_replay(kw, B, 17, acts, torch.float32):
        if t < 0:
            continue
        o = got[0]
        if o.dtype.kind == "f":
            assert o.dtype == np.float32
            r64 = ref[0].astype(np.float64)
            np.testing.assert_array_equal(o, ref[0].astype(np.float32), err_msg=f"t={t}")
            assert np.all(np.abs(o.astype(np.float64) - r64) <= F32_REL_TOL * np.abs(r64))
        else:
            np.testing.assert_array_equal(o.astype(np.int64), ref[0].astype(np.int64), err_msg=f"t={t}")
        for name, a, b in zip(("rew", "term", "trunc"), ref[1:], got[1:]):
            np.testing.assert_array_equal(np.asarray(a).astype(np.float64), b.astype(np.float64),
                                          err_msg=f"{name} t={t}")
        eps += int((ref[2] | ref[3]).sum())
    m = env.metrics()
    assert m["episodes"] == eps and m["env_steps"] == 120 * B


def test_philox_rollout_equals_single_steps(gpu_device):
    import torch
    B, K = 7001, 33
    kw = {"obs_type": "vector_goal_mdp", "use_velocity": True, "goal_xy": None, "time_limit": 20}
    a, b = make_env(kw, B), make_env(kw, B)
    a.reset(seed=3)
    b.reset(seed=3)
    acts = torch.rand((K, B, 2), device=gpu_device) * 2 - 1
    ro, rr, rd, rt = a.rollout(acts)
    for t in range(K):
        o, r, d, tr, _ = b.step(acts[t])
        assert torch.equal(o, ro[t]) and torch.equal(r, rr[t]) and torch.equal(d, rd[t]) and torch.equal(tr, rt[t])
    for x, y in zip(a.get_state(), b.get_state()):
        assert torch.equal(x, y)


@pytest.mark.parametrize("B,K", [(1 << 21, 16), (100003, 9)])
def test_philox_specialised_kernel_equals_generic(B, K, gpu_device):
    """configs[4]'s shape (continuous float32 actions, vector_mdp, fixed goal, no velocity) runs a compile-time
    specialised philox rollout (crooms_rollout<GP_OBS_F32, false, 1>); the generic kernel (forced by the
    `generic_kernels` debug knob) must produce the same outputs and state bit for bit, at the config size and on
    a ragged size."""
    import torch
    from gym_po_amd._lib import debug_knobs
    kw = {"obs_type": "vector_mdp"}
    a = make_env(kw, B)
    with debug_knobs(generic_kernels=1):
        b = make_env(kw, B)
    a.reset(seed=21)
    b.reset(seed=21)
    acts = torch.rand((K, B, 2), device=gpu_device) * 2 - 1
    for x, y in zip(a.rollout(acts), b.rollout(acts)):
        assert torch.equal(x, y)
    for x, y in zip(a.get_state(), b.get_state()):
        assert torch.equal(x, y)
    ma, mb = a.metrics(), b.metrics()
    assert {k: v for k, v in ma.items() if k != "return_sum"} == {k: v for k, v in mb.items() if k != "return_sum"}
    assert ma["return_sum"] == pytest.approx(mb["return_sum"], rel=1e-6)


def test_philox_action_noise_law(gpu_device):
    """Zero actions from cell centres far from walls: the displacement is the action noise N(0, 0.2)."""
    import torch
    from scipy.stats import kstest
    B = 1 << 20
    env = make_env({"obs_type": "vector_mdp", "layout": "1", "time_limit": 10}, B, dtype=torch.float64)
    env.reset(seed=8)
    H, W = env.grid.shape
    cy, cx = H // 2 + 0.5, W // 2 + 0.5
    start = np.tile([cy, cx], (B, 1))
    env.set_state(agent_yx=start, elapsed=np.zeros(B, np.int32))
    o, r, d, tr, _ = env.step(torch.zeros((B, 2), dtype=torch.float64, device=gpu_device))
    disp = (env.agent_yx.cpu().numpy() - start).ravel()
    assert abs(disp.mean()) < 3e-3 and abs(disp.std() - 0.2) < 2e-3
    assert kstest(disp / 0.2, "norm").pvalue > 1e-4


def test_philox_reset_cells_uniform(gpu_device):
    import torch
    from scipy.stats import chisquare
    B = 1 << 20
    env = make_env({"obs_type": "vector_goal_mdp", "goal_xy": None}, B, dtype=torch.float64)
    env.reset(seed=1)
    a, g, _, _ = env.get_state()
    H, W = env.grid.shape
    ac = np.floor(a.cpu().numpy()).astype(int)
    cells = ac[:, 0] * W + ac[:, 1]
    idx = np.searchsorted(env.valid_states, cells)
    assert np.array_equal(env.valid_states[idx], cells)
    counts = np.bincount(idx, minlength=len(env.valid_states))
    assert chisquare(counts).pvalue > 1e-4
    gc = g.cpu().numpy()
    gidx = np.searchsorted(env.valid_states, gc[:, 0] * W + gc[:, 1])
    assert chisquare(np.bincount(gidx, minlength=len(env.valid_states))).pvalue > 1e-4


def _device_normals(words, n, gpu_device):
    import ctypes
    import torch
    from gym_po_amd import _lib as L
    dw = torch.from_numpy(words.view(np.int64)).to(gpu_device)
    out = torch.empty(n, dtype=torch.float64, device=gpu_device)
    used = ctypes.c_int64()
    L.check(L.lib().gp_standard_normal_words(ctypes.c_void_p(dw.data_ptr()), len(words),
                                             ctypes.c_void_p(out.data_ptr()), n, ctypes.byref(used),
                                             ctypes.c_void_p(torch.cuda.current_stream(gpu_device).cuda_stream)),
            "gp_standard_normal_words")
    return out.cpu().numpy(), used.value


def test_device_ziggurat_matches_numpy_words(gpu_device):
    """gp_standard_normal_words over numpy's raw PCG64 words returns numpy's standard_normal bit for bit, the
    layer-0 tail included (its log1p is glibc's restated, tests/test_log1p_cpu.py), and consumes the words
    numpy consumed."""
    from oracle.ziggurat import R, standard_normals
    n, seed = 200000, 4242
    want = np.random.Generator(np.random.PCG64(seed)).standard_normal(n)
    words = np.random.PCG64(seed).random_raw(2 * n)
    _, used_want = standard_normals(words, n)
    got, used = _device_normals(words, n, gpu_device)
    assert used == used_want
    assert (np.abs(want) > R).sum() > 10
    np.testing.assert_array_equal(got.view(np.uint64), want.view(np.uint64))


def test_device_ziggurat_tail_heavy_stream_exact(gpu_device):
    """A word stream that sends every normal to layer 0 (low byte of every word zeroed): about half of them take
    the tail (r + x, x = -log1p(-u1) / r, with rejection pairs), i.e. ~2.6e4 tail values and their accept tests
    through log1p over uniform u. Device == the oracle (math.log1p = the C library's, as numpy) bit for bit, and
    the same word count consumed (a 1-ulp log1p would flip last bits and, at a tie, the word count)."""
    from oracle.ziggurat import R, standard_normals
    n = 400000
    words = np.random.PCG64(99).random_raw(4 * n) & np.uint64(0xFFFFFFFFFFFFFF00)
    want, used_want = standard_normals(words, n)
    want = np.asarray(want, np.float64)
    got, used = _device_normals(words, n, gpu_device)
    assert used == used_want
    assert (np.abs(want) > R).sum() > 20000
    np.testing.assert_array_equal(got.view(np.uint64), want.view(np.uint64))


def test_device_ziggurat_wedge_heavy_stream_exact(gpu_device):
    """A word stream that sends most normals to the wedge test (the top 7 bits of the 52-bit magnitude set, so
    rabs >= ki[idx] on nearly every layer): ~2e5 accept tests (fi[i-1] - fi[i]) u + fi[i] < exp(-x^2 / 2) over
    random x in each layer's wedge. The device's exp is glibc's restated (csrc/gp_libm.h); device == the oracle
    (math.exp = the C library's, as numpy) bit for bit and the same word count."""
    from oracle.ziggurat import standard_normals
    n = 300000
    words = np.random.PCG64(123).random_raw(4 * n)
    words[::2] |= np.uint64(0x7F) << np.uint64(54)  # bits 54..60: the top 7 of rabs = word bits 9..60
    want, used_want = standard_normals(words, n)
    want = np.asarray(want, np.float64)
    got, used = _device_normals(words, n, gpu_device)
    assert used == used_want
    assert used_want > 1.3 * n  # the wedge test drew a second word for a large share of the normals
    np.testing.assert_array_equal(got.view(np.uint64), want.view(np.uint64))


def test_device_ziggurat_words_run_out_mid_normal(gpu_device):
    """A normal whose wedge / tail draws run past the caller's words is NaN, not a value built from
    zero words; with every word it needs it is numpy's value."""
    from oracle.ziggurat import standard_normals
    words = np.random.PCG64(5).random_raw(256) & np.uint64(0xFFFFFFFFFFFFFF00)  # layer 0: many multi-word
    used = [standard_normals(words, k)[1] for k in range(40)]
    j = next(k for k in range(39) if used[k + 1] - used[k] > 1)  # normal j takes more than one word
    want = np.asarray(standard_normals(words, j + 1)[0], np.float64)
    got, _ = _device_normals(words[:used[j + 1] - 1].copy(), j + 2, gpu_device)
    np.testing.assert_array_equal(got[:j].view(np.uint64), want[:j].view(np.uint64))
    assert np.isnan(got[j:]).all()
    got, u = _device_normals(words[:used[j + 1]].copy(), j + 1, gpu_device)
    assert u == used[j + 1]
    np.testing.assert_array_equal(got.view(np.uint64), want.view(np.uint64))


def test_philox_normal_tail_mass(gpu_device):
    """The philox-mode sampler has the normal law's tails: exceedance counts of |z| beyond 3..6.5 sigma over
    2^36 draws within 6 Poisson standard deviations of n * erfc(t / sqrt 2) (the former float32 Box-Muller
    could not exceed 5.77 sigma), and the first two moments within 6 standard errors."""
    import ctypes
    import math
    import torch
    from gym_po_amd import _lib as L
    from oracle.philox import philox_key
    n = 1 << 36
    thr = [3.0, 4.0, 5.0, 6.0, 6.5]
    k0, k1 = philox_key(11)
    counts = (ctypes.c_uint64 * len(thr))()
    mom = (ctypes.c_double * 2)()
    torch.cuda.synchronize(gpu_device)
    L.check(L.lib().gp_normal_tail_counts((k1 << 32) | k0, n, (ctypes.c_double * len(thr))(*thr), len(thr), counts,
                                          mom, ctypes.c_void_p(torch.cuda.current_stream(gpu_device).cuda_stream)),
            "gp_normal_tail_counts")
    for t, c in zip(thr, counts):
        lam = n * math.erfc(t / math.sqrt(2.0))
        assert abs(c - lam) <= 6 * math.sqrt(lam) + 1, (t, c, lam)
    assert counts[3] > 0  # beyond 6 sigma (expected ~136)
    mean, var = mom[0] / n, mom[1] / n
    assert abs(mean) < 6 / math.sqrt(n) and abs(var - 1.0) < 6 * math.sqrt(2.0 / n)
