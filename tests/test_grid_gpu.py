"""GPU parity of the GRID kernels (FourRooms / ROOMS) against the reference fixtures and the oracle.

numpy mode must be bit-exact with the reference on identical seeds: every step's obs / reward /
terminated / truncated, the final env state and the final PCG64 state. Large-batch runs are
checked against the oracle step by step; the Lemire-rejection slow path is forced by planting
rejected words in the PCG64 stream.
"""
import numpy as np
import pytest

from fixtures import digest, load_case, load_index, step_actions
from oracle import gridworld
from oracle.pcg64 import MASK128, PCG64, lemire_threshold, pcg_advance_params, pcg_output

pytestmark = pytest.mark.gpu

CASES = {k: v for k, v in load_index()["cases"].items() if v["kind"] in ("fourrooms", "rooms")}


def make_env(meta, num_envs=None, **extra):
    from gym_po_amd import MultistoryFourRoomsEnv, RoomsEnv
    kw = dict(meta["kwargs"])
    B = num_envs or meta["num_envs"]
    if meta["kind"] == "fourrooms":
        if kw.get("goal_xyz") is not None:
            kw["goal_xyz"] = tuple(kw["goal_xyz"])
        return MultistoryFourRoomsEnv(B, **kw, **extra)
    return RoomsEnv(B, **kw, **extra)


def make_oracle(meta, num_envs=None):
    kw = dict(meta["kwargs"])
    B = num_envs or meta["num_envs"]
    if meta["kind"] == "fourrooms":
        if kw.get("goal_xyz") is not None:
            kw["goal_xyz"] = tuple(kw["goal_xyz"])
        return gridworld.FourRoomsOracle(B, **kw)
    return gridworld.RoomsOracle(B, **kw)


def reset_obs(env, seed):
    r = env.reset(seed=seed)
    return r[0] if isinstance(r, tuple) else r


def np_obs(o):
    return o.cpu().numpy()


def obs_digest(o, float_ref):
    return digest(o.astype(np.float64) if float_ref else o)


def rng_tuple(st):
    s, inc = st["state"]["state"], st["state"]["inc"]
    m = (1 << 64) - 1
    return [s >> 64, s & m, inc >> 64, inc & m, st["has_uint32"], st["uinteger"]]


@pytest.mark.parametrize("name", sorted(CASES))
def test_numpy_mode_bit_exact_vs_reference_fixture(name, gpu_device):
    meta, data = load_case(name)
    env = make_env(meta)
    acts = step_actions(meta)
    float_ref = data["obs0"].dtype.kind == "f"
    o0 = np_obs(reset_obs(env, meta["seed"]))
    np.testing.assert_array_equal(o0.astype(np.float64), data["obs0"].astype(np.float64))
    for t in range(meta["steps"]):
        o, r, d, tr, info = env.step(acts[t])
        o, r, d, tr = np_obs(o), r.cpu().numpy(), d.cpu().numpy(), tr.cpu().numpy()
        if meta["full"]:
            np.testing.assert_array_equal(o.astype(np.float64), data["obs"][t].astype(np.float64), err_msg=f"t={t}")
            np.testing.assert_array_equal(r, data["rew"][t], err_msg=f"t={t}")
            np.testing.assert_array_equal(d, data["term"][t], err_msg=f"t={t}")
            np.testing.assert_array_equal(tr, data["trunc"][t], err_msg=f"t={t}")
        dg = [obs_digest(o, float_ref), digest(r), digest(d), digest(tr)]
        assert dg == list(data["digests"][t]), f"digest mismatch at step {t}"
    a, g, e = (x.cpu().numpy() for x in env.get_state())
    shape = env.grid.shape
    np.testing.assert_array_equal(np.ravel_multi_index(tuple(data["final_agent"].T), shape), a)
    np.testing.assert_array_equal(data["final_elapsed"], e)
    fg = data["final_goal"]
    if np.all(fg[:, -2] < shape[-2]):
        np.testing.assert_array_equal(np.ravel_multi_index(tuple(fg.T), shape), g)
    assert rng_tuple(env.rng_state) == [int(x) for x in data["final_rng_state"]]


def _run_vs_oracle(meta, B, steps, seed, action_seed):
    env = make_env(meta, B)
    ora = make_oracle(meta, B)
    rng = np.random.default_rng(action_seed)
    o_g = np_obs(reset_obs(env, seed))
    o_o = np.asarray(ora.reset_seed(seed))
    np.testing.assert_array_equal(o_g.astype(np.float64), o_o.astype(np.float64))
    n_act = env.single_action_space.n
    for t in range(steps):
        a = rng.integers(0, n_act, B)
        o, r, d, tr, _ = env.step(a)
        oo, ro, do, tro = ora.step_seeded(a)
        np.testing.assert_array_equal(np_obs(o).astype(np.float64), np.asarray(oo).astype(np.float64),
                                      err_msg=f"t={t}")
        np.testing.assert_array_equal(r.cpu().numpy(), ro)
        np.testing.assert_array_equal(d.cpu().numpy(), do)
        np.testing.assert_array_equal(tr.cpu().numpy(), tro)
    assert rng_tuple(env.rng_state) == rng_tuple(ora.gen.bit_generator.state)
    return env, ora


def test_fourrooms_1m_envs_bit_exact_vs_oracle(gpu_device):
    """BASELINE config 2 shape (2^20 envs, FR_MAP Hansen-4), 12 steps vs the numpy oracle."""
    meta, _ = load_case("fr_hansen_b256")
    _run_vs_oracle(meta, 1 << 20, 12, seed=2024, action_seed=5)


@pytest.mark.parametrize("B", [1, 3, 1023, 1025, 4099])
def test_ragged_batch_sizes(B, gpu_device):
    meta, _ = load_case("fr_hansen_tl20")
    _run_vs_oracle(meta, B, 60, seed=B, action_seed=B + 1)


@pytest.mark.parametrize("name,B,T", [("rooms_2_goal_mdp_randgoal", 2048 * 40, 40), ("rooms_4_hansen8", 2048 * 40, 40),
                                       ("fr_goal_mdp_z2_randgoal", 2048 * 64, 30),
                                       ("rooms_2_goal_mdp_randgoal", 1 << 20, 6)])
def test_staged_fused_kernel_variants(name, B, T, gpu_device):
    """Batch sizes of whole 2048-env tiles per block take the LDS-staged fused kernel (store waves, resetter
    obs written by the control wave): random goals (two reset calls, coverage rounds), table obs, Hansen-8."""
    meta, _ = load_case(name)
    _run_vs_oracle(meta, B, T, seed=B % 97, action_seed=7)


def test_rooms_random_goal_two_pass_large(gpu_device):
    meta, _ = load_case("rooms_2_goal_mdp_randgoal")
    _run_vs_oracle(meta, 50_000, 70, seed=3, action_seed=4)


# ---------------------------------------------------------------- forced Lemire rejections ----
def _rotl(x, r):
    return ((x << r) | (x >> ((64 - r) & 63))) & ((1 << 64) - 1)


def _state_with_output_half(half_value, half, hi_seed):
    """A PCG64 state whose output has the given low (half=0) or high (half=1) 32 bits."""
    rng = np.random.default_rng(hi_seed)
    hi = int(rng.integers(0, 2 ** 63)) * 2 + 1
    other = int(rng.integers(0, 2 ** 32))
    x = (other << 32) | half_value if half == 0 else (half_value << 32) | other
    rot = hi >> 58
    lo = hi ^ _rotl(x, rot)
    s = (hi << 64) | lo
    assert pcg_output(s) == x
    return s


def _rejected_word(n, k=1):
    thr = lemire_threshold(n)
    for kk in range(k, k + 10000):
        r = -(-(kk << 32) // n)
        if r < (1 << 32) and (r * n) & 0xFFFFFFFF < thr:
            return r
    raise AssertionError


def _plant(inc, B, words, n):
    """Start state s0 (has_uint32=0) such that each word position in `words` (counted after
    random(B)) is a rejected Lemire draw for range n."""
    # plant the first word by construction, the others by searching is impractical; use one
    w = words[0]
    q, half = w >> 1, w & 1
    s_star = _state_with_output_half(_rejected_word(n), half, w)
    a, c = pcg_advance_params((1 << 128) - (B + q + 1), inc)
    return (a * s_star + c) & MASK128


@pytest.mark.parametrize("word", [0, 1, 777, 4094])
def test_forced_rejection_slow_path_step(word, gpu_device):
    meta, _ = load_case("fr_hansen_tl20")  # time_limit 20
    B = 4096
    env = make_env(meta, B)
    ora = make_oracle(meta, B)
    reset_obs(env, 11)
    ora.reset_seed(11)
    # every env truncates on the next step -> b = B resets, words 0..B-1 (+rejections) consumed
    import torch
    a, g, e = env.get_state()
    env.set_state(elapsed=torch.full_like(e, 20))
    ora.elapsed[:] = 20
    inc = ora.gen.bit_generator.state["state"]["inc"]
    s0 = _plant(inc, B, [word], len(ora.valid_agent))
    st = {"bit_generator": "PCG64", "state": {"state": s0, "inc": inc}, "has_uint32": 0, "uinteger": 0}
    env.rng_state = st
    ora.gen.bit_generator.state = st
    acts = np.random.default_rng(0).integers(0, 4, B)
    o, r, d, tr, _ = env.step(acts)
    oo, ro, do, tro = ora.step_seeded(acts)
    np.testing.assert_array_equal(np_obs(o).astype(np.float64), np.asarray(oo).astype(np.float64))
    np.testing.assert_array_equal(tr.cpu().numpy(), tro)
    assert rng_tuple(env.rng_state) == rng_tuple(ora.gen.bit_generator.state)
    # and the streams stay in lockstep afterwards
    for t in range(5):
        acts = np.random.default_rng(t + 1).integers(0, 4, B)
        o, r, d, tr, _ = env.step(acts)
        oo, *_ = ora.step_seeded(acts)
        np.testing.assert_array_equal(np_obs(o).astype(np.float64), np.asarray(oo).astype(np.float64))


def test_forced_rejection_in_reset(gpu_device):
    meta, _ = load_case("fr_hansen_b256")
    B = 5000
    env = make_env(meta, B)
    ora = make_oracle(meta, B)
    reset_obs(env, 1)
    ora.reset_seed(1)
    inc = ora.gen.bit_generator.state["state"]["inc"]
    s0 = _plant(inc, 0, [1234], len(ora.valid_agent))  # reset: no random(B) before the words
    st = {"bit_generator": "PCG64", "state": {"state": s0, "inc": inc}, "has_uint32": 0, "uinteger": 0}
    env.rng_state = st
    ora.gen = np.random.Generator(np.random.PCG64())
    ora.gen.bit_generator.state = st
    from oracle.draws import NumpyDraws
    o = np_obs(env.reset()[0])
    oo = np.asarray(ora.reset(NumpyDraws(ora.gen)))
    np.testing.assert_array_equal(o.astype(np.float64), oo.astype(np.float64))
    assert rng_tuple(env.rng_state) == rng_tuple(ora.gen.bit_generator.state)


def test_buffered_half_word_carried_across_steps(gpu_device):
    """A step that consumes an odd number of words leaves numpy's uint32 buffer full."""
    meta, _ = load_case("fr_hansen_tl20")
    env, ora = _run_vs_oracle(meta, 333, 45, seed=99, action_seed=98)
    st = env.rng_state
    assert st == ora.gen.bit_generator.state


# ---------------------------------------------------------------- counter modes ----
def test_replay_mode_matches_oracle_with_same_draws(gpu_device):
    import torch
    from oracle.draws import ReplayDraws
    meta, _ = load_case("fr_vgh_z3_randgoal")
    B = 2048
    env = make_env(meta, B, rng_mode="replay")
    ora = make_oracle(meta, B)
    rng = np.random.default_rng(7)
    ng, na = len(ora.valid_goal), len(ora.valid_agent)
    gi, ai = rng.integers(0, ng, B), rng.integers(0, na, B)
    dev = gpu_device
    env.set_replay(i0=torch.as_tensor(gi, dtype=torch.int32, device=dev),
                   i1=torch.as_tensor(ai, dtype=torch.int32, device=dev))
    o = np_obs(env.reset()[0])
    oo = np.asarray(ora.reset(ReplayDraws({"goal": gi, "agent": ai})))
    np.testing.assert_array_equal(o.astype(np.float64), oo.astype(np.float64))
    for t in range(150):
        k = rng.integers(0, 2 ** 53, B, dtype=np.uint64)
        gi, ai = rng.integers(0, ng, B), rng.integers(0, na, B)
        a = rng.integers(0, env.single_action_space.n, B)
        env.set_replay(u=torch.as_tensor(k.view(np.int64), device=dev),
                       i0=torch.as_tensor(gi, dtype=torch.int32, device=dev),
                       i1=torch.as_tensor(ai, dtype=torch.int32, device=dev))
        o, r, d, tr, _ = env.step(a)
        oo, ro, do, tro = ora.step(a, ReplayDraws({"uniform": k.astype(np.float64) * 2.0 ** -53, "goal": gi,
                                                   "agent": ai}))
        np.testing.assert_array_equal(np_obs(o).astype(np.float64), np.asarray(oo).astype(np.float64),
                                      err_msg=f"t={t}")
        np.testing.assert_array_equal(r.cpu().numpy(), ro)
        np.testing.assert_array_equal(d.cpu().numpy(), do)
        np.testing.assert_array_equal(tr.cpu().numpy(), tro)


def test_philox_rollout_equals_stepwise_and_is_sane(gpu_device):
    import torch
    meta, _ = load_case("fr_hansen_b256")
    B, K = 10_000, 64
    e1 = make_env(meta, B, rng_mode="philox")
    e2 = make_env(meta, B, rng_mode="philox")
    e1.reset(seed=5)
    e2.reset(seed=5)
    acts = torch.randint(0, 4, (K, B), device=gpu_device, dtype=torch.int32)
    o1, r1, d1, t1 = e1.rollout(acts)
    for k in range(K):
        o2, r2, d2, t2, _ = e2.step(acts[k])
        assert torch.equal(o1[k], o2) and torch.equal(r1[k], r2) and torch.equal(d1[k], d2)
    # obs always a valid Hansen index; reward only at the goal
    assert int(o1.min()) >= 0 and int(o1.max()) < e1.single_observation_space.n
    assert torch.all((r1 == 0) | (r1 == 1))
    m = e1.metrics()
    assert m["env_steps"] == B * K


def test_numpy_rollout_equals_stepwise(gpu_device):
    import torch
    meta, _ = load_case("rooms_4_hansen_card")
    B, K = 3000, 40
    e1 = make_env(meta, B)
    e2 = make_env(meta, B)
    e1.reset(seed=8)
    e2.reset(seed=8)
    acts = torch.randint(0, 4, (K, B), device=gpu_device, dtype=torch.int32)
    o1, r1, d1, t1 = e1.rollout(acts)
    for k in range(K):
        o2, r2, d2, t2, _ = e2.step(acts[k])
        assert torch.equal(o1[k], o2) and torch.equal(r1[k], r2) and torch.equal(t1[k], t2)
    assert e1.rng_state == e2.rng_state


@pytest.mark.parametrize("name", ["fr_hansen_tl20", "fr_vgh_z3_randgoal", "rooms_2_goal_mdp_randgoal",
                                  "rooms_4_grid3"])
def test_two_kernel_numpy_path_bit_exact(name, gpu_device):
    """The non-fused numpy path (streaming step kernel + reset resolver), used above 4M envs."""
    from gym_po_amd._lib import debug_knobs
    meta, data = load_case(name)
    with debug_knobs(disable_fused=1):
        env = make_env(meta)
    assert env.query("fused_blocks") == 0
    acts = step_actions(meta)
    np.testing.assert_array_equal(np_obs(reset_obs(env, meta["seed"])).astype(np.float64),
                                  data["obs0"].astype(np.float64))
    for t in range(meta["steps"]):
        o, r, d, tr, _ = env.step(acts[t])
        np.testing.assert_array_equal(np_obs(o).astype(np.float64), data["obs"][t].astype(np.float64),
                                      err_msg=f"t={t}")
        np.testing.assert_array_equal(tr.cpu().numpy(), data["trunc"][t])
    assert rng_tuple(env.rng_state) == [int(x) for x in data["final_rng_state"]]


def test_two_kernel_forced_rejection(gpu_device):
    from gym_po_amd._lib import debug_knobs
    with debug_knobs(disable_fused=1):
        test_forced_rejection_slow_path_step(777, gpu_device)


@pytest.mark.parametrize("B", [4096 * 256 + 5, 2_500_000])
def test_fused_multi_tile_per_block(B, gpu_device):
    """QPT > 1 (several 4096-env tiles per persistent block) vs the oracle, few steps."""
    meta, _ = load_case("fr_hansen_tl20")
    _run_vs_oracle(meta, B, 4, seed=17, action_seed=18)


@pytest.mark.parametrize("name", ["fr_hansen_b256", "fr_mdp_z2", "rooms_10b_hansen", "fr_vector_hansen8_z2"])
def test_obs_dtype_reference_matches_fixture_dtype_and_values(name, gpu_device):
    """obs_dtype="reference": the reference's own obs arrays (float64 for the scalar Hansen obs, whose goal multiplier
    is a float array (msrooms.py:180-189, observations.py:62-71); int64 otherwise), dtype and values, against the
    reference fixtures (no cast in the comparison). The default stays the compact native layout (int32 / uint8)."""
    meta, data = load_case(name)
    env = make_env(meta, obs_dtype="reference")
    native = make_env(meta)
    o0 = np_obs(reset_obs(env, meta["seed"]))
    assert np_obs(reset_obs(native, meta["seed"])).dtype in (np.int32, np.uint8)
    assert o0.dtype == data["obs0"].dtype
    np.testing.assert_array_equal(o0, data["obs0"])
    acts = step_actions(meta)
    for t in range(min(meta["steps"], 40)):
        o = np_obs(env.step(acts[t])[0])
        assert o.dtype == data["obs0"].dtype
        assert digest(o) == data["digests"][t][0], f"t={t}"
