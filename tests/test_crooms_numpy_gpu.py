"""GPU parity of C-ROOMS exact mode (rng_mode="numpy", csrc/crooms.hip: crooms_numpy_rollout for B <= 1024
(XG_MIN_ENVS, the measured crossover), the multi-workgroup xg_* draw-call kernels above; both paths are also
forced on the other side of the crossover).

The device draws the reference's own PCG64 stream word for word — rng.random / rng.normal (numpy's
256-layer ziggurat, a data-dependent number of words per normal) / rng.choice (buffered 32-bit Lemire) in
the reference's call order (crooms.py:175-198, :300-331, :217-244, :276-298) — so with the same seed the
trajectory must equal the reference's bit for bit:
  * against the reference's own fixtures (float64 I/O): obs, rewards, flags, final state;
  * against the fixture-pinned oracle (oracle/crooms.py driven by numpy's Generator) at every step for
    configurations that exercise the slow ziggurat paths (wedge / tail), wall resamples, odd reset counts
    (a buffered uint32 half carried across calls), discrete actions (rng.random) and K-step launches;
    the final PCG64 state (incl. has_uint32 / uinteger) must equal numpy's.
Tolerance: none (bit-exact), except the float32-I/O case, where obs = float32(reference obs) exactly.
"""
import numpy as np
import pytest

from fixtures import load_case, load_index, step_actions
from oracle.crooms import CRoomsOracle

pytestmark = pytest.mark.gpu

CASES = {k: v for k, v in load_index()["cases"].items() if v["kind"] == "crooms"}


def _kw(kw):
    kw = dict(kw)
    if kw.get("goal_xy") is not None:
        kw["goal_xy"] = tuple(kw["goal_xy"])
    return kw


def _np_state(gen):
    st = gen.bit_generator.state
    return (st["state"]["state"], st["state"]["inc"], st["has_uint32"], st["uinteger"])


def _dev_state(env):
    st = env.rng_state
    return (st["state"]["state"], st["state"]["inc"], st["has_uint32"], st["uinteger"])


@pytest.mark.parametrize("name", sorted(CASES))
def test_numpy_mode_bit_exact_vs_reference_fixture(name, gpu_device):
    import torch
    from gym_po_amd import CRoomsEnv
    meta, data = load_case(name)
    B = meta["num_envs"]
    env = CRoomsEnv(B, **_kw(meta["kwargs"]), rng_mode="numpy", dtype=torch.float64)
    o = env.reset(seed=meta["seed"]).cpu().numpy()
    np.testing.assert_array_equal(o.astype(np.float64), data["obs0"].astype(np.float64))
    acts = step_actions(meta)
    for t in range(acts.shape[0]):
        a = torch.as_tensor(acts[t]).to(torch.float64) if acts.dtype.kind == "f" else acts[t]
        o, r, d, tr, _ = env.step(a)
        np.testing.assert_array_equal(o.cpu().numpy().astype(np.float64), data["obs"][t].astype(np.float64),
                                      err_msg=f"obs t={t}")
        np.testing.assert_array_equal(r.cpu().numpy(), data["rew"][t], err_msg=f"rew t={t}")
        np.testing.assert_array_equal(d.cpu().numpy().astype(bool), data["term"][t], err_msg=f"term t={t}")
        np.testing.assert_array_equal(tr.cpu().numpy().astype(bool), data["trunc"][t], err_msg=f"trunc t={t}")
    a, g, v, e = (x.cpu().numpy() for x in env.get_state())
    np.testing.assert_array_equal(a, data["final_agent"])
    np.testing.assert_array_equal(g + 0.5, data["final_goal"])
    np.testing.assert_array_equal(v, data["final_velocity"])
    np.testing.assert_array_equal(e, data["final_elapsed"])
    # the stream position: the oracle (pinned to the same fixture) replayed on numpy's Generator
    ora = CRoomsOracle(B, **_kw(meta["kwargs"]))
    ora.reset_seed(meta["seed"])
    for t in range(acts.shape[0]):
        ora.step_seeded(acts[t])
    assert _dev_state(env) == _np_state(ora.gen)


ORACLE_CASES = [
    # (kwargs, B, steps, K per launch)
    ({"obs_type": "vector_goal_mdp", "goal_xy": None, "use_velocity": True, "time_limit": 25}, 3001, 60, 1),
    ({"obs_type": "mdp", "layout": "4", "action_std": 0.6, "action_power": 1.5, "time_limit": 30}, 2047, 50, 7),
    ({"obs_type": "hansen8", "action_type": "ordinal", "layout": "16", "goal_xy": None, "time_limit": 20}, 1500, 45, 1),
    ({"obs_type": "grid", "action_type": "cardinal", "action_std": 0.0, "time_limit": 15}, 999, 40, 40),
    ({"obs_type": "goal_room", "layout": "8b", "goal_xy": None, "time_limit": 12}, 4099, 30, 5),
    # larger: the multi-workgroup path (grid-wide draw calls, cluster-resolved ziggurat chains) at scale
    ({"obs_type": "vector_mdp", "action_std": 0.5, "time_limit": 6}, 65536, 12, 6),
    ({"obs_type": "vector_goal_mdp", "goal_xy": None, "use_velocity": True, "time_limit": 25}, 30001, 30, 3),
    ({"obs_type": "hansen8", "action_type": "ordinal", "layout": "16", "goal_xy": None, "time_limit": 20}, 20000, 25, 5),
    ({"obs_type": "grid", "action_type": "cardinal", "action_std": 0.0, "time_limit": 9}, 8193, 20, 20),
    # 1,026 env blocks: the env kernels' 4-block workgroups with a partial last one; time-limit resets
    ({"obs_type": "vector_mdp", "action_std": 0.5, "time_limit": 4}, 262444, 10, 5),
    # BASELINE configs[4]'s size: 2^21 envs (4M normals per step, ~1e3 tail normals, wall resamples)
    ({"obs_type": "vector_mdp"}, 1 << 21, 4, 2),
]


# the two-launch draw calls (the form above XG_FUSE_MAX_ENVS = 2^21 envs), forced at a size the oracle runs fast
SPLIT_CASES = [({"obs_type": "vector_mdp", "action_std": 0.5, "time_limit": 6}, 65536, 12, 6),
               ({"obs_type": "vector_goal_mdp", "goal_xy": None, "use_velocity": True, "time_limit": 25}, 30001, 30, 3)]


@pytest.mark.parametrize("kw,B,steps,K", SPLIT_CASES)
def test_numpy_mode_two_launch_calls_vs_oracle(kw, B, steps, K, gpu_device):
    from gym_po_amd._lib import debug_knobs
    with debug_knobs(disable_fused=1):
        test_numpy_mode_vs_oracle(kw, B, steps, K, gpu_device)


# each path on the other side of the crossover (gp_debug_set xg_min_envs at create): the one-workgroup kernel up to
# its 4096-env limit, the grid-wide calls down to a single partial block
CROSS_CASES = [(ORACLE_CASES[0], 4096), (ORACLE_CASES[1], 4096), (ORACLE_CASES[3], 0),
               (({"obs_type": "vector_mdp", "action_std": 0.5, "time_limit": 6}, 64, 20, 4), 0)]


@pytest.mark.parametrize("case,xg_min", CROSS_CASES)
def test_numpy_mode_both_paths_across_crossover(case, xg_min, gpu_device):
    from gym_po_amd._lib import debug_knobs
    with debug_knobs(xg_min_envs=xg_min):
        test_numpy_mode_vs_oracle(*case, gpu_device)


# Round 6: the grid-wide K-step launch sequence replayed as a hipGraph (gp_debug_set xg_graph at create): 1 = from
# the first call (every call above captures anew or replays), 0 = never (the eager launches).
GRAPH_CASES = [(ORACLE_CASES[5], 1), (ORACLE_CASES[6], 1), (ORACLE_CASES[9], 1), (ORACLE_CASES[8], 0),
               (ORACLE_CASES[5], 0)]


@pytest.mark.parametrize("case,mode", GRAPH_CASES)
def test_numpy_mode_graph_knob_vs_oracle(case, mode, gpu_device):
    from gym_po_amd._lib import debug_knobs
    with debug_knobs(xg_graph=mode):
        test_numpy_mode_vs_oracle(*case, gpu_device)


@pytest.mark.parametrize("mode", [-1, 1])
@pytest.mark.parametrize("kw,B,K", [({"obs_type": "vector_goal_mdp", "goal_xy": None, "use_velocity": True,
                                      "time_limit": 7}, 30001, 4),
                                     ({"obs_type": "vector_mdp", "action_std": 0.5, "time_limit": 5}, 65536, 3)])
def test_numpy_mode_graph_replay_vs_oracle(kw, B, K, mode, gpu_device):
    """The same action / output buffers on every call (rollout_plan), so the graph is replayed: by default it is
    captured on the 2nd call and replayed from the 3rd. Every step against the oracle, and the final PCG64 state."""
    import torch
    from gym_po_amd import CRoomsEnv
    from gym_po_amd._lib import debug_knobs
    calls = 6
    acts = np.random.default_rng(5).uniform(-1, 1, (calls * K, B, 2))
    ora = CRoomsOracle(B, **kw)
    o_ref = ora.reset_seed(77)
    with debug_knobs(xg_graph=mode):
        env = CRoomsEnv(B, **kw, rng_mode="numpy", dtype=torch.float64)
    o = env.reset(seed=77).cpu().numpy()
    np.testing.assert_array_equal(o.astype(np.float64), np.asarray(o_ref).astype(np.float64))
    a = torch.zeros((K, B, 2), dtype=torch.float64, device=env.device)
    run, (obs, rew, term, trunc) = env.rollout_plan(a)
    eps = 0
    for c in range(calls):
        a.copy_(torch.as_tensor(acts[c * K:(c + 1) * K]))
        run()
        got = [x.cpu().numpy() for x in (obs, rew, term, trunc)]
        for j in range(K):
            ro, rr, rd, rt = ora.step_seeded(acts[c * K + j])
            tag = f"call {c} step {j}"
            np.testing.assert_array_equal(got[0][j].astype(np.float64), np.asarray(ro).astype(np.float64),
                                          err_msg="obs " + tag)
            np.testing.assert_array_equal(got[1][j], rr, err_msg="rew " + tag)
            np.testing.assert_array_equal(got[2][j].astype(bool), rd, err_msg="term " + tag)
            np.testing.assert_array_equal(got[3][j].astype(bool), rt, err_msg="trunc " + tag)
            eps += int((rd | rt).sum())
        assert _dev_state(env) == _np_state(ora.gen), f"PCG64 state after call {c}"
    m = env.metrics()
    assert m["episodes"] == eps and m["env_steps"] == calls * K * B


@pytest.mark.parametrize("kw,B,steps,K", ORACLE_CASES)
def test_numpy_mode_vs_oracle(kw, B, steps, K, gpu_device):
    """Every step against the oracle on numpy's Generator; K-step launches; final PCG64 state."""
    import torch
    from gym_po_amd import CRoomsEnv
    rng = np.random.default_rng(11)
    yx = kw.get("action_type", "yx") == "yx"
    acts = (rng.uniform(-1, 1, (steps, B, 2)) if yx else
            rng.integers(0, 8 if kw.get("action_type") == "ordinal" else 4, (steps, B)))
    ora = CRoomsOracle(B, **kw)
    o_ref = ora.reset_seed(123)
    env = CRoomsEnv(B, **kw, rng_mode="numpy", dtype=torch.float64)
    o = env.reset(seed=123).cpu().numpy()
    np.testing.assert_array_equal(o.astype(np.float64), np.asarray(o_ref).astype(np.float64))
    eps = 0
    for t0 in range(0, steps, K):
        k = min(K, steps - t0)
        ta = torch.as_tensor(acts[t0:t0 + k])
        if yx:
            ta = ta.to(torch.float64)
        else:
            ta = ta.to(torch.int32)
        if k == 1:
            got = [x.cpu().numpy()[None] for x in env.step(ta[0])[:4]]
        else:
            got = [x.cpu().numpy() for x in env.rollout(ta)[:4]]
        for j in range(k):
            ro, rr, rd, rt = ora.step_seeded(acts[t0 + j])
            tag = f"t={t0 + j}"
            np.testing.assert_array_equal(got[0][j].astype(np.float64), np.asarray(ro).astype(np.float64),
                                          err_msg="obs " + tag)
            np.testing.assert_array_equal(got[1][j], rr, err_msg="rew " + tag)
            np.testing.assert_array_equal(got[2][j].astype(bool), rd, err_msg="term " + tag)
            np.testing.assert_array_equal(got[3][j].astype(bool), rt, err_msg="trunc " + tag)
            eps += int((rd | rt).sum())
        assert _dev_state(env) == _np_state(ora.gen), f"PCG64 state after t={t0 + k - 1}"
    a, g, v, e = (x.cpu().numpy() for x in env.get_state())
    np.testing.assert_array_equal(a, ora.agent)
    np.testing.assert_array_equal(e, ora.elapsed)
    m = env.metrics()
    assert m["episodes"] == eps and m["env_steps"] == steps * B


def test_numpy_mode_f32_io_and_state_roundtrip(gpu_device):
    """float32 I/O (obs = f32(reference obs)); np_random get/set continues the reference stream."""
    import torch
    from gym_po_amd import CRoomsEnv
    B, steps = 2000, 20
    kw = {"obs_type": "vector_mdp", "time_limit": 10}
    acts = np.random.default_rng(3).uniform(-1, 1, (steps, B, 2)).astype(np.float32).astype(np.float64)
    ora = CRoomsOracle(B, **kw)
    ora.reset_seed(9)
    env = CRoomsEnv(B, **kw, rng_mode="numpy")
    env.reset(seed=9)
    for t in range(steps):
        if t == 10:  # hand the stream to numpy and back: the device continues from the set state
            env.np_random = ora.gen
        o = env.step(torch.as_tensor(acts[t], dtype=torch.float32))[0].cpu().numpy()
        ro = ora.step_seeded(acts[t])[0]
        assert o.dtype == np.float32
        np.testing.assert_array_equal(o, np.asarray(ro).astype(np.float32), err_msg=f"t={t}")
    assert _dev_state(env) == _np_state(ora.gen)
