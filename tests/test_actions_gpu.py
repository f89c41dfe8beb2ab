"""Action indexing as the reference does it (VERDICT r2 "next" #1b and #7).

The reference indexes a per-action table with the raw action: `self.action_matrix[action]` (msrooms.py:400,
rooms.py:208) and `self.ACTIONS_YX[actions]` (extended_taxi.py:248). numpy therefore
- wraps negative actions in [-n, 0) (action -1 is the last action), and
- raises IndexError for anything outside [-n, n).
Here:
- negative actions wrap exactly as numpy's: bit-exact against the oracle (which indexes the same way) on the
  staged fused kernel at the bench size (2^20 envs, FourRooms cardinal) and on ROOMS ordinal, and on the
  two-kernel numpy path;
- out-of-range actions given as host arrays raise the reference's IndexError before anything is launched;
  given as device tensors they cannot be checked without a sync, so the kernels flag the handle
  (GP_DERR_ACTION) and check() / metrics() raise GymPoError; reseeding clears the flag.
"""
import numpy as np
import pytest

from oracle import gridworld

pytestmark = pytest.mark.gpu


def _rng_tuple(st):
    s, inc = st["state"]["state"], st["state"]["inc"]
    m = (1 << 64) - 1
    return [s >> 64, s & m, inc >> 64, inc & m, st["has_uint32"], st["uinteger"]]


def _obs0(r):
    return (r[0] if isinstance(r, tuple) else r).cpu().numpy().astype(np.int64)


def _rollouts_vs_oracle(env, ora, n_act, chunks, seed):
    import torch
    rng = np.random.default_rng(seed)
    for K in chunks:
        a_np = rng.integers(-n_act, n_act, (K, env.num_envs)).astype(np.int32)
        run, (obs, rew, term, trunc) = env.rollout_plan(torch.as_tensor(a_np, device=env.device))
        run()
        o, r, d, t = (x.cpu().numpy() for x in (obs, rew, term, trunc))
        for k in range(K):
            oo, ro, do, tro = ora.step_seeded(a_np[k].astype(np.int64))
            np.testing.assert_array_equal(o[k].astype(np.int64), np.asarray(oo).astype(np.int64), err_msg=f"K={K} k={k}")
            np.testing.assert_array_equal(r[k], ro, err_msg=f"K={K} k={k}")
            np.testing.assert_array_equal(d[k], do, err_msg=f"K={K} k={k}")
            np.testing.assert_array_equal(t[k], tro, err_msg=f"K={K} k={k}")
    env.check()  # in-range negative actions are not flagged
    assert _rng_tuple(env.rng_state) == _rng_tuple(ora.gen.bit_generator.state)


def test_negative_actions_fourrooms_bench_kernel(gpu_device):
    from gym_po_amd import MultistoryFourRoomsEnv
    B = 1 << 20
    env = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device=gpu_device)
    assert env.query("fused_staged") == 1 and env.query("fused_blocks") > 0
    ora = gridworld.FourRoomsOracle(B, 1, obs_type="hansen")
    np.testing.assert_array_equal(_obs0(env.reset(seed=41)), np.asarray(ora.reset_seed(41)).astype(np.int64))
    _rollouts_vs_oracle(env, ora, 4, (20, 7), seed=42)


def test_negative_actions_rooms_ordinal_fused(gpu_device):
    from gym_po_amd import RoomsEnv
    B = 1 << 20
    kw = dict(layout="4", obs_type="hansen", action_type="ordinal", time_limit=80)
    env = RoomsEnv(B, **kw, device=gpu_device)
    assert env.query("fused_blocks") > 0
    ora = gridworld.RoomsOracle(B, **kw)
    np.testing.assert_array_equal(_obs0(env.reset(seed=43)), np.asarray(ora.reset_seed(43)).astype(np.int64))
    _rollouts_vs_oracle(env, ora, 8, (16,), seed=44)


@pytest.mark.parametrize("kind", ["fourrooms", "rooms"])
def test_negative_actions_two_kernel_path(kind, gpu_device):
    from gym_po_amd import MultistoryFourRoomsEnv, RoomsEnv
    from gym_po_amd._lib import debug_knobs
    B, T = (1 << 16) + 5, 30
    with debug_knobs(disable_fused=1):
        if kind == "fourrooms":
            env = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", time_limit=40, device=gpu_device)
            ora, n = gridworld.FourRoomsOracle(B, 1, obs_type="hansen", time_limit=40), 4
        else:
            kw = dict(layout="4", obs_type="hansen", action_type="ordinal", time_limit=40)
            env, ora, n = RoomsEnv(B, **kw, device=gpu_device), gridworld.RoomsOracle(B, **kw), 8
    assert env.query("fused_blocks") == 0
    np.testing.assert_array_equal(_obs0(env.reset(seed=45)), np.asarray(ora.reset_seed(45)).astype(np.int64))
    rng = np.random.default_rng(46)
    for t in range(T):
        a = rng.integers(-n, n, B)
        o, r, d, tr, _ = env.step(a)
        oo, ro, do, tro = ora.step_seeded(a)
        np.testing.assert_array_equal(o.cpu().numpy().astype(np.int64), np.asarray(oo).astype(np.int64), err_msg=f"t={t}")
        np.testing.assert_array_equal(r.cpu().numpy(), ro)
        np.testing.assert_array_equal(d.cpu().numpy(), do)
        np.testing.assert_array_equal(tr.cpu().numpy(), tro)
    env.check()
    assert _rng_tuple(env.rng_state) == _rng_tuple(ora.gen.bit_generator.state)


def _make(kind, gpu_device, **kw):
    from gym_po_amd import HansenTaxiVecEnv, MultistoryFourRoomsEnv, RoomsEnv
    if kind == "fourrooms":
        return MultistoryFourRoomsEnv(4096, grid_z=1, obs_type="hansen", device=gpu_device, **kw), 4
    if kind == "rooms":
        return RoomsEnv(4096, layout="4", obs_type="hansen", action_type="ordinal", device=gpu_device, **kw), 8
    return HansenTaxiVecEnv(4096, device=gpu_device, **kw), 5


@pytest.mark.parametrize("kind,mode,fused", [("fourrooms", "numpy", True), ("fourrooms", "numpy", False),
                                             ("rooms", "philox", True), ("taxi", "philox", True)])
@pytest.mark.parametrize("bad", ["n", "-n-1"])
def test_out_of_range_device_actions_flag_the_handle(kind, mode, fused, bad, gpu_device):
    import torch
    from gym_po_amd._lib import GymPoError, debug_knobs
    with debug_knobs(disable_fused=not fused):
        env, n = _make(kind, gpu_device, rng_mode=mode)
    env.reset(seed=5)
    acts = torch.randint(-n, n, (3, env.num_envs), dtype=torch.int32, device=gpu_device)
    env.rollout(acts)
    env.check()  # in range (negatives wrap): no flag
    acts[1, 1234] = n if bad == "n" else -n - 1
    env.rollout(acts)  # asynchronous: the step still runs (clamped), the handle is flagged
    with pytest.raises(GymPoError, match="outside"):
        env.check()
    with pytest.raises(GymPoError, match="outside"):
        env.metrics()
    env.reset(seed=6)  # a new seed clears the flag
    env.check()


@pytest.mark.parametrize("kind", ["fourrooms", "rooms", "taxi"])
def test_out_of_range_host_actions_raise_index_error(kind, gpu_device):
    env, n = _make(kind, gpu_device)
    env.reset(seed=1)
    a = np.zeros(env.num_envs, np.int64)
    for bad in (n, -n - 1):
        a[7] = bad
        with pytest.raises(IndexError, match=f"index {bad} is out of bounds for axis 0 with size {n}"):
            env.step(a)
    a[7] = -n  # the most negative valid index wraps
    env.step(a)
    env.check()
