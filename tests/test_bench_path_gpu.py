"""Parity of the EXACT kernel path bench.py times (VERDICT r1 "next" #1).

bench.py's headline is `MultistoryFourRoomsEnv(2^20, grid_z=1, obs_type="hansen")` in numpy mode,
stepped through `rollout_plan` with chunks of C steps per launch (C = 20 at the driver's
`--steps 20`, 128 by default). At 2^20 envs on a 256-CU MI355X that is one persistent launch of the
windowed kernel `wgrid_rollout<8, 4>` (csrc/wgrid.hip): 256 blocks of 4096 envs, each step's reset count
published early from the truncations and the goal-adjacent envs' words, outputs staged in LDS and copied out
by the store waves while the env waves run the next step, env state in registers across the K steps.
These tests run that kernel with K > 1 and compare EVERY step's obs,
reward, terminated and truncated, plus the final env state and PCG64 state, against the numpy
oracle (tests/test_oracle_golden.py pins the oracle to reference-generated fixtures):
- K = 20 and K = 128 launches (the driver's and bench's chunks), one after the other;
- a launch that straddles chunk boundaries (K = 128 then K = 7);
- time_limit=20: every env that has not reached the goal truncates inside one launch (a mass
  reset far beyond the speculative rejection-check window: the coverage-round path);
- random goals (two choice() calls per reset: coverage round for the agent words) on the staged
  kernel with K > 1.
Reference semantics followed: msrooms.py:369-413 (step/_reset_some), rooms.py:177-222.
"""
import numpy as np
import pytest

from oracle import gridworld

pytestmark = pytest.mark.gpu

B_BENCH = 1 << 20


def _rng_tuple(st):
    s, inc = st["state"]["state"], st["state"]["inc"]
    m = (1 << 64) - 1
    return [s >> 64, s & m, inc >> 64, inc & m, st["has_uint32"], st["uinteger"]]


def _reset_obs(env, seed):
    r = env.reset(seed=seed)
    return (r[0] if isinstance(r, tuple) else r).cpu().numpy()


def _staged_geometry(env):
    """The launch geometry the bench kernel needs (else the test would not cover it)."""
    G, q, stg = env.query("fused_blocks"), env.query("fused_tiles_per_block"), env.query("fused_staged")
    tile = env.query("fused_tile_envs")
    return G, q, stg, tile


def _check_chunks(env, ora, chunks, action_seed, n_act):
    import torch
    dev = env.device
    rng = np.random.default_rng(action_seed)
    for K in chunks:
        a_np = rng.integers(0, n_act, (K, env.num_envs)).astype(np.int32)
        acts = torch.as_tensor(a_np, device=dev)
        run, (obs, rew, term, trunc) = env.rollout_plan(acts)
        run()
        o, r, d, t = (x.cpu().numpy() for x in (obs, rew, term, trunc))
        for k in range(K):
            oo, ro, do, tro = ora.step_seeded(a_np[k].astype(np.int64))
            np.testing.assert_array_equal(o[k].astype(np.int64), np.asarray(oo).astype(np.int64),
                                          err_msg=f"obs K={K} k={k}")
            np.testing.assert_array_equal(r[k], ro, err_msg=f"rew K={K} k={k}")
            np.testing.assert_array_equal(d[k], do, err_msg=f"term K={K} k={k}")
            np.testing.assert_array_equal(t[k], tro, err_msg=f"trunc K={K} k={k}")
    env.check()
    assert _rng_tuple(env.rng_state) == _rng_tuple(ora.gen.bit_generator.state)
    a, g, e = (x.cpu().numpy() for x in env.get_state())
    np.testing.assert_array_equal(a, np.ravel_multi_index(tuple(ora.agent.T), ora.grid.shape))
    np.testing.assert_array_equal(g, np.ravel_multi_index(tuple(ora.goal.T), ora.grid.shape))
    np.testing.assert_array_equal(e, ora.elapsed)


# (1, 4, 20): bench.py's driver sequence (two warmup launches of 1 and W - 1 = 4 steps, then the timed 20).
# kernel "wgrid": the windowed rollout (csrc/wgrid.hip), which bench.py times; "fused": the older fused kernel
# (no_wgrid knob; its speculative word windows SPW_NJ on or forced off). The first steps after a reset predict
# the window from a stale reset total (exact regeneration), time_limit=20 puts mass resets (every env truncated
# in one step: the slow path's coverage rounds) inside the launches.
@pytest.mark.parametrize("kernel,chunks,time_limit,spw", [
    ("wgrid", (20, 128), 500, 1), ("wgrid", (128, 7), 500, 1), ("wgrid", (20, 20), 20, 1), ("wgrid", (1, 4, 20), 500, 1),
    ("fused", (20, 128), 500, 1), ("fused", (20, 20), 20, 1), ("fused", (1, 4, 20), 500, 0)])
def test_bench_kernel_staged_k_step_launches_bit_exact(kernel, chunks, time_limit, spw, gpu_device):
    from gym_po_amd import MultistoryFourRoomsEnv
    from gym_po_amd._lib import debug_knobs
    with debug_knobs(no_spw=1 - spw, no_wgrid=kernel != "wgrid"):
        env = MultistoryFourRoomsEnv(B_BENCH, grid_z=1, obs_type="hansen", time_limit=time_limit, device=gpu_device)
    assert env.query("wgrid") == (kernel == "wgrid")
    if kernel == "wgrid":
        assert (env.query("wgrid_blocks"), env.query("wgrid_block_envs")) == (256, 4096)
    else:
        G, q, stg, tile = _staged_geometry(env)
        if G * q * tile != B_BENCH or not stg:
            pytest.skip(f"this GPU does not give the bench geometry (G={G}, tiles/block={q}, staged={stg})")
        assert env.query("fused_spw") == spw
    ora = gridworld.FourRoomsOracle(B_BENCH, 1, obs_type="hansen", time_limit=time_limit)
    o_g = _reset_obs(env, 2024)
    np.testing.assert_array_equal(o_g.astype(np.int64), np.asarray(ora.reset_seed(2024)).astype(np.int64))
    _check_chunks(env, ora, chunks, action_seed=11 + time_limit, n_act=4)
    if time_limit == 20:  # every env truncated or reached the goal inside the launches
        assert env.metrics()["episodes"] >= B_BENCH


def test_bench_kernel_random_goal_staged_k_steps(gpu_device):
    """rooms_2_goal_mdp_randgoal shape (random goal and agent: two choice() calls per reset) at 2^20 envs."""
    from gym_po_amd import RoomsEnv
    kw = dict(layout="2", obs_type="goal_mdp", time_limit=60, goal_xy=None)
    env = RoomsEnv(B_BENCH, **kw, device=gpu_device)
    G, q, stg, tile = _staged_geometry(env)
    if G * q * tile != B_BENCH or not stg:
        pytest.skip(f"this GPU does not give the staged geometry (G={G}, tiles/block={q}, staged={stg})")
    ora = gridworld.RoomsOracle(B_BENCH, **kw)
    o_g = _reset_obs(env, 77)
    np.testing.assert_array_equal(o_g.astype(np.int64), np.asarray(ora.reset_seed(77)).astype(np.int64))
    _check_chunks(env, ora, (24, 40), action_seed=5, n_act=8)


@pytest.mark.parametrize("B,force_tile", [(1 << 17, 0), (1 << 18, 0), (1 << 17, 2048), (1 << 18, 512),
                                          (3 << 17, 0)])
def test_strong_scaling_shard_sizes_staged_bit_exact(B, force_tile, gpu_device):
    """(The older fused kernel; the windowed kernel's shard sizes: test_wgrid_gpu.py.) The per-GPU shard of a strong-scaling run (1M envs over 8 / 4 GPUs): 2^17 / 2^18 envs get tiles of 512 /
    1024 envs (2 / 4 env waves per block) so that every CU has one; also forced to 2048-env tiles (64 blocks of
    8 env waves) and 512-env tiles (two tiles per block), and 3 * 2^17 (1024-env tiles, 1.5 per CU). K = 20
    then 128 steps per launch, bit-exact."""
    from gym_po_amd import MultistoryFourRoomsEnv
    from gym_po_amd._lib import debug_knobs
    with debug_knobs(fused_tile=force_tile, no_wgrid=1):
        env = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device=gpu_device)
    G, q, stg, tile = _staged_geometry(env)
    assert G * (q - 1) * tile < B <= G * q * tile, (G, q, stg, tile)
    assert tile == (force_tile or {1 << 17: 512, 1 << 18: 1024, 3 << 17: 1024}[B])
    assert bool(stg) == (B == G * q * tile), (G, q, stg, tile)  # staged iff the tiles are complete
    ora = gridworld.FourRoomsOracle(B, 1, obs_type="hansen")
    o_g = _reset_obs(env, 31)
    np.testing.assert_array_equal(o_g.astype(np.int64), np.asarray(ora.reset_seed(31)).astype(np.int64))
    _check_chunks(env, ora, (20, 128), action_seed=3, n_act=4)
