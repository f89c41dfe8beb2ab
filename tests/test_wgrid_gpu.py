"""GPU parity of the windowed numpy-exact rollout (csrc/wgrid.hip), the kernel bench.py times.

Every case compares each step's obs / reward / terminated / truncated, the final env state and the final PCG64
state (incl. numpy's buffered half-word) with the numpy oracle (pinned to reference fixtures by
tests/test_oracle_golden.py), through K-step launches of the C-ABI plan (`rollout_plan`) exactly as bench.py
drives them. Reference semantics: msrooms.py:369-413, rooms.py:177-222, action_utils.py:84-90.

What each case forces:
- block sizes E = 512 / 1024 / 2048 / 4096 envs (the strong-scaling shards of 1M envs over 8 / 4 / 2 GPUs);
- a window halo of 512 draws, and a prediction bias that puts every step's window outside its halo (the exact
  regeneration after the exchange);
- a Lemire rejection planted in the choice() stream inside a launch (the slow path: rejected positions listed,
  every resetter placed exactly);
- ordinal actions (8 thresholds per row) and table obs (ROOMS layouts);
- the kernel choice by launch length (launches of more than wg_kmax steps run the fused kernel on the same stream
  and state): every launch on either kernel, and the default split, over mixed launch lengths.
"""
import numpy as np
import pytest

from oracle import gridworld
from oracle.pcg64 import MASK128, lemire_threshold, pcg_advance_params, pcg_output

pytestmark = pytest.mark.gpu


def _rng_tuple(st):
    s, inc = st["state"]["state"], st["state"]["inc"]
    m = (1 << 64) - 1
    return [s >> 64, s & m, inc >> 64, inc & m, st["has_uint32"], st["uinteger"]]


def _reset_obs(env, seed):
    r = env.reset(seed=seed)
    return (r[0] if isinstance(r, tuple) else r).cpu().numpy()


def _check_chunks(env, ora, chunks, action_seed, n_act, before_chunk=None):
    import torch
    rng = np.random.default_rng(action_seed)
    for ci, K in enumerate(chunks):
        if before_chunk:
            before_chunk(ci)
        a_np = rng.integers(0, n_act, (K, env.num_envs)).astype(np.int32)
        run, (obs, rew, term, trunc) = env.rollout_plan(torch.as_tensor(a_np, device=env.device))
        run()
        o, r, d, t = (x.cpu().numpy() for x in (obs, rew, term, trunc))
        for k in range(K):
            oo, ro, do, tro = ora.step_seeded(a_np[k].astype(np.int64))
            np.testing.assert_array_equal(o[k].astype(np.int64), np.asarray(oo).astype(np.int64),
                                          err_msg=f"obs chunk {ci} K={K} k={k}")
            np.testing.assert_array_equal(r[k], ro, err_msg=f"rew chunk {ci} k={k}")
            np.testing.assert_array_equal(d[k], do, err_msg=f"term chunk {ci} k={k}")
            np.testing.assert_array_equal(t[k], tro, err_msg=f"trunc chunk {ci} k={k}")
    env.check()
    assert _rng_tuple(env.rng_state) == _rng_tuple(ora.gen.bit_generator.state)
    a, g, e = (x.cpu().numpy() for x in env.get_state())
    np.testing.assert_array_equal(a, np.ravel_multi_index(tuple(ora.agent.T), ora.grid.shape))
    np.testing.assert_array_equal(e, ora.elapsed)


def _fourrooms(B, device, **kw):
    from gym_po_amd import MultistoryFourRoomsEnv
    return MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device=device, **kw)


@pytest.mark.parametrize("kmax", [0, 24, 1000])
def test_kernel_choice_by_launch_length_bit_exact(kmax, gpu_device):
    from gym_po_amd._lib import debug_knobs
    B = 1 << 18
    with debug_knobs(wg_kmax=kmax):
        env = _fourrooms(B, gpu_device)
    assert env.query("wgrid") == 1
    ora = gridworld.FourRoomsOracle(B, 1, obs_type="hansen")
    np.testing.assert_array_equal(_reset_obs(env, 41).astype(np.int64), np.asarray(ora.reset_seed(41)).astype(np.int64))
    _check_chunks(env, ora, (1, 20, 33, 2, 64, 24, 25), action_seed=8, n_act=4)
    assert env.metrics()["env_steps"] == B * 169


@pytest.mark.parametrize("fstep", [8185, 16380])
def test_fused_tag_wrap_between_windowed_launches_bit_exact(fstep, gpu_device):
    """The fused kernel's 15-bit granule tags ((step + 1) * 4 + round) wrap every 8192 of its steps; round 0 of the
    wrapping step expects tag 0. Its tag counter (GridCtl::step, started near the wrap by the fused_step knob) is
    advanced only by fused launches, its slots start at a tag it never expects, and windowed launches interleave:
    the results must stay the oracle's through the wrap (zeroed slots matched tag 0)."""
    from gym_po_amd._lib import debug_knobs
    B = 1 << 19  # (2048-env blocks: launches of > 24 steps default to the fused kernel)
    with debug_knobs(fused_step=fstep):
        env = _fourrooms(B, gpu_device)
        ora = gridworld.FourRoomsOracle(B, 1, obs_type="hansen")
        np.testing.assert_array_equal(_reset_obs(env, 77).astype(np.int64),
                                      np.asarray(ora.reset_seed(77)).astype(np.int64))
    assert env.query("wgrid") == 1 and env.query("wgrid_kmax") == 24
    # windowed (3), fused across the wrap (40), windowed (2), fused (33)
    _check_chunks(env, ora, (3, 40, 2, 33), action_seed=12, n_act=4)
    assert env.metrics()["env_steps"] == B * 78


def test_small_blocks_default_to_windowed_at_every_length(gpu_device):
    """Blocks of <= 1,024 envs (2^17 / 2^18 envs: the strong-scaling shards) and of 4,096 envs (2^20, the headline)
    run the windowed kernel for every launch length by default; 2048-env blocks hand launches of more than 24 steps
    to the fused kernel."""
    for B, kmax in ((1 << 17, 1 << 30), (1 << 18, 1 << 30), (1 << 19, 24), (1 << 20, 1 << 30)):
        env = _fourrooms(B, gpu_device)
        assert env.query("wgrid_kmax") == kmax, B
        env.close()


@pytest.mark.parametrize("B,E", [(1 << 17, 512), (1 << 18, 1024), (1 << 19, 2048), (3 << 17, 2048), (8192, 512)])
def test_wgrid_block_sizes_bit_exact(B, E, gpu_device):
    env = _fourrooms(B, gpu_device)
    assert env.query("wgrid") == 1
    assert env.query("wgrid_block_envs") == E and env.query("wgrid_blocks") * E == B
    ora = gridworld.FourRoomsOracle(B, 1, obs_type="hansen")
    np.testing.assert_array_equal(_reset_obs(env, 31).astype(np.int64), np.asarray(ora.reset_seed(31)).astype(np.int64))
    _check_chunks(env, ora, (20, 33, 1), action_seed=3, n_act=4)
    m = env.metrics()
    assert m["env_steps"] == B * 54


@pytest.mark.parametrize("knobs", [dict(wg_halo=512), dict(wg_bias=3000), dict(wg_bias=-600), dict(wg_fill_simd=0xFFF3),
                                   dict(wg_fill_simd=0x6EEE), dict(wg_fill_simd=0x6EEE, wg_bias=3000),
                                   dict(wg_halo=512, wg_fill_simd=0x11E0), dict(wg_fill_wave=0xEEEE2222),
                                   dict(wg_fill_wave=0x1E2F0E11, wg_bias=-600)])
def test_wgrid_halo_and_forced_window_misses(knobs, gpu_device):
    """wg_bias shifts every step's predicted reset count (3000 resets = ~1500 draws, far beyond the 256-draw
    halo; -600 wraps to a huge count): each step's window is regenerated exactly after the exchange.
    wg_fill_simd moves window rows between the SIMDs' env waves (every distribution fills the same words)."""
    from gym_po_amd._lib import debug_knobs
    B = 1 << 20
    with debug_knobs(**knobs):
        env = _fourrooms(B, gpu_device)
    assert env.query("wgrid") == 1
    assert env.query("wgrid_halo") == knobs.get("wg_halo", 256)
    ora = gridworld.FourRoomsOracle(B, 1, obs_type="hansen")
    np.testing.assert_array_equal(_reset_obs(env, 5).astype(np.int64), np.asarray(ora.reset_seed(5)).astype(np.int64))
    _check_chunks(env, ora, (12, 5), action_seed=9, n_act=4)


def _rejected_word(n, k=1):
    thr = lemire_threshold(n)
    for kk in range(k, k + 10000):
        r = -(-(kk << 32) // n)
        if r < (1 << 32) and (r * n) & 0xFFFFFFFF < thr:
            return r
    raise AssertionError


def _rotl(x, r):
    return ((x << r) | (x >> ((64 - r) & 63))) & ((1 << 64) - 1)


def _state_with_output_half(half_value, half, seed):
    rng = np.random.default_rng(seed)
    hi = int(rng.integers(0, 2 ** 63)) * 2 + 1
    other = int(rng.integers(0, 2 ** 32))
    x = (other << 32) | half_value if half == 0 else (half_value << 32) | other
    lo = hi ^ _rotl(x, hi >> 58)
    s = (hi << 64) | lo
    assert pcg_output(s) == x
    return s


@pytest.mark.parametrize("word", [3, 2001, 40000])
def test_wgrid_planted_rejection_inside_launch(word, gpu_device):
    """The PCG64 state is set so that half-word `word` of the next step's choice() stream is a rejected Lemire
    draw (word 40000 lies beyond the first 124 G half-words: a coverage round is needed only if that step resets
    more envs than that, otherwise the flag alone takes the slow path). Then one 9-step launch and one of 3."""
    B = 1 << 20
    env = _fourrooms(B, gpu_device)
    ora = gridworld.FourRoomsOracle(B, 1, obs_type="hansen")
    _reset_obs(env, 7)
    ora.reset_seed(7)
    n = len(ora.valid_agent)

    def plant(ci):
        if ci != 1:
            return
        inc = ora.gen.bit_generator.state["state"]["inc"]
        q, half = word >> 1, word & 1
        s_star = _state_with_output_half(_rejected_word(n), half, word)
        a, c = pcg_advance_params((1 << 128) - (B + q + 1), inc)
        st = {"bit_generator": "PCG64", "state": {"state": (a * s_star + c) & MASK128, "inc": inc},
              "has_uint32": 0, "uinteger": 0}
        env.rng_state = st
        ora.gen.bit_generator.state = st

    _check_chunks(env, ora, (4, 9, 3), action_seed=21, n_act=4, before_chunk=plant)


@pytest.mark.parametrize("kind,kw,B", [
    ("rooms", dict(layout="4", obs_type="hansen"), 1 << 18),       # ordinal (8 actions), binary Hansen-4
    ("rooms", dict(layout="4", obs_type="mdp"), 1 << 17),          # table obs
    ("fourrooms", dict(grid_z=1, obs_type="mdp"), 1 << 18),        # table obs, cardinal
])
def test_wgrid_other_fixed_goal_configs(kind, kw, B, gpu_device):
    from gym_po_amd import MultistoryFourRoomsEnv, RoomsEnv
    if kind == "rooms":
        env = RoomsEnv(B, **kw, device=gpu_device)
        ora = gridworld.RoomsOracle(B, **kw)
    else:
        env = MultistoryFourRoomsEnv(B, **kw, device=gpu_device)
        ora = gridworld.FourRoomsOracle(B, **kw)
    assert env.query("wgrid") == 1
    np.testing.assert_array_equal(_reset_obs(env, 13).astype(np.int64), np.asarray(ora.reset_seed(13)).astype(np.int64))
    _check_chunks(env, ora, (16, 16), action_seed=4, n_act=env.single_action_space.n)


def test_wgrid_single_steps_equal_rollout(gpu_device):
    """env.step (K = 1 launches of the same kernel) equals one K-step rollout, outputs and RNG state."""
    import torch
    B, K = 1 << 16, 24
    e1, e2 = _fourrooms(B, gpu_device), _fourrooms(B, gpu_device)
    e1.reset(seed=8)
    e2.reset(seed=8)
    acts = torch.randint(0, 4, (K, B), device=gpu_device, dtype=torch.int32)
    o1, r1, d1, t1 = e1.rollout(acts)
    for k in range(K):
        o2, r2, d2, t2, _ = e2.step(acts[k])
        assert torch.equal(o1[k], o2) and torch.equal(r1[k], r2) and torch.equal(d1[k], d2) and torch.equal(t1[k], t2)
    assert e1.rng_state == e2.rng_state
    assert e1.metrics() == e2.metrics()


def _goal_adjacent_cells(ora):
    """Flat cells from which some move lands on the (fixed) goal, and the goal itself (msrooms.py:401-407)."""
    shape = ora.grid.shape
    goal = np.asarray(ora.goal[0])
    out = [int(np.ravel_multi_index(tuple(goal), shape))]
    for c in np.asarray(ora.valid_agent).ravel():
        zyx = np.array(np.unravel_index(int(c), shape))
        if any((zyx + off == goal).all() for off in np.asarray(ora.actions)):
            out.append(int(c))
    return np.unique(np.array(out, np.int64))


@pytest.mark.parametrize("B,frac", [(1 << 20, 0.9), (1 << 20, 0.2), (1 << 20, 0.05), (1 << 17, 0.5)])
def test_wgrid_goal_crowd_bit_exact(B, frac, gpu_device):
    """Most (or many) envs put on goal-adjacent cells with set_state, so that hundreds of thousands (0.9) down to
    a few hundred per block (0.05) reach the goal in the same step: the step's reset count, the rank-ordered
    resetter lists and the window regeneration (the count lands far outside the predicted window) stay exact, and
    every later step is bit-exact too."""
    env = _fourrooms(B, gpu_device)
    assert env.query("wgrid") == 1
    ora = gridworld.FourRoomsOracle(B, 1, obs_type="hansen")
    _reset_obs(env, 17)
    ora.reset_seed(17)
    near = _goal_adjacent_cells(ora)
    assert len(near) >= 2
    rng = np.random.default_rng(5)
    valid = np.asarray(ora.valid_agent).ravel()
    cells = np.where(rng.random(B) < frac, rng.choice(near, B), rng.choice(valid, B)).astype(np.int64)
    el = rng.integers(0, ora.time_limit + 1, B).astype(np.int64)
    env.set_state(agent_cells=cells.astype(np.int32), elapsed=el.astype(np.int32))
    ora.agent = np.array(np.unravel_index(cells, ora.grid.shape)).swapaxes(0, 1).astype(int)
    ora.elapsed = el.astype(int)
    _check_chunks(env, ora, (6, 1, 9), action_seed=11, n_act=4)


@pytest.mark.parametrize("tmode", [4, 64, 128, 32 | 512, 8 | 16, 4096, 8192, 16384, 16384 | 128])
def test_wgrid_schedule_variants_bit_exact(tmode, gpu_device):
    """Test-only schedules of the windowed kernel (gp_debug_set wg_tmode, wgrid.hip TM_*): 4 = next actions loaded
    after the transitions, 64 = store waves copy a step as soon as it is final, 128 = no candidate cells (every
    resetter's word drawn after the exchange), 32|512 = env-wave priority off / always high, 8|16 = throttled
    stores and busy polling, 4096 = next actions loaded at the step start, 8192 = round 5's prologue, 16384 = the
    control wave places the resetters' cells (at this size the env waves do by default). Results must not depend
    on the schedule."""
    from gym_po_amd._lib import debug_knobs
    B = 1 << 18
    with debug_knobs(wg_tmode=tmode):
        env = _fourrooms(B, gpu_device)
    assert env.query("wgrid") == 1
    ora = gridworld.FourRoomsOracle(B, 1, obs_type="hansen")
    np.testing.assert_array_equal(_reset_obs(env, 23).astype(np.int64), np.asarray(ora.reset_seed(23)).astype(np.int64))
    _check_chunks(env, ora, (7, 12), action_seed=2, n_act=4)


def test_autotune_leaves_the_state_exactly(gpu_device):
    """gp_autotune times both kernels on scratch state and restores the handle's: a tuned env and an untuned one
    from the same seed give identical outputs, state, metrics and PCG64 state afterwards, over launches of the
    tuned length and others."""
    import torch
    B = 1 << 18
    e1, e2 = _fourrooms(B, gpu_device), _fourrooms(B, gpu_device)
    o1, o2 = _reset_obs(e1, 12), _reset_obs(e2, 12)
    acts = torch.randint(0, 4, (45, B), device=gpu_device, dtype=torch.int32)
    e1.rollout(acts[:5])
    e2.rollout(acts[:5])
    chosen = e1.autotune(20, reps=3)
    assert chosen in (0, 1)
    assert (e1.query("wgrid_kmax") >= 20) == (chosen == 1)
    for a, b in ((5, 25), (25, 26), (26, 45)):
        r1, r2 = e1.rollout(acts[a:b]), e2.rollout(acts[a:b])
        for x, y in zip(r1, r2):
            assert torch.equal(x, y)
    assert e1.rng_state == e2.rng_state
    assert e1.metrics() == e2.metrics()
    for x, y in zip(e1.get_state(), e2.get_state()):
        assert torch.equal(x, y)


def test_autotune_is_a_no_op_where_there_is_nothing_to_choose(gpu_device):
    """Other kinds and modes have one kernel per launch length: gp_autotune returns -1 and changes nothing."""
    from gym_po_amd import CRoomsEnv, TaxiVecEnv
    envs = [_fourrooms(1 << 16, gpu_device, rng_mode="philox"), TaxiVecEnv(4096, device=gpu_device),
            CRoomsEnv(4096, rng_mode="numpy", device=gpu_device)]
    for env in envs:
        env.reset(seed=3)
        assert env.autotune(20) == -1
