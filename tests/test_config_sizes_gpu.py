"""Parity at BASELINE.json's own config sizes for the non-headline workloads (VERDICT r2 "next" #1a, #1c).

- configs[4]: `CRoomsEnv(2^21, obs_type="vector_mdp")`, float32 actions in / float32 obs out (crooms.py:251-338).
  Replay mode is fed the values the reference's own numpy stream produced (the fixture-pinned oracle on the
  same seed) for 8 steps: obs == float32(reference obs) exactly (|err| <= 2^-24 |ref|, the one float32
  rounding of the float64 state), reward / terminated / truncated equal. Philox mode (the bench kernel,
  `crooms_rollout<GP_OBS_F32,false>`): one K = 128 rollout launch equals 128 single steps bit for bit.
- configs[3]: grid Ant-Tag at 2^21 envs per GPU (the per-GPU shard of 16M over 8): philox mode against the
  oracle that recomputes the device's Philox counters (oracle/anttag.py, build-defined spec; ant_tag.py:88-157
  rules) for 24 steps, bit for bit, plus the final state.
"""
import numpy as np
import pytest

from test_crooms_gpu import F32_REL_TOL, make_env, run_replay

pytestmark = pytest.mark.gpu

B21 = 1 << 21


def test_crooms_config4_replay_f32_vs_oracle(gpu_device):
    import torch
    kw = {"obs_type": "vector_mdp"}
    acts = np.random.default_rng(21).uniform(-1, 1, (8, B21, 2)).astype(np.float32).astype(np.float64)
    steps = 0
    for t, ref, got, ora, env in run_replay(kw, B21, 2024, acts, torch.float32):
        if t < 0:
            np.testing.assert_array_equal(got[0], np.asarray(ref).astype(np.float32))
            continue
        o = got[0]
        assert o.dtype == np.float32 and o.shape == (B21, 2)
        r64 = np.asarray(ref[0]).astype(np.float64)
        np.testing.assert_array_equal(o, r64.astype(np.float32), err_msg=f"t={t}")
        assert np.all(np.abs(o.astype(np.float64) - r64) <= F32_REL_TOL * np.abs(r64))
        for name, a, b in zip(("rew", "term", "trunc"), ref[1:], got[1:]):
            np.testing.assert_array_equal(np.asarray(a).astype(np.float64), b.astype(np.float64),
                                          err_msg=f"{name} t={t}")
        steps += 1
    assert steps == 8
    agent, goal, vel, el = (x.cpu().numpy() for x in env.get_state())
    np.testing.assert_array_equal(agent, ora.agent)  # the float64 state itself, bit for bit
    np.testing.assert_array_equal(goal + 0.5, ora.goal)
    np.testing.assert_array_equal(el, ora.elapsed)


def test_crooms_config4_philox_rollout_k128_equals_single_steps(gpu_device):
    import torch
    kw = {"obs_type": "vector_mdp"}
    a, b = make_env(kw, B21), make_env(kw, B21)  # philox mode, float32 I/O: the bench configuration
    a.reset(seed=4)
    b.reset(seed=4)
    g = torch.Generator(device=gpu_device)
    g.manual_seed(7)
    acts = torch.rand((128, B21, 2), device=gpu_device, generator=g) * 2 - 1
    ro, rr, rd, rt = a.rollout(acts)
    eps = 0
    for t in range(128):
        o, r, d, tr, _ = b.step(acts[t])
        assert torch.equal(o, ro[t]) and torch.equal(r, rr[t]), f"t={t}"
        assert torch.equal(d, rd[t]) and torch.equal(tr, rt[t]), f"t={t}"
        eps += int((d | tr).sum())
    for x, y in zip(a.get_state(), b.get_state()):
        assert torch.equal(x, y)
    ma, mb = a.metrics(), b.metrics()
    assert ma == mb and ma["episodes"] == eps and ma["env_steps"] == 128 * B21


def test_anttag_config3_shard_philox_vs_oracle(gpu_device):
    from gym_po_amd import AntTagGridEnv
    from oracle.anttag import AntTagOracle
    from oracle.philox import philox_key
    T, seed = 24, 99
    env = AntTagGridEnv(B21)
    ora = AntTagOracle(B21)
    key = philox_key(seed)
    o = env.reset(seed=seed)[0]
    np.testing.assert_array_equal(o.cpu().numpy(), ora.reset(ora.philox_draws(0, key)))
    rng = np.random.default_rng(3)
    eps = 0
    for t in range(T):
        a = rng.integers(0, 5, B21)
        o, r, d, tr, _ = env.step(a)
        ro, rr, rd, rt = ora.step(a, ora.philox_draws(t + 1, key))
        np.testing.assert_array_equal(o.cpu().numpy(), ro, err_msg=f"t={t}")
        np.testing.assert_array_equal(r.cpu().numpy(), rr, err_msg=f"t={t}")
        np.testing.assert_array_equal(d.cpu().numpy(), rd, err_msg=f"t={t}")
        np.testing.assert_array_equal(tr.cpu().numpy(), rt, err_msg=f"t={t}")
        eps += int((rd | rt).sum())
    ant, tgt, el = (x.cpu().numpy() for x in env.get_state())
    np.testing.assert_array_equal(ant, ora.ant)
    np.testing.assert_array_equal(tgt, ora.target)
    np.testing.assert_array_equal(el, ora.elapsed)
    assert eps > 0 and env.metrics()["episodes"] == eps
