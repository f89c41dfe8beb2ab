"""Seed-identical Taxi (rng_mode="numpy", csrc/taxi.hip: taxi_np_kernel up to 1024 envs, the grid-wide taxi_npg_*
launches above) against the reference's fixtures and numpy.

The fixtures were recorded from the reference's TaxiVecEnv (tests/golden/make_golden.py): reset(seed) and every
step's obs / reward / terminated / truncated, the final env state and the final np_random PCG64 state. Here the
device walks the same stream itself -- `integers(L)` for task completions (extended_taxi.py:354-364) and
`multinomial(ns, state_distribution, b).argmax(-1)` for resets (:344-352) -- so the run starts from the seed alone,
with no draws handed over. Launches of several steps (K > 1) and single steps are both exercised, and the
>= 4096-env case checks a whole-batch reset burst (every env truncates at the same step) against numpy itself.
"""
import numpy as np
import pytest

from fixtures import digest, load_case, step_actions

pytestmark = pytest.mark.gpu

FIXTURES = ["taxi_hansen_b64", "taxi_plain_b256", "taxi_ext_hansen", "taxi_2pass_hansen", "taxi_ext_3pass_rew"]


def _kw(kw):
    from gym_po_amd.maps import EXTENDED_TAXI_MAP
    kw = dict(kw)
    if kw.get("map") == "EXTENDED":
        kw["map"] = EXTENDED_TAXI_MAP
    return kw


def _rng6(st):
    s, inc = st["state"]["state"], st["state"]["inc"]
    m = (1 << 64) - 1
    return [s >> 64, s & m, inc >> 64, inc & m, int(st["has_uint32"]), int(st["uinteger"])]


def _run_chunks(env, acts, chunks):
    import torch
    outs = []
    t = 0
    for K in chunks:
        a = torch.as_tensor(acts[t:t + K].astype(np.int32), device=env.device)
        if K == 1:
            o, r, d, tr, _ = env.step(a[0])
            outs.append(tuple(x.cpu().numpy()[None] for x in (o, r, d, tr)))
        else:
            o, r, d, tr = env.rollout(a)
            outs.append(tuple(x.cpu().numpy() for x in (o, r, d, tr)))
        t += K
    return [np.concatenate([o[i] for o in outs]) for i in range(4)]


def _chunks(T):
    out, K, t = [], 1, 0
    while t < T:  # 1, 7, 40, 1, 7, 40, ... steps per launch
        k = min((1, 7, 40)[len(out) % 3], T - t)
        out.append(k)
        t += k
    return out


@pytest.mark.parametrize("name", FIXTURES)
def test_numpy_mode_replays_reference_fixture_from_seed(name, gpu_device):
    from gym_po_amd import TaxiVecEnv
    meta, data = load_case(name)
    B, T = meta["num_envs"], meta["steps"]
    env = TaxiVecEnv(B, **_kw(meta["kwargs"]), rng_mode="numpy", device=gpu_device)
    o0, _ = env.reset(seed=meta["seed"])
    np.testing.assert_array_equal(o0.cpu().numpy().astype(np.int64), data["obs0"])
    acts = step_actions(meta)
    o, r, d, tr = _run_chunks(env, acts, _chunks(T))
    for t in range(T):
        np.testing.assert_array_equal(o[t].astype(np.int64), data["obs"][t].astype(np.int64), err_msg=f"obs t={t}")
        np.testing.assert_array_equal(r[t], data["rew"][t], err_msg=f"rew t={t}")
        np.testing.assert_array_equal(d[t].astype(bool), data["term"][t], err_msg=f"term t={t}")
        np.testing.assert_array_equal(tr[t].astype(bool), data["trunc"][t], err_msg=f"trunc t={t}")
        assert [digest(o[t].astype(np.int64)), digest(r[t]), digest(d[t].astype(bool)),
                digest(tr[t].astype(bool))] == list(data["digests"][t]), f"digest t={t}"
    env.check()
    s, el, nd = (x.cpu().numpy() for x in env.get_state())
    np.testing.assert_array_equal(s, data["final_s"])
    np.testing.assert_array_equal(el, data["final_elapsed"])
    np.testing.assert_array_equal(nd.astype(np.float64), data["final_n_dropoffs"])
    assert _rng6(env.rng_state) == [int(v) for v in data["final_rng_state"]]


@pytest.mark.parametrize("kw,B,T", [({"hansen_obs": True}, 4096, 230),
                                    ({"map": "EXTENDED", "num_passengers": 2, "time_limit": 40}, 4099, 90)])
def test_numpy_mode_matches_numpy_oracle_4096_envs(kw, B, T, gpu_device):
    """Every env truncates at step time_limit + 1 together: a 4096-row multinomial burst (and, with 2 passengers
    and a short limit, task completions that redraw p/d), against the oracle driven by numpy's own Generator."""
    from gym_po_amd import TaxiVecEnv
    from oracle.taxi import TaxiOracle
    env = TaxiVecEnv(B, **_kw(kw), rng_mode="numpy", device=gpu_device)
    ora = TaxiOracle(B, **kw)
    o0, _ = env.reset(seed=5)
    np.testing.assert_array_equal(o0.cpu().numpy().astype(np.int64), np.asarray(ora.reset_seed(5)).astype(np.int64))
    acts = np.random.default_rng(9).integers(0, 5, (T, B))
    o, r, d, tr = _run_chunks(env, acts, [T // 2, T - T // 2])
    eps = 0
    for t in range(T):
        ro, rr, rd, rt = ora.step_seeded(acts[t])
        np.testing.assert_array_equal(o[t].astype(np.int64), np.asarray(ro).astype(np.int64), err_msg=f"obs t={t}")
        np.testing.assert_array_equal(r[t], rr, err_msg=f"rew t={t}")
        np.testing.assert_array_equal(d[t].astype(bool), rd, err_msg=f"term t={t}")
        np.testing.assert_array_equal(tr[t].astype(bool), rt, err_msg=f"trunc t={t}")
        eps += int((rd | rt).sum())
    assert eps >= B  # the burst happened
    assert _rng6(env.rng_state) == _rng6(ora.gen.bit_generator.state)
    m = env.metrics()
    assert m["episodes"] == eps and m["env_steps"] == T * B


def test_numpy_mode_rng_state_roundtrip(gpu_device):
    """rng_state can be read and written like np_random's bit_generator.state; a written state is the one used."""
    import torch
    from gym_po_amd import TaxiVecEnv
    B = 64
    e1 = TaxiVecEnv(B, rng_mode="numpy", device=gpu_device)
    e2 = TaxiVecEnv(B, rng_mode="numpy", device=gpu_device)
    e1.reset(seed=3)
    acts = torch.randint(0, 5, (230, B), device=gpu_device, dtype=torch.int32)
    e1.rollout(acts[:100])
    e2.reset(seed=99)
    e2.set_state(*e1.get_state())
    e2.rng_state = e1.rng_state
    a = e1.rollout(acts[100:])
    b = e2.rollout(acts[100:])
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert e1.rng_state == e2.rng_state


@pytest.mark.parametrize("name", ["taxi_hansen_b64", "taxi_ext_3pass_rew"])
def test_numpy_mode_grid_wide_path_on_fixtures(name, gpu_device):
    """The grid-wide form (pass 1 / draws / pass 2 launches per step, taxi.hip taxi_npg_*) forced on the fixtures'
    small batches (one partial tile), from the seed, as test_numpy_mode_replays_reference_fixture_from_seed."""
    from gym_po_amd._lib import debug_knobs
    with debug_knobs(taxi_npg_min=0):
        test_numpy_mode_replays_reference_fixture_from_seed(name, gpu_device)


@pytest.mark.parametrize("one_hot", [False, True])
def test_numpy_mode_grid_wide_65536_envs_burst(one_hot, gpu_device):
    """65,536 envs (64 tiles on the grid-wide path): every env truncates together at step 16 (a 65,536-row
    multinomial burst), task completions redraw p / d, against the oracle on numpy's Generator; Hansen obs as
    int32 or as one-hot uint8 rows (checked as argmax + row sums on the device)."""
    import torch
    from gym_po_amd import HansenTaxiVecEnv
    from oracle.taxi import TaxiOracle
    B, T, kw = 65536, 24, {"time_limit": 15}
    env = HansenTaxiVecEnv(B, **kw, rng_mode="numpy", one_hot=one_hot, device=gpu_device)
    ora = TaxiOracle(B, hansen_obs=True, **kw)

    def idx(o):
        if not one_hot:
            return o.cpu().numpy().astype(np.int64)
        assert bool((o.sum(-1) == 1).all())
        return o.argmax(-1).cpu().numpy().astype(np.int64)

    o0, _ = env.reset(seed=21)
    np.testing.assert_array_equal(idx(o0), np.asarray(ora.reset_seed(21)).astype(np.int64))
    acts = np.random.default_rng(4).integers(0, 5, (T, B))
    eps, t = 0, 0
    for K in (1, 13, 10):
        o, r, d, tr = env.rollout(torch.as_tensor(acts[t:t + K].astype(np.int32), device=gpu_device))
        for j in range(K):
            ro, rr, rd, rt = ora.step_seeded(acts[t + j])
            np.testing.assert_array_equal(idx(o[j]), np.asarray(ro).astype(np.int64), err_msg=f"obs t={t + j}")
            np.testing.assert_array_equal(r[j].cpu().numpy(), rr, err_msg=f"rew t={t + j}")
            np.testing.assert_array_equal(d[j].cpu().numpy().astype(bool), rd, err_msg=f"term t={t + j}")
            np.testing.assert_array_equal(tr[j].cpu().numpy().astype(bool), rt, err_msg=f"trunc t={t + j}")
            eps += int((rd | rt).sum())
        t += K
    assert eps >= B
    env.check()
    assert _rng6(env.rng_state) == _rng6(ora.gen.bit_generator.state)
    m = env.metrics()
    assert m["episodes"] == eps and m["env_steps"] == T * B
