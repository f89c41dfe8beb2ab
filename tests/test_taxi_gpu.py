"""GPU parity of the Taxi backend (csrc/taxi.hip) against the reference fixtures and the oracle.

Replay mode must reproduce the reference bit-for-bit: the oracle (pinned to the reference by
tests/test_oracle_golden.py) is driven by the reference's own numpy stream, and the states it
lands in after every reset / task completion are handed to the GPU as replay draws. Everything
else (moves, walls, pickup/dropoff, rewards, done/truncated, observations) is the kernel's own.
Philox mode is checked in law: the reset-state histogram against the exact argmax-multinomial law
and against 2M reference resets, the passenger/destination pairs against uniform-over-p!=d.
"""
import numpy as np
import pytest

from fixtures import digest, load_case, load_index, step_actions
from oracle.taxi import TaxiOracle

pytestmark = pytest.mark.gpu

CASES = {k: v for k, v in load_index()["cases"].items() if v["kind"] == "taxi"}


def _map(kw):
    from gym_po_amd.maps import EXTENDED_TAXI_MAP, TAXI_MAP
    kw = dict(kw)
    if kw.get("map") == "EXTENDED":
        kw["map"] = EXTENDED_TAXI_MAP
    elif kw.get("map") in (None, "TAXI"):
        kw["map"] = TAXI_MAP
    return kw


def make_env(kw, B, **extra):
    from gym_po_amd import TaxiVecEnv
    return TaxiVecEnv(B, **_map(kw), **extra)


def make_oracle(kw, B):
    return TaxiOracle(B, **kw)


def _np(x):
    return x.cpu().numpy()


def run_replay(kw, B, seed, acts, env=None, check=None):
    """Drive oracle (reference numpy stream) and GPU (replay) side by side; yield per-step outputs."""
    ora = make_oracle(kw, B)
    env = env or make_env(kw, B, rng_mode="replay")
    o_ref = ora.reset_seed(seed)
    env.set_replay(reset_states=ora.s.astype(np.int32))
    o, _ = env.reset()
    o_ref = np.asarray(o_ref).astype(np.int64)
    if env.one_hot:
        o_ref = np.eye(env.no, dtype=np.int64)[o_ref]
    np.testing.assert_array_equal(_np(o).astype(np.int64), o_ref)
    lpl = ora.nlocs * (ora.nlocs + 1)
    for t in range(acts.shape[0]):
        ro, rr, rd, rt = ora.step_seeded(acts[t])
        s_after = ora.s.astype(np.int32)
        env.set_replay(reset_states=s_after, pd=(s_after % lpl).astype(np.int32))
        o, r, d, tr, _ = env.step(acts[t])
        yield t, (np.asarray(ro), rr, rd, rt), (_np(o), _np(r), _np(d), _np(tr)), ora, env


@pytest.mark.parametrize("name", sorted(CASES))
def test_replay_bit_exact_vs_reference_fixture(name, gpu_device):
    meta, data = load_case(name)
    acts = step_actions(meta)
    for t, ref, got, ora, env in run_replay(meta["kwargs"], meta["num_envs"], meta["seed"], acts):
        o, r, d, tr = got
        np.testing.assert_array_equal(o.astype(np.int64), data["obs"][t].astype(np.int64), err_msg=f"t={t}")
        np.testing.assert_array_equal(r, data["rew"][t], err_msg=f"t={t}")
        np.testing.assert_array_equal(d.astype(bool), data["term"][t], err_msg=f"t={t}")
        np.testing.assert_array_equal(tr.astype(bool), data["trunc"][t], err_msg=f"t={t}")
        assert [digest(o.astype(np.int64)), digest(r), digest(d.astype(bool)), digest(tr.astype(bool))] == \
            list(data["digests"][t]), f"digest t={t}"
    s, el, nd = (_np(x) for x in env.get_state())
    np.testing.assert_array_equal(s, data["final_s"])
    np.testing.assert_array_equal(el, data["final_elapsed"])
    np.testing.assert_array_equal(nd.astype(np.float64), data["final_n_dropoffs"])


@pytest.mark.parametrize("kw,B", [({"hansen_obs": True}, 65536 + 37),
                                  ({"map": "EXTENDED", "num_passengers": 3, "time_limit": 150}, 20000 + 3),
                                  ({"num_passengers": 2, "time_limit": 60}, 4099)])
def test_replay_bit_exact_vs_oracle_ragged(kw, B, gpu_device):
    rng = np.random.default_rng(7)
    acts = rng.integers(0, 5, (250, B))
    eps = 0
    for t, ref, got, ora, env in run_replay(kw, B, 11, acts):
        for name, a, b in zip(("obs", "rew", "term", "trunc"), ref, got):
            np.testing.assert_array_equal(np.asarray(a).astype(np.float64), b.astype(np.float64),
                                          err_msg=f"{name} t={t}")
        eps += int((ref[2] | ref[3]).sum())
    m = env.metrics()
    assert m["episodes"] == eps and m["env_steps"] == 250 * B


def test_negative_actions_index_like_numpy(gpu_device):
    """ACTIONS_YX[a] wraps a in -5..-1; -1 moves (0,0) but is not a pickup/dropoff (a == 4 test)."""
    B = 512
    rng = np.random.default_rng(3)
    acts = rng.integers(-5, 5, (60, B))
    for t, ref, got, ora, env in run_replay({"hansen_obs": True, "num_passengers": 2}, B, 5, acts):
        for name, a, b in zip(("obs", "rew", "term", "trunc"), ref, got):
            np.testing.assert_array_equal(np.asarray(a).astype(np.float64), b.astype(np.float64),
                                          err_msg=f"{name} t={t}")


@pytest.mark.parametrize("kw", [{"hansen_obs": True}, {}, {"map": "EXTENDED", "hansen_obs": True}])
def test_one_hot_rows_match_scalar_obs(kw, gpu_device):
    import torch
    for B in (4096, 1000 + 3):
        a = make_env(kw, B, rng_mode="philox")
        b = make_env(kw, B, rng_mode="philox", one_hot=True)
        oa, _ = a.reset(seed=9)
        ob, _ = b.reset(seed=9)
        eye = torch.eye(a.no, dtype=torch.uint8, device=oa.device)
        assert torch.equal(eye[oa.long()], ob)
        acts = torch.randint(0, 5, (8, B), dtype=torch.int32, device=oa.device)
        for t in range(3):
            oa, ra, da, ta, _ = a.step(acts[t])
            ob, rb, db, tb, _ = b.step(acts[t])
            assert torch.equal(eye[oa.long()], ob) and torch.equal(ra, rb) and torch.equal(da, db)
        # fused K-step rollout into [K,B,n_obs]
        oa, ra, _, _ = a.rollout(acts[3:])
        ob, rb, _, _ = b.rollout(acts[3:])
        assert torch.equal(eye[oa.long()], ob) and torch.equal(ra, rb)


def test_one_hot_odd_width_byte_path(gpu_device):
    """A custom 1x3 map with two locations: n_obs = 18 (not a multiple of 4) -> byte chunks."""
    import torch
    kw = {"map": ("R G",)}
    for B in (257, 1024):
        a = make_env(kw, B, rng_mode="philox")
        b = make_env(kw, B, rng_mode="philox", one_hot=True)
        assert b.no == 18
        oa, _ = a.reset(seed=1)
        ob, _ = b.reset(seed=1)
        eye = torch.eye(a.no, dtype=torch.uint8, device=oa.device)
        assert torch.equal(eye[oa.long()], ob)
        acts = torch.randint(0, 5, (6, B), dtype=torch.int32, device=oa.device)
        oa, *_ = a.rollout(acts)
        ob, *_ = b.rollout(acts)
        assert torch.equal(eye[oa.long()], ob)


def test_philox_rollout_equals_single_steps(gpu_device):
    import torch
    B, K = 5000, 37
    a = make_env({"num_passengers": 2, "time_limit": 30}, B)
    b = make_env({"num_passengers": 2, "time_limit": 30}, B)
    a.reset(seed=4)
    b.reset(seed=4)
    acts = torch.randint(0, 5, (K, B), dtype=torch.int32, device=gpu_device)
    ro, rr, rd, rt = a.rollout(acts)
    for t in range(K):
        o, r, d, tr, _ = b.step(acts[t])
        assert torch.equal(o, ro[t]) and torch.equal(r, rr[t]) and torch.equal(d, rd[t]) and torch.equal(tr, rt[t])
    for x, y in zip(a.get_state(), b.get_state()):
        assert torch.equal(x, y)


def _chi2_p(counts, probs):
    from scipy.stats import chisquare
    n = counts.sum()
    return chisquare(counts, probs * n).pvalue


def test_philox_reset_law(gpu_device):
    """Start states follow the exact argmax-multinomial law, and agree with 2M reference resets."""
    B = 1 << 21
    env = make_env({}, B)
    env.reset(seed=2024)
    s = _np(env.get_state()[0])
    law = env.reset_distribution
    idx = np.searchsorted(env.valid_states, s)
    assert np.array_equal(env.valid_states[idx], s), "reset into an invalid state"
    counts = np.bincount(idx, minlength=len(law)).astype(np.float64)
    assert _chi2_p(counts, law) > 1e-4
    meta = load_index()["taxi_reset_hist"]
    ref = np.load(f"{__import__('fixtures').GOLDEN_DIR}/{meta['file']}", allow_pickle=False)
    ref_counts = ref["TAXI"].astype(np.float64)[env.valid_states]
    # two-sample homogeneity (GPU philox draws vs reference numpy draws)
    from scipy.stats import chi2_contingency
    assert chi2_contingency(np.stack([counts, ref_counts]))[1] > 1e-4


def test_philox_passenger_destination_law(gpu_device):
    """Task completion draws p uniform and d uniform over the other locations; taxi cell kept."""
    import torch
    B = 1 << 20
    env = make_env({"num_passengers": 2}, B)
    env.reset(seed=5)
    L = env.nlocs
    # every env: passenger in taxi (p = L), destination d, taxi parked on loc[d]
    rng = np.random.default_rng(0)
    d = rng.integers(0, L, B)
    r, c = env.np_locs[d, 0], env.np_locs[d, 1]
    s = env.encode(r, c, L, d)
    env.set_state(s=s, elapsed=np.zeros(B, np.int32), n_dropoffs=np.zeros(B, np.int32))
    o, rew, term, trunc, _ = env.step(torch.full((B,), 4, dtype=torch.int32, device=gpu_device))
    assert bool((rew == env.GOAL_MOVE).all()) and not bool(term.any())
    s2 = _np(env.get_state()[0])
    r2, c2, p2, d2 = env.decode(s2)
    np.testing.assert_array_equal(r2, r)
    np.testing.assert_array_equal(c2, c)
    assert (p2 != d2).all() and (p2 < L).all()
    counts = np.bincount(p2 * L + d2, minlength=L * L).reshape(L, L)
    off = counts[~np.eye(L, dtype=bool)].astype(np.float64)
    assert _chi2_p(off, np.full(off.size, 1.0 / off.size)) > 1e-4
    assert int(_np(env.get_state()[2]).min()) == 1


@pytest.mark.parametrize("name", ["taxi_hansen_b64", "taxi_ext_hansen"])
def test_one_hot_replay_bit_exact_vs_reference_fixture(name, gpu_device):
    """configs[2]'s one-hot encoding pinned to the reference: row t of the one-hot obs == eye(n_obs)[the
    reference's Hansen obs] at every step (extended_taxi.py:366-372 gives the index; one-hot is the build's
    encoding of it)."""
    meta, data = load_case(name)
    kw = dict(meta["kwargs"])
    assert kw.get("hansen_obs")
    acts = step_actions(meta)
    env = make_env(kw, meta["num_envs"], rng_mode="replay", one_hot=True)
    eye = np.eye(env.no, dtype=np.uint8)
    for t, ref, got, ora, env in run_replay(kw, meta["num_envs"], meta["seed"], acts, env=env):
        o, r, d, tr = got
        np.testing.assert_array_equal(o, eye[data["obs"][t].astype(np.int64)], err_msg=f"t={t}")
        np.testing.assert_array_equal(r, data["rew"][t], err_msg=f"t={t}")
        np.testing.assert_array_equal(d.astype(bool), data["term"][t], err_msg=f"t={t}")
        np.testing.assert_array_equal(tr.astype(bool), data["trunc"][t], err_msg=f"t={t}")


def test_one_hot_4m_envs_rollout_properties(gpu_device):
    """configs[2] at full size (2^22 envs, one-hot uint8[B, 320], the bench's 4-step launches): every row is
    one-hot, its index equals the scalar Hansen obs of a same-seed scalar env, and the start states follow
    the exact argmax-multinomial reset law (chi-square)."""
    import torch
    from gym_po_amd import HansenTaxiVecEnv
    B, K = 1 << 22, 4
    a = HansenTaxiVecEnv(B, device=gpu_device, rng_mode="philox")
    b = HansenTaxiVecEnv(B, device=gpu_device, rng_mode="philox", one_hot=True)
    oa, _ = a.reset(seed=21)
    ob, _ = b.reset(seed=21)
    assert ob.shape == (B, 320) and ob.dtype == torch.uint8
    assert torch.equal(ob.sum(-1, dtype=torch.int32), torch.ones(B, dtype=torch.int32, device=gpu_device))
    assert torch.equal(ob.argmax(-1).to(torch.int32), oa.to(torch.int32))
    s = _np(b.get_state()[0])
    law = b.reset_distribution
    idx = np.searchsorted(b.valid_states, s)
    assert np.array_equal(b.valid_states[idx], s), "reset into an invalid state"
    assert _chi2_p(np.bincount(idx, minlength=len(law)).astype(np.float64), law) > 1e-4
    acts = torch.randint(0, 5, (K, B), dtype=torch.int32, device=gpu_device)
    oa, ra, da, ta = a.rollout(acts)
    ob, rb, db, tb = b.rollout(acts)
    for k in range(K):
        assert torch.equal(ob[k].sum(-1, dtype=torch.int32), torch.ones(B, dtype=torch.int32, device=gpu_device))
        assert torch.equal(ob[k].argmax(-1).to(torch.int32), oa[k].to(torch.int32))
    assert torch.equal(ra, rb) and torch.equal(da, db) and torch.equal(ta, tb)
    assert int(oa.min()) >= 0 and int(oa.max()) < 320
