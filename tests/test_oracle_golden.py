"""Pin the oracle (CPU restatement) against golden fixtures produced by the reference itself.

CPU-only. Every fixture case is replayed through the oracle with the same seed and actions and
must agree bit-for-bit on every step's obs / reward / terminated / truncated, on the final env
state and on the final PCG64 state (so the oracle consumes the numpy stream exactly as the
reference does).
"""
import numpy as np
import pytest

from fixtures import digest, load_case, load_index, step_actions
from oracle import gridworld

CASES = load_index()["cases"]


def _oracle_for(meta):
    kw = dict(meta["kwargs"])
    B = meta["num_envs"]
    if meta["kind"] == "fourrooms":
        if "goal_xyz" in kw and kw["goal_xyz"] is not None:
            kw["goal_xyz"] = tuple(kw["goal_xyz"])
        return gridworld.FourRoomsOracle(B, **kw)
    if meta["kind"] == "rooms":
        return gridworld.RoomsOracle(B, **kw)
    if meta["kind"] == "taxi":
        from oracle import taxi
        return taxi.TaxiOracle(B, **kw)
    if meta["kind"] == "crooms":
        from oracle import crooms
        return crooms.CRoomsOracle(B, **kw)
    raise ValueError(meta["kind"])


def _rng_state(gen):
    st = gen.bit_generator.state
    s, inc = st["state"]["state"], st["state"]["inc"]
    m = (1 << 64) - 1
    return np.array([s >> 64, s & m, inc >> 64, inc & m, st["has_uint32"], st["uinteger"]], dtype=np.uint64)


def _check_obs(o, ref):
    o = np.asarray(o)
    if ref.dtype.kind == "f":
        np.testing.assert_array_equal(o, ref)
    else:
        np.testing.assert_array_equal(o.astype(np.float64), ref.astype(np.float64))


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_reference_fixture(name):
    meta, data = load_case(name)
    env = _oracle_for(meta)
    acts = step_actions(meta)
    obs0 = env.reset_seed(meta["seed"])
    _check_obs(obs0, data["obs0"])
    for t in range(meta["steps"]):
        o, r, d, tr = env.step_seeded(acts[t])
        o = np.asarray(o)
        if meta["full"]:
            _check_obs(o, data["obs"][t])
            np.testing.assert_array_equal(r, data["rew"][t])
            np.testing.assert_array_equal(d, data["term"][t])
            np.testing.assert_array_equal(tr, data["trunc"][t])
        dg = [digest(o.astype(np.float64) if o.dtype.kind == "f" else o), digest(r), digest(d), digest(tr)]
        assert dg == list(data["digests"][t]), f"step {t} digest mismatch"
    for k in data.files:
        if k.startswith("final_") and k != "final_rng_state":
            np.testing.assert_array_equal(np.asarray(getattr(env, env.STATE_ALIASES[k[6:]])), data[k], err_msg=k)
    np.testing.assert_array_equal(_rng_state(env.gen), data["final_rng_state"])
