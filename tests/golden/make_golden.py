"""Generate golden fixtures by running the REFERENCE (read-only, annotation-repaired in memory,
stubbed gymnasium) in the build container. Committed outputs: tests/golden/*.npz + index.json.

    python tests/golden/make_golden.py            # all cases
    python tests/golden/make_golden.py fr_        # cases whose name starts with a prefix

Every case: construct the reference env with the recorded kwargs, reset(seed=seed), then step
with actions regenerated from `default_rng(action_seed)` (fixtures.step_actions). Recorded per
step: obs, reward, terminated, truncated (full arrays for small cases, per-step digests for large
ones), plus the final internal state and the final PCG64 state of the env's Generator.
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refload  # noqa: E402
from fixtures import INDEX, digest, step_actions  # noqa: E402

FR = "fourrooms"
RO = "rooms"
TX = "taxi"
CR = "crooms"

# name: (kind, ctor kwargs, num_envs, steps, seed, action_seed, full)
CASES = {
    # ---- Multistory FourRooms (msrooms.py) ----
    "fr_hansen_b256": (FR, dict(grid_z=1, obs_type="hansen"), 256, 600, 0, 1, True),
    "fr_hansen_b4096": (FR, dict(grid_z=1, obs_type="hansen"), 4096, 600, 1, 2, False),
    "fr_hansen_tl20": (FR, dict(grid_z=1, obs_type="hansen", time_limit=20), 512, 200, 7, 3, True),
    "fr_hansen8_ordinal": (FR, dict(grid_z=1, obs_type="hansen8", action_type="ordinal"), 128, 300, 3, 4, True),
    "fr_vgh_z3_randgoal": (FR, dict(grid_z=3, obs_type="vector_goal_hansen", goal_xyz=None, time_limit=60),
                           128, 300, 5, 5, True),
    "fr_mdp_z2": (FR, dict(grid_z=2, obs_type="mdp", time_limit=80), 64, 300, 11, 6, True),
    "fr_goal_mdp_z2_randgoal": (FR, dict(grid_z=2, obs_type="goal_mdp", goal_xyz=None, time_limit=80),
                                64, 300, 12, 7, True),
    "fr_vector_goal_mdp_z2": (FR, dict(grid_z=2, obs_type="vector_goal_mdp", time_limit=50), 64, 200, 13, 8, True),
    "fr_vector_hansen8_z2": (FR, dict(grid_z=2, obs_type="vector_hansen8", action_type="ordinal", time_limit=40),
                             64, 200, 14, 9, True),
    "fr_rewards_p0": (FR, dict(grid_z=1, obs_type="hansen", action_failure_probability=0.0, step_reward=-0.01,
                               wall_reward=-0.1, goal_reward=2.0, time_limit=30), 256, 200, 15, 10, True),
    # ---- ROOMS (rooms.py) ----
    "rooms_4_hansen_card": (RO, dict(layout="4", obs_type="hansen", action_type="cardinal"), 256, 600, 0, 11, True),
    "rooms_4_hansen8": (RO, dict(layout="4", obs_type="hansen8", time_limit=100), 128, 300, 1, 12, True),
    "rooms_4_grid3": (RO, dict(layout="4", obs_type="grid", time_limit=100), 128, 300, 2, 13, True),
    "rooms_8b_grid5": (RO, dict(layout="8b", obs_type="grid", obs_n=5, time_limit=100), 64, 300, 3, 14, True),
    "rooms_8_hansen": (RO, dict(layout="8", obs_type="hansen", time_limit=100), 64, 300, 24, 25, True),
    "rooms_10b_hansen": (RO, dict(layout="10b", obs_type="hansen", time_limit=120), 64, 300, 21, 22, True),
    "rooms_16b_vhansen_randgoal": (RO, dict(layout="16b", obs_type="vector_hansen", goal_xy=None, time_limit=150),
                                   64, 300, 23, 24, True),
    "rooms_16_vgh8": (RO, dict(layout="16", obs_type="vector_goal_hansen8", time_limit=100), 64, 300, 4, 15, True),
    "rooms_4b_room": (RO, dict(layout="4b", obs_type="room", time_limit=100), 64, 300, 5, 16, True),
    "rooms_10_goal_room_randgoal": (RO, dict(layout="10", obs_type="goal_room", goal_xy=None, time_limit=100),
                                    64, 300, 6, 17, True),
    "rooms_2_goal_mdp_randgoal": (RO, dict(layout="2", obs_type="goal_mdp", goal_xy=None, time_limit=60),
                                  64, 300, 7, 18, True),
    "rooms_4_vector_goal_mdp": (RO, dict(layout="4", obs_type="vector_goal_mdp", time_limit=100), 64, 300, 8, 19, True),
    "rooms_1_vector_hansen_rew": (RO, dict(layout="1", obs_type="vector_hansen", step_reward=-1.0, wall_reward=-5.0,
                                           goal_reward=10.0, action_failure_probability=1.0 / 3, time_limit=40),
                                  64, 300, 9, 20, True),
    "rooms_32_mdp": (RO, dict(layout="32", obs_type="mdp", time_limit=100), 64, 300, 10, 21, True),
    "rooms_32b_hansen": (RO, dict(layout="32b", obs_type="hansen", time_limit=100), 64, 300, 11, 22, True),
    "rooms_4_hansen_b4096": (RO, dict(layout="4", obs_type="hansen", action_type="cardinal"), 4096, 600, 12, 23,
                             False),
    # ---- Taxi (extended_taxi.py) ----
    "taxi_hansen_b64": (TX, dict(hansen_obs=True), 64, 1000, 0, 31, True),
    "taxi_plain_b256": (TX, dict(), 256, 500, 1, 32, True),
    "taxi_ext_hansen": (TX, dict(hansen_obs=True, map="EXTENDED"), 128, 500, 2, 33, True),
    "taxi_2pass_hansen": (TX, dict(hansen_obs=True, num_passengers=2, time_limit=400), 128, 800, 3, 34, True),
    "taxi_ext_3pass_rew": (TX, dict(map="EXTENDED", num_passengers=3, time_limit=300, reward_goal=2.0,
                                    reward_bad=-1.0, reward_any=-0.1), 64, 700, 4, 35, True),
    # ---- C-ROOMS (crooms.py), float64 ----
    "crooms_yx_vmdp": (CR, dict(obs_type="vector_mdp"), 64, 400, 0, 41, True),
    "crooms_vel_vgmdp_randgoal": (CR, dict(obs_type="vector_goal_mdp", use_velocity=True, goal_xy=None,
                                           time_limit=100), 64, 300, 1, 42, True),
    "crooms_card_hansen": (CR, dict(obs_type="hansen", action_type="cardinal", time_limit=100), 64, 300, 2, 43, True),
    "crooms_8_grid": (CR, dict(layout="8", obs_type="grid", action_power=1.5, time_limit=100), 64, 300, 3, 44, True),
}


def make_env(m, kind, kw, B):
    kw = dict(kw)
    if kind == FR:
        return m["msrooms"].MultistoryFourRoomsEnv(B, **kw)
    if kind == RO:
        return m["rooms"].RoomsEnv(B, **kw)
    if kind == TX:
        if kw.get("map") == "EXTENDED":
            kw["map"] = m["extended_taxi"].EXTENDED_TAXI_MAP
        return m["extended_taxi"].TaxiVecEnv(B, **kw)
    if kind == CR:
        return m["crooms"].CRoomsEnv(B, **kw)
    raise ValueError(kind)


def num_actions(env, kind):
    if kind == CR and not hasattr(env.single_action_space, "n"):
        return None
    return int(env.single_action_space.n)


def final_state(env, kind):
    out = {}
    if kind == FR:
        out.update(agent=env.agent_zyx, goal=env.goal_zyx, elapsed=env.elapsed)
        gen = env.np_random
    elif kind == RO:
        out.update(agent=env.agent_yx, goal=env.goal_yx, elapsed=env.elapsed)
        gen = env.np_random
    elif kind == TX:
        out.update(s=env.s, elapsed=env.elapsed, n_dropoffs=env.n_dropoffs_completed)
        gen = env.np_random
    else:
        out.update(agent=env.agent_yx, goal=env.goal_yx, elapsed=env.elapsed, velocity=env.agent_yx_velocity)
        gen = env.rng
    st = gen.bit_generator.state
    out["rng_state"] = np.array([st["state"]["state"] >> 64, st["state"]["state"] & ((1 << 64) - 1),
                                 st["state"]["inc"] >> 64, st["state"]["inc"] & ((1 << 64) - 1),
                                 st["has_uint32"], st["uinteger"]], dtype=np.uint64)
    return out


def obs_store_dtype(obs):
    if obs.dtype.kind == "f":
        if np.all(obs == np.round(obs)):
            return np.int32
        return np.float64
    return np.int32


def run_case(m, name, spec):
    kind, kw, B, T, seed, aseed, full = spec
    env = make_env(m, kind, kw, B)
    meta = dict(kind=kind, kwargs=kw, num_envs=B, steps=T, seed=seed, action_seed=aseed, full=full,
                numpy=np.__version__, file=f"{name}.npz")
    na = num_actions(env, kind)
    if na is None:
        meta["action_kind"] = "box2"
    else:
        meta["num_actions"] = na
    acts = step_actions(meta)
    r0 = env.reset(seed=seed)
    obs0 = np.array(r0[0] if isinstance(r0, tuple) else r0)  # copy: C-ROOMS vector_mdp aliases state
    obs_l, rew_l, term_l, trunc_l = [], [], [], []
    dig = np.zeros((T, 4), dtype=np.uint64)
    for t in range(T):
        o, r, d, tr, _ = env.step(acts[t])
        o = np.asarray(o)
        dig[t] = [digest(o.astype(np.float64) if o.dtype.kind == "f" else o), digest(r), digest(d), digest(tr)]
        if full:
            obs_l.append(o.copy())
            rew_l.append(r.copy())
            term_l.append(d.copy())
            trunc_l.append(tr.copy())
    arrays = dict(obs0=np.asarray(obs0), digests=dig)
    if full:
        obs = np.stack(obs_l)
        arrays["obs"] = obs.astype(obs_store_dtype(obs))
        arrays["rew"] = np.stack(rew_l)
        arrays["term"] = np.stack(term_l)
        arrays["trunc"] = np.stack(trunc_l)
    for k, v in final_state(env, kind).items():
        arrays["final_" + k] = np.asarray(v)
    np.savez_compressed(os.path.join(HERE, meta["file"]), **arrays)
    return meta


def taxi_reset_histogram(m, n_samples=2_000_000, seed=123):
    """Empirical start-state histogram of TaxiVecEnv._reset_mask (multinomial argmax)."""
    out = {}
    for mapname in ("TAXI", "EXTENDED"):
        kw = {} if mapname == "TAXI" else {"map": "EXTENDED"}
        env = make_env(m, TX, kw, 1)
        gen = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        counts = np.zeros(env.ns, dtype=np.int64)
        left = n_samples
        while left:
            b = min(left, 50_000)
            s = gen.multinomial(env.ns, env.state_distribution, b).argmax(-1)
            counts += np.bincount(s, minlength=env.ns)
            left -= b
        out[mapname] = counts
    np.savez_compressed(os.path.join(HERE, "taxi_reset_hist.npz"), **out)
    return dict(file="taxi_reset_hist.npz", n_samples=n_samples, seed=seed, numpy=np.__version__)


def main():
    import json
    prefix = sys.argv[1] if len(sys.argv) > 1 else ""
    m = refload.load()
    index = {"cases": {}}
    if os.path.exists(INDEX):
        with open(INDEX) as f:
            index = json.load(f)
    for name, spec in CASES.items():
        if not name.startswith(prefix):
            continue
        t0 = time.time()
        index["cases"][name] = run_case(m, name, spec)
        print(f"{name}: {time.time() - t0:.1f}s", flush=True)
    if prefix in ("", "taxi_reset_hist"):
        t0 = time.time()
        index["taxi_reset_hist"] = taxi_reset_histogram(m)
        print(f"taxi_reset_hist: {time.time() - t0:.1f}s")
    index["generator"] = "tests/golden/make_golden.py (reference imported via tests/golden/refload.py)"
    with open(INDEX, "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
