"""Debug: step a fixture case on the GPU and the oracle side by side; report RNG divergence."""
import os, sys
sys.path[:0] = ["tests", "tests/golden", "gym-po-taxi_amd", "."]
import numpy as np
from fixtures import load_case, step_actions
from test_grid_gpu import make_env, make_oracle, reset_obs, np_obs
names = sys.argv[1:] or ["fr_goal_mdp_z2_randgoal"]
for name in names:
    meta, data = load_case(name)
    env = make_env(meta)
    ora = make_oracle(meta)
    acts = step_actions(meta)
    o0 = np_obs(reset_obs(env, meta["seed"]))
    ora.reset_seed(meta["seed"])
    def st(s):
        return (hex(s["state"]["state"])[-8:], s["has_uint32"], s["uinteger"])
    print(name, "obs0 eq", np.array_equal(o0, data["obs0"]), st(env.rng_state), st(ora.gen.bit_generator.state))
    for t in range(4):
        o, r, d, tr, _ = env.step(acts[t])
        _, _, d2, tr2 = ora.step_seeded(np.asarray(acts[t]))
        print(t, "obs eq", np.array_equal(np_obs(o), data["obs"][t]), "resets", int((d2 | tr2).sum()),
              "dev", st(env.rng_state), "ora", st(ora.gen.bit_generator.state))
