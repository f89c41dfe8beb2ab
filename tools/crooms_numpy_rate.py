"""Throughput of C-ROOMS exact mode (rng_mode='numpy': one workgroup up to 1,024 envs (XG_MIN_ENVS), the
multi-workgroup draw calls above) beside philox mode, same config.

Usage (GPU box): python tools/crooms_numpy_rate.py [B ...] -> one JSON line per (mode, B). XG_MIN=n: the
one-workgroup kernel only up to n envs (gp_debug_set xg_min_envs; crossover measurements). GP_KNOBS="k=v,...":
other library knobs (recorded in the line). MODES=numpy: one mode.
"""
import json
import os
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # as bench.py
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gym-po-taxi_amd"))
import torch  # noqa: E402

from gym_po_amd import CRoomsEnv  # noqa: E402


def rate(mode, B, K=None, reps=3):
    K = K or (50 if B <= 65536 else 8)
    from gym_po_amd._lib import debug_knobs
    knobs = {"xg_min_envs": int(os.environ["XG_MIN"])} if os.environ.get("XG_MIN") else {}
    knobs.update((kv.split("=")[0], int(kv.split("=")[1])) for kv in os.environ.get("GP_KNOBS", "").split(",") if kv)
    with debug_knobs(**knobs):
        env = CRoomsEnv(B, obs_type="vector_mdp", rng_mode=mode)
    env.reset(seed=0)
    a = torch.rand((K, B, 2), device=env.device) * 2 - 1
    out = env._alloc_outputs(K)  # the same buffers every call (round 6: the hipGraph replay is keyed by them)
    for _ in range(3):  # (by default the graph is captured on the 2nd identical call)
        env.rollout(a, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        env.rollout(a, out=out)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"mode": mode, "num_envs": B, "steps": K * reps, "us_per_step": dt / (K * reps) * 1e6,
            "env_steps_per_s": B * K * reps / dt, "knobs": knobs}


if __name__ == "__main__":
    for B in [int(x) for x in sys.argv[1:]] or (1024, 4096, 65536, 1 << 21):
        for mode in os.environ.get("MODES", "numpy philox").split():
            print(json.dumps(rate(mode, B)), flush=True)
