"""Throughput of seed-identical Taxi (rng_mode='numpy', csrc/taxi.hip) beside philox mode, same config
(BASELINE configs[2]: HansenTaxiVecEnv(one_hot=True), uniform random actions).

Usage (GPU box): python tools/taxi_numpy_rate.py [B ...] -> one JSON line per (mode, B). MODES="numpy": one mode;
NPG_MIN=n: the one-workgroup kernel only up to n envs (gp_debug_set taxi_npg_min; crossover measurements).
"""
import json
import os
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # as bench.py
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gym-po-taxi_amd"))
import torch  # noqa: E402

from gym_po_amd import HansenTaxiVecEnv  # noqa: E402


def rate(mode, B, K=None, reps=3):
    K = K or (50 if B <= 65536 else 10)
    from gym_po_amd._lib import debug_knobs
    knobs = {"taxi_npg_min": int(os.environ["NPG_MIN"])} if os.environ.get("NPG_MIN") else {}
    with debug_knobs(**knobs):
        env = HansenTaxiVecEnv(B, rng_mode=mode, one_hot=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    env.reset(seed=0)
    torch.cuda.synchronize()
    reset_s = time.perf_counter() - t0  # every env draws a start state: B multinomial rows (numpy mode)
    a = torch.randint(0, 5, (K, B), device=env.device, dtype=torch.int32)
    env.rollout(a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        env.rollout(a)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    m = env.metrics()
    return {"mode": mode, "num_envs": B, "steps": K * reps, "us_per_step": dt / (K * reps) * 1e6,
            "env_steps_per_s": B * K * reps / dt, "episodes_so_far": m["episodes"], "reset_s": reset_s,
            "path": ("grid-wide" if B > knobs.get("taxi_npg_min", 4096) else "one workgroup") if mode == "numpy" else "-"}


if __name__ == "__main__":
    for B in [int(x) for x in sys.argv[1:]] or (64, 4096, 65536, 1 << 22):
        for mode in os.environ.get("MODES", "numpy philox").split():
            print(json.dumps(rate(mode, B)), flush=True)
