"""The driver's bench sequence (`bench.py --steps 20 --warmup 5`: warmup of 5 steps, then ONE timed 20-step call),
with the timed call repeated: how much slower the first timed call is than the following ones, and why.

    python tools/first_call_probe.py [variant...]
variants: plain (as bench.py), prerun (the 20-step plan launched once before the warmup), touchacts / touchouts /
touchall (the action / output buffers read / rewritten once after setup), hbm (bench.py's HBM-ceiling copies,
2 GiB x 10 copies + 10 fills, run before the env is built), events (plain, with each call's kernel time from
HIP events as well), split / split5 (the W warmup steps as 3 + 2 / W single-step launches).
"""
import os
import sys
import time

os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-po-taxi_amd"))
import torch  # noqa: E402
from gym_po_amd import MultistoryFourRoomsEnv  # noqa: E402

B, C, W = 1 << 20, 20, 5
dev = torch.device("cuda", 0)
for variant in sys.argv[1:] or ["plain", "prerun"]:
    if variant == "hbm":
        a = torch.empty(1 << 31, dtype=torch.uint8, device=dev)
        b = torch.empty_like(a)
        for _ in range(10):
            b.copy_(a)
            a.fill_(1)
        torch.cuda.synchronize(dev)
        del a, b
    env = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device=dev)
    env.seed(0)
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    acts = torch.randint(0, 4, (C, B), device=dev, dtype=torch.int32, generator=g)
    out = env._alloc_outputs(C)
    for o in out:
        o.zero_()
    plans = {C: env.rollout_plan(acts, out)[0]}
    plans[W] = env.rollout_plan(acts[:W], tuple(o[:W] for o in out))[0]
    if variant == "prerun":
        plans[C]()
    if variant in ("touchacts", "touchall"):
        acts.view(torch.uint8).max()
    if variant in ("touchouts", "touchall"):
        for o in out:
            o.zero_()
    if variant == "events":
        env.set_profiling(True)
    if variant in ("split", "split5"):  # the same W warmup steps as 2 (3 + 2) or W (1 each) launches
        parts = [3, W - 3] if variant == "split" else [1] * W
        done = 0
        for k in parts:
            if k not in plans:
                plans[k] = env.rollout_plan(acts[done:done + k], tuple(o[done:done + k] for o in out))[0]
            plans[k]()
            done += k
    else:
        plans[W]()
    if variant == "events":
        torch.cuda.synchronize(dev)
        env.profile_read()
    ts, ks = [], []
    for rep in range(6):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        plans[C]()
        torch.cuda.synchronize(dev)
        ts.append((time.perf_counter() - t0) * 1e6)
        if variant == "events":
            ks.append(env.profile_read()[0] * 1e3)
    print(f"{variant}: timed 20-step calls (us): " + " ".join(f"{t:.1f}" for t in ts), flush=True)
    if ks:
        print(f"{variant}: their kernel events (us): " + " ".join(f"{t:.1f}" for t in ks), flush=True)
    env.close()
