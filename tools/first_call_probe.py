"""The driver's bench sequence (`bench.py --steps 20 --warmup 5`: warmup of 5 steps, then ONE timed 20-step call),
with the timed call repeated: how much slower the first timed call is than the following ones, and why.

    python tools/first_call_probe.py [variant...]
variants: plain (as bench.py), prerun (the 20-step plan launched once before the warmup), touchacts / touchouts /
touchall (the action / output buffers read / rewritten once after setup).
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
    plans[W]()
    ts = []
    for rep in range(6):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        plans[C]()
        torch.cuda.synchronize(dev)
        ts.append((time.perf_counter() - t0) * 1e6)
    print(f"{variant}: timed 20-step calls (us): " + " ".join(f"{t:.1f}" for t in ts), flush=True)
    env.close()
