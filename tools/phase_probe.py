"""Event-timed K-step launches of the numpy FourRooms rollout at different distances from reset (the episode
phase changes the per-step reset count): 10 launches right after reset, then after `skip` more steps.

    python tools/phase_probe.py [B] [K] [skip...]      (GAP_US=n: sync + n us of host sleep after every launch)
"""
import os
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # as bench.py
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-po-taxi_amd"))
import torch  # noqa: E402
from gym_po_amd import MultistoryFourRoomsEnv  # noqa: E402
from gym_po_amd._lib import debug_knobs  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
skips = [int(x) for x in sys.argv[3:]] or [0, 200, 400, 1000, 2000]
GAP = float(os.environ.get("GAP_US", "0")) * 1e-6
knobs = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in os.environ.get("GP_KNOBS", "").split(",") if kv)
with debug_knobs(**knobs):
    env = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen")
env.reset(seed=0)
acts = torch.randint(0, 4, (K, B), device="cuda", dtype=torch.int32)
out = env._alloc_outputs(K)
run, _ = env.rollout_plan(acts, out)
done = 0
for s in skips:
    while done < s:
        run()
        done += K
    m0 = env.metrics()["episodes"]
    env.set_profiling(True)
    for _ in range(10):
        run()
        if GAP:  # idle the GPU between launches (GAP_US): the launch then starts from an idle chip
            torch.cuda.synchronize()
            time.sleep(GAP)
    ms, nk = env.profile_read()
    env.set_profiling(False)
    done += 10 * K
    torch.cuda.synchronize()
    eps = env.metrics()["episodes"] - m0
    print(f"{knobs} steps {s}-{done}: {ms / nk * 1e3:.1f} us per {K}-step launch; resets per step {eps / (10 * K):.0f}",
          flush=True)
