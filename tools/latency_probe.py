"""Host-side fixed cost of one fused rollout call (launch + sync), the part of a short timed region that the
kernel's event time does not see.

    python tools/latency_probe.py [--spin early|late] [B] [K...]

Per case: median host wall (perf_counter around plan() + torch.cuda.synchronize()) over 100 reps, and
the HIP-event kernel time of the same launch. `--spin early` calls hipSetDeviceFlags(hipDeviceScheduleSpin)
on torch's HIP runtime before the first device call, `--spin late` after it.
"""
import ctypes
import os
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # as bench.py
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-po-taxi_amd"))
args = [a for a in sys.argv[1:]]
spin = None
if "--spin" in args:
    i = args.index("--spin")
    spin = args[i + 1]
    del args[i:i + 2]
B = int(args[0]) if args else 1 << 20
Ks = [int(a) for a in args[1:]] or [1, 20, 128]

import torch  # noqa: E402


def set_spin():
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"), mode=ctypes.RTLD_GLOBAL)
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))
    print(f"hipSetDeviceFlags(spin) rc={rc}", flush=True)


if spin == "early":
    set_spin()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
x = torch.zeros(16, device=dev)
torch.cuda.synchronize()
if spin == "late":
    set_spin()


def med(fn, reps=100):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6, float(np.percentile(ts, 10)) * 1e6


print(f"empty torch op + sync: median {med(lambda: x.add_(1))[0]:.1f} us", flush=True)
from gym_po_amd import MultistoryFourRoomsEnv  # noqa: E402

# GP_KNOBS="no_spw=1,..." : gp_debug_set knobs for the env (in-call A/B of kernel variants in one library)
from gym_po_amd._lib import debug_knobs  # noqa: E402
knobs = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in os.environ.get("GP_KNOBS", "").split(",") if kv)
with debug_knobs(**knobs):
    env = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device=dev)
print(f"knobs {knobs}", flush=True)
env.reset(seed=0)
for K in Ks:
    acts = torch.randint(0, 4, (K, B), device=dev, dtype=torch.int32)
    out = env._alloc_outputs(K)
    run, _ = env.rollout_plan(acts, out)
    for _ in range(5):
        run()
    m, p10 = med(run)
    env.set_profiling(True)
    for _ in range(20):
        run()
    ms, nk = env.profile_read()
    env.set_profiling(False)
    kus = ms / nk * 1e3
    print(f"B={B} K={K}: host wall median {m:.1f} us (p10 {p10:.1f}); kernel (events) {kus:.1f} us; "
          f"host - kernel = {m - kus:.1f} us; wall per step {m / K:.2f} us", flush=True)
env.close()
