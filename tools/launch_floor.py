"""Launch-footprint probe: event-timed duration of launches with the headline kernel's footprint
that do (almost) nothing, beside the real wgrid_rollout<8,4> at K = 1 and K = 20, in one process.

    python tools/launch_floor.py [reps]

Builds tools/launch_floor.so (hipcc -shared) if missing. Every case: `reps` launches back to back on torch's
stream, each bracketed by its own HIP events (as bench.py's profiling pass), median and mean in µs; then the
host wall of one launch + torch.cuda.synchronize() from an idle stream (median of 50).
Cases 'real K=1 -tables' / '-first' / '-both' are the real kernel with the table staging and / or the first
window fill skipped (timing knobs wg_tmode 1024 / 2048: results invalid, measurement only).
Run it under `rocprofv3 --kernel-trace --stats` to get the same launches' dispatch-timestamp durations.
"""
import ctypes
import os
import subprocess
import sys
import time

os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # as bench.py
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-po-taxi_amd"))
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 200
SO = os.path.join(ROOT, "tools", "launch_floor.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    os.path.join(ROOT, "tools", "launch_floor.hip"), "-o", SO], check=True)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_po_amd import MultistoryFourRoomsEnv  # noqa: E402
from gym_po_amd._lib import debug_knobs  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
B = 1 << 20
env = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device=dev)
env.reset(seed=0)
G, E, lds = env.query("wgrid_blocks"), env.query("wgrid_block_envs"), env.query("wgrid_lds")
variants = {}
for name, tm in (("-tables", 1024), ("-first", 2048), ("-both", 3072)):
    with debug_knobs(wg_tmode=tm):
        v = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device=dev)
    v.reset(seed=0)
    variants[name] = v
lf = ctypes.CDLL(SO)
lf.lf_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int] + \
    [ctypes.c_void_p] * 5
STATIC = 12 * 1024  # the real kernel's static LDS (WgShared) on top of the dynamic bytes
assert lf.lf_setup(lds + STATIC) == 0
print(f"B={B} G={G} E={E} dynamic LDS {lds} B (+{STATIC} static in the probe)", flush=True)

K = 20
g = torch.Generator(device=dev)
g.manual_seed(1)
acts = torch.randint(0, 4, (K, B), device=dev, dtype=torch.int32, generator=g)
out = env._alloc_outputs(K)
for o in out:
    o.zero_()
plans = {k: env.rollout_plan(acts[:k], tuple(o[:k] for o in out))[0] for k in (1, 20)}
vplans = {n: v.rollout_plan(acts[:1], tuple(o[:1] for o in v._alloc_outputs(1)))[0] for n, v in variants.items()}
tab = torch.zeros(64 * 1024, dtype=torch.uint8, device=dev)
ptrs = [out[0].data_ptr() * 0 + acts.data_ptr()] + [o.data_ptr() for o in out]
stream = torch.cuda.current_stream(dev).cuda_stream


def probe(v, K_=0, P=None):
    def f():
        rc = lf.lf_launch(v, G, lds + STATIC, ctypes.c_void_p(stream), ctypes.c_void_p(P), K_, *[ctypes.c_void_p(p) for p in ptrs])
        assert rc == 0, rc
    return f


cases = [("trivial 256x64", probe(0)),
         ("footprint 704t+LDS+155v", probe(1)),
         ("footprint + 1 step nt outputs", probe(2)),
         ("footprint + 1 step sc1 outputs", probe(3)),
         ("footprint + table staging (lds.total)", probe(4, env.query("wgrid_lds") // 8 // 16 * 16, tab.data_ptr())),
         ("real K=1", plans[1]),
         ("real K=1 -tables", vplans["-tables"]),
         ("real K=1 -first", vplans["-first"]),
         ("real K=1 -both", vplans["-both"]),
         ("real K=20", plans[20])]


def timed(fn, reps):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return np.array([a.elapsed_time(b) * 1e3 for a, b in ev])


def wall(fn, reps=50):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    return float(np.median(ts))


for name, fn in cases:  # warm every case (first launches of a kernel carry one-time costs)
    for _ in range(3):
        fn()
torch.cuda.synchronize()
for rnd in range(2):
    print(f"--- round {rnd}: {REPS} back-to-back event-bracketed launches per case", flush=True)
    for name, fn in cases:
        t = timed(fn, REPS)
        print(f"{name:42s} event median {np.median(t):8.2f} us  mean {t.mean():8.2f}  p10 {np.percentile(t, 10):8.2f}"
              f"  p90 {np.percentile(t, 90):8.2f}  | idle-stream launch+sync wall {wall(fn):8.2f} us", flush=True)
for v in variants.values():
    v.close()
env.metrics()
env.close()
