"""Phase breakdown of the windowed numpy rollout (csrc/wgrid.hip) from a GP_STAMPS diagnostic build.

    python gym-po-taxi_amd/build.py --stamps && python tools/wstamps.py [B] [K]

Stamps are s_memrealtime (100 MHz, synchronous across XCDs), kept in LDS, for the first 32 steps of a launch,
per block and step k (round-5 schedule: windows, early count by the env waves, ranks):
  env wave 0: 16 cells_done seen, 0 resetter cells taken (window regenerated if it missed), 12 window ready,
              1 early count added, 3 next window filled, 2 transitions done, 18 next actions converted;
              20 + w: env wave w's transitions done
  control:    7 S(y) / next window base published, 5 block count ready, 6 granule published, 8 ranks + candidate
              cells done, 9 all-gather done, 10 cells placed / cells_done, 11 next rejection check done
  store wave: 13 copy start, 14 copy issued
Launch stamps per block: 0 entry, 1 P1 passed (control), 3 step loop done, 4 kernel end.
"""
import ctypes
import os
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # as bench.py
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-po-taxi_amd"))
os.environ.setdefault("GYM_PO_AMD_LIB", os.path.join(ROOT, "gym-po-taxi_amd", "gym_po_amd", "libgympo_amd_stamps.so"))
import torch  # noqa: E402
from gym_po_amd import MultistoryFourRoomsEnv, _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
from gym_po_amd._lib import debug_knobs  # noqa: E402
knobs = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in os.environ.get("GP_KNOBS", "").split(",") if kv)
with debug_knobs(**knobs):
    env = MultistoryFourRoomsEnv(B, 1, obs_type="hansen")
print(f"knobs {knobs}")
assert env.query("wgrid") == 1, "the windowed kernel is not eligible for this size"
G = int(env.query("wgrid_blocks"))
env.reset(seed=0)
acts = torch.randint(0, 4, (K, B), device="cuda", dtype=torch.int32)
for _ in range(4):
    env.rollout(acts)
torch.cuda.synchronize()
L = _lib.lib()
fn = L.gp_debug_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
NS = 256 * 32 * 32
buf = (ctypes.c_ulonglong * (NS + 256 * 8))()
fn(env._handle, buf, NS + 256 * 8)
raw = np.frombuffer(buf, dtype=np.uint64).astype(np.int64) * 10  # ns
a = raw[:NS].reshape(256, 32, 32)[:G]
ls = raw[NS:].reshape(256, 8)[:G]
t0 = ls[:, 0].min()
out = os.environ.get("WSTAMPS_RAW")
if out:
    np.savez_compressed(out, a=a, ls=ls)
print(f"B={B} K={K} G={G} E={env.query('wgrid_block_envs')}")
print(f"launch: entry spread {ls[:, 0].max() - t0} ns; P1 passed (max) {ls[:, 1].max() - t0}; "
      f"loop done (max) {ls[:, 3].max() - t0}; kernel end (max) {ls[:, 4].max() - t0} ns")
print(f"first step: env start (max) {a[:, 0, 0].max() - t0}; first publish (max) {a[:, 0, 6].max() - t0} ns")
env.set_profiling(True)
for _ in range(5):
    env.rollout(acts)
ms, nk = env.profile_read()
env.set_profiling(False)
print(f"event-timed kernel: {ms / nk * 1e3:.1f} us per launch ({ms / nk / K * 1e6:.0f} ns/step)")
if K < 8:
    sys.exit(0)
kk = min(K, 32)
x = a[:, 2:kk - 1]
nx = a[:, 3:kk]   # the next step's stamps
pv = a[:, 1:kk - 2]  # the previous step's stamps


def rep(name, d):
    print(f"  {name:46s} median {np.median(d):7.0f} ns  p90 {np.percentile(d, 90):7.0f}  max-over-blocks(median) "
          f"{np.median(d.max(0)):7.0f}")


rep("step (env wave 0 start -> next start)", nx[:, :, 0] - x[:, :, 0])
rep("env: window wait (0->12)", x[:, :, 12] - x[:, :, 0])
rep("env: early count (12->1)", x[:, :, 1] - x[:, :, 12])
rep("env: next window fill (1->3)", x[:, :, 3] - x[:, :, 1])
rep("env: transitions (3->2)", x[:, :, 2] - x[:, :, 3])
rep("env: next actions (2->18)", x[:, :, 18] - x[:, :, 2])
rep("env: wait cells_done (18->next 16)", nx[:, :, 16] - x[:, :, 18])
rep("env: take cells (16->0)", x[:, :, 0] - x[:, :, 16])
rep("ctrl: trans wait + S(y) (prev 11 -> 7)", x[:, :, 7] - pv[:, :, 11])
rep("ctrl: count wait (7 -> 5)", x[:, :, 5] - x[:, :, 7])
rep("ctrl: publish (5->6)", x[:, :, 6] - x[:, :, 5])
rep("ctrl: ranks + candidates (6->8)", x[:, :, 8] - x[:, :, 6])
rep("ctrl: gather (8->9)", x[:, :, 9] - x[:, :, 8])
rep("ctrl: publish -> gather done (6->9)", x[:, :, 9] - x[:, :, 6])
rep("ctrl: cells (9->10)", x[:, :, 10] - x[:, :, 9])
rep("ctrl: next rejection check (10->11)", x[:, :, 11] - x[:, :, 10])
rep("cells_done -> next count ready (10 -> next 5)", nx[:, :, 5] - x[:, :, 10])
pub = x[:, :, 6]
print(f"  publish spread across blocks (max-min)         median {np.median(pub.max(0) - pub.min(0)):.0f} ns")
print(f"  gather done - last publish                     median {np.median(x[:, :, 9] - pub.max(0)[None]):.0f} ns")
rep("store: copy issue (13->14)", x[:, :, 14] - x[:, :, 13])
tw = x[:, :, 20:28] - x[:, :, 3][:, :, None]
print("  transitions done per env wave (from wave 0's start), median:", [int(v) for v in np.median(tw, (0, 1))])
print("  transitions done per env wave, p90:", [int(v) for v in np.percentile(tw, 90, (0, 1))])
print("block 0, step 10 (ns from env start):", (a[0, 10] - a[0, 10, 0]).tolist())
