"""Phase breakdown of the windowed numpy rollout (csrc/wgrid.hip) from a GP_STAMPS diagnostic build.

    python gym-po-taxi_amd/build.py --stamps && python tools/wstamps.py [B] [K]

Stamps are s_memrealtime (100 MHz, synchronous across XCDs), kept in LDS during the launch (round 6: a global store
per stamp was waited for by later vmcnt(0) waits and stretched the phases), per block and step k < 24 (42 slots):
  env wave 0: 0 step start, 1 transitions done, 2 S(y) seen, 3 coarse states done, 4 resetters listed,
              5 window filled (before B2); env wave 7: 15 window filled
  control:    6 S(y) + rejection check + window base published, 7 transitions seen, 8 granule publish,
              9 all-gather done, 10 cells drawn (before B2), 11 after B2, 12 next state done
  store wave: 13 copy start (after B2), 14 copy issued
  every env wave w: 16 + w transitions done, 24 + w window filled (before B2), 32 + w step start
  env wave 0: 41 loop top (before the next actions' loads), 40 after issuing them
Launch stamps per block: 0 entry, 1 P1 passed (control), 2 env wave 0's first window filled, 3 control step loop
done, 4 kernel end, 5 / 6 table staging done (control wave / store wave 0), 7 env wave 0 has the first
window's offset.
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
knobs.setdefault("wg_kmax", 1 << 20)  # every launch on the windowed kernel (longer ones would run the fused kernel)
with debug_knobs(**knobs):
    env = MultistoryFourRoomsEnv(B, 1, obs_type="hansen")
print(f"knobs {knobs}")
assert env.query("wgrid") == 1, "the windowed kernel is not eligible for this size"
G = int(env.query("wgrid_blocks"))
env.reset(seed=0)
acts = torch.randint(0, 4, (K, B), device="cuda", dtype=torch.int32)
for _ in range(int(os.environ.get("SKIP", "0")) // K):  # SKIP=n: n steps first (a later episode phase)
    env.rollout(acts)
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
a = raw[:NS].reshape(256, 1024)[:, :24 * 42].reshape(256, 24, 42)[:G]
ls = raw[NS:].reshape(256, 8)[:G]
t0 = ls[:, 0].min()
print(f"B={B} K={K} G={G} E={env.query('wgrid_block_envs')} H={env.query('wgrid_halo')}")
print(f"launch: entry spread {ls[:, 0].max() - t0} ns; P1 passed (control, max) {ls[:, 1].max() - t0}; "
      f"control loop done (max) {ls[:, 3].max() - t0}; kernel end (max) {ls[:, 4].max() - t0} ns")
e0 = ls[:, 0]
print("prologue per block (median/max ns from the block's entry): env first window filled "
      f"{np.median(ls[:, 2] - e0):.0f}/{(ls[:, 2] - e0).max()}; table staging done: control wave "
      f"{np.median(ls[:, 5] - e0):.0f}/{(ls[:, 5] - e0).max()}, store wave 0 {np.median(ls[:, 6] - e0):.0f}/"
      f"{(ls[:, 6] - e0).max()}; control past P1, first window published {np.median(ls[:, 1] - e0):.0f}/"
      f"{(ls[:, 1] - e0).max()}; env wave 0 sees it {np.median(ls[:, 7] - e0):.0f}/{(ls[:, 7] - e0).max()}; "
      f"env wave 0 starts step 0 {np.median(a[:, 0, 0] - e0):.0f}/{(a[:, 0, 0] - e0).max()}")


def at(k, i):  # stamp i of step k over blocks, ns from the first block's entry
    v = a[:, k, i] - t0
    return f"{np.median(v):6.0f}/{v.max():6.0f}"


print("first steps (median/max over blocks, ns from launch):")
for k in range(min(K, 3)):
    print(f"  k={k}: env start {at(k, 0)}  transitions done {at(k, 1)}  publish {at(k, 8)}  gather done {at(k, 9)}  "
          f"cells {at(k, 10)}")
kl = min(K, 24) - 1
print(f"last step k={kl}: env start {at(kl, 0)}  publish {at(kl, 8)}  gather done {at(kl, 9)}  next state {at(kl, 12)}")
print(f"  tail: last next-state (max) -> kernel end (max) {ls[:, 4].max() - (a[:, kl, 12].max())} ns")
env.set_profiling(True)
for _ in range(5):
    env.rollout(acts)
ms, nk = env.profile_read()
env.set_profiling(False)
print(f"event-timed kernel: {ms / nk * 1e3:.1f} us per launch ({ms / nk / K * 1e6:.0f} ns/step)")
if K < 8:
    sys.exit(0)
kk = min(K, 24)
x = a[:, 2:kk - 1]


def rep(name, d):
    print(f"  {name:44s} median {np.median(d):7.0f} ns  p90 {np.percentile(d, 90):7.0f}  max-over-blocks(median) "
          f"{np.median(d.max(0)):7.0f}")


step = a[:, 3:kk, 0] - a[:, 2:kk - 1, 0]
rep("step (env wave 0 start -> next start)", step)
rep("env: transitions (0->1)", x[:, :, 1] - x[:, :, 0])
rep("env: S(y) wait (1->2)", x[:, :, 2] - x[:, :, 1])
rep("env: coarse states (2->3)", x[:, :, 3] - x[:, :, 2])
rep("env: resetter listing (3->4)", x[:, :, 4] - x[:, :, 3])
rep("env: window fill (4->5)", x[:, :, 5] - x[:, :, 4])
rep("env: B2 wait (5 -> ctrl 11)", x[:, :, 11] - x[:, :, 5])
rep("env wave 7 window done - wave 0 (15-5)", x[:, :, 15] - x[:, :, 5])
rep("ctrl: step-start work (prev 12 -> 6)", a[:, 3:kk, 6] - a[:, 2:kk - 1, 12])
rep("ctrl: after B2 -> next state (11->12)", x[:, :, 12] - x[:, :, 11])
rep("ctrl: trans wait (6->7)", x[:, :, 7] - x[:, :, 6])
rep("ctrl: publish (7->8)", x[:, :, 8] - x[:, :, 7])
rep("ctrl: gather (8->9)", x[:, :, 9] - x[:, :, 8])
rep("ctrl: cells (9->10)", x[:, :, 10] - x[:, :, 9])
rep("ctrl: B2 wait (10->11)", x[:, :, 11] - x[:, :, 10])
pub = x[:, :, 8]
print(f"  publish spread across blocks (max-min)       median {np.median(pub.max(0) - pub.min(0)):.0f} ns")
print(f"  gather done - last publish                   median {np.median(x[:, :, 9] - pub.max(0)[None]):.0f} ns")
rep("store: copy issue (13->14)", x[:, :, 14] - x[:, :, 13])
print("block 0, step 10 (ns from env start):", (a[0, 10] - a[0, 10, 0]).tolist())
print("median over blocks and steps of stamp i - env start (ns):", np.median(x[:, :, :16] - x[:, :, :1], axis=(0, 1)).astype(int).tolist())
# per env wave (SIMD w % 4 under round-robin wave placement: the control wave is wave 8 -> SIMD 0, the store waves 9, 10
# -> SIMDs 1, 2): transitions done and window filled, ns after env wave 0's step start
tw = x[:, :, 16:24] - x[:, :, :1]
fw = x[:, :, 24:32] - x[:, :, :1]
print("per env wave, median ns after wave 0's step start: transitions done | window filled")
print("  trans: " + " ".join(f"w{w}:{np.median(tw[:, :, w]):5.0f}" for w in range(8)))
print("  fill:  " + " ".join(f"w{w}:{np.median(fw[:, :, w]):5.0f}" for w in range(8)))
print("  slowest wave's transitions (max over w), median %.0f p90 %.0f; slowest fill median %.0f p90 %.0f; next env start %.0f" % (
    np.median(tw.max(2)), np.percentile(tw.max(2), 90), np.median(fw.max(2)), np.percentile(fw.max(2), 90),
    np.median(step)))
sw = x[:, :, 32:40] - x[:, :, :1]
print("  start: " + " ".join(f"w{w}:{np.median(sw[:, :, w]):5.0f}" for w in range(8)))
nxt = a[:, 3:kk, 32:40] - a[:, 2:kk - 1, :1]  # every wave's NEXT step start, from wave 0's start of this step
print("  next start: " + " ".join(f"w{w}:{np.median(nxt[:, :, w]):5.0f}" for w in range(8)))
lt = a[:, 3:kk, 41] - a[:, 2:kk - 1, 0]
fd = a[:, 3:kk, 40] - a[:, 2:kk - 1, 0]
print("  wave 0 next loop top %.0f, next actions issued %.0f, next start %.0f (median, from this step's start)" % (
    np.median(lt), np.median(fd), np.median(step)))
print("  which wave is slowest (transitions / fill), counts over blocks x steps:",
      np.bincount(tw.argmax(2).ravel(), minlength=8).tolist(), np.bincount(fw.argmax(2).ravel(), minlength=8).tolist())
# per block: median over steps of (publish - the step's median publish); the slowest blocks and their XCD
pubrel = x[:, :, 8] - np.median(x[:, :, 8], axis=0)[None]
bm = np.median(pubrel, axis=1)
order = np.argsort(bm)[::-1]
print("slowest publishers (block: median ns behind the step's median publish, xcd):",
      ", ".join(f"{b}:{bm[b]:.0f}/x{b % 8}" for b in order[:12]))
print("publish lateness per block, quantiles over blocks of the per-block median: ",
      " ".join(f"q{q}:{np.percentile(bm, q):.0f}" for q in (0, 10, 50, 90, 99, 100)))
last = x[:, :, 8].argmax(0)
print("last publisher per step (block/xcd):", " ".join(f"{b}/{b % 8}" for b in last[:24]))
# a last publisher's phases vs the median block: env start / trans done (slowest wave) / publish, relative to the step's median env start
ms0 = np.median(x[:, :, 0], axis=0)
lp = np.array([[x[last[j], j, 0] - ms0[j], tw[last[j], j].max() + x[last[j], j, 0] - ms0[j], x[last[j], j, 8] - ms0[j]] for j in range(x.shape[1])])
print("last publisher vs the step's median env start (median over steps): env start %.0f, slowest-wave transitions %.0f, publish %.0f" % tuple(np.median(lp, axis=0)))
# per-XCD phase (blocks beta with beta % 8 = x: round-robin dispatch puts them on XCD x), median over steps of the
# block's stamp minus the step's earliest env start over all blocks
st0 = x[:, :, 0].min(0)[None]
print("per XCD (beta % 8), median ns after the step's earliest env start: env start / transitions done / publish / gather done / cells")
for xcd in range(8):
    sel = np.arange(G) % 8 == xcd
    vals = [np.median(x[sel, :, i] - st0) for i in (0, 1, 8, 9, 10)]
    print(f"  XCD {xcd}: " + " / ".join(f"{v:6.0f}" for v in vals) + f"   transitions {np.median(x[sel, :, 1] - x[sel, :, 0]):5.0f}")
