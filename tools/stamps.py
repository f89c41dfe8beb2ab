"""Phase breakdown of the fused numpy rollout kernel from a GP_STAMPS diagnostic build.

    python gym-po-taxi_amd/build.py --stamps && python tools/stamps.py [B]
All stamps are s_memrealtime (100 MHz, synchronous across XCDs), per block and step:
0 step start (env wave 0), 1 transitions done, 2 B1 passed, 3 resets done (env wave 0),
4 B2 passed, 5 step end, 6 granule published (control wave), 7 exchange done (control wave).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-po-taxi_amd"))
os.environ.setdefault("GYM_PO_AMD_LIB", os.path.join(ROOT, "gym-po-taxi_amd", "gym_po_amd", "libgympo_amd_stamps.so"))
import torch  # noqa: E402
from gym_po_amd import MultistoryFourRoomsEnv, _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
env = MultistoryFourRoomsEnv(B, 1, obs_type="hansen")
env.reset(seed=0)
acts = torch.randint(0, 4, (K, B), device="cuda", dtype=torch.int32)
for _ in range(3):
    env.rollout(acts)
torch.cuda.synchronize()
L = _lib.lib()
fn = L.gp_debug_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
NS = 256 * 64 * 16
buf = (ctypes.c_ulonglong * (NS + 256 * 8))()
n = fn(env._handle, buf, NS + 256 * 8)
raw = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
a = raw[:NS].reshape(256, 64, 16)
G = int(env.query("fused_blocks"))
# launch-level view of the last launch: entry, tables staged, step loop done, kernel end (per block)
L4 = raw[NS:].reshape(256, 8)[:G, :4] * 10
t0 = L4[:, 0].min()
print(f"launch (K={K}, G={G}): entry spread {L4[:, 0].max() - t0} ns; entry->tables staged median "
      f"{np.median(L4[:, 1] - L4[:, 0]):.0f} max {np.max(L4[:, 1] - L4[:, 0])} ns; first entry -> last staged "
      f"{L4[:, 1].max() - t0} ns")
s0 = a[:G, 0, 0] * 10
print(f"  first entry -> step 0 start: min {s0.min() - t0} max {s0.max() - t0} ns; "
      f"loop done -> kernel end median {np.median(L4[:, 3] - L4[:, 2]):.0f} max {np.max(L4[:, 3] - L4[:, 2])} ns")
print(f"  first entry -> last kernel end {L4[:, 3].max() - t0} ns = {(L4[:, 3].max() - t0) / K:.0f} ns/step; "
      f"last step start -> last loop done {L4[:, 2].max() - (a[:G, min(K, 64) - 1, 0] * 10).max()} ns")
L6 = raw[NS:].reshape(256, 8)[:G, 4:6] * 10
print(f"  env prologue after the barrier: action rows done median {np.median(L6[:, 0] - L4[:, 1]):.0f} ns, lane "
      f"states ready median {np.median(L6[:, 1] - L4[:, 1]):.0f} ns (max over blocks {np.max(L6[:, 1] - t0)} ns from "
      f"first entry)")
L7 = raw[NS:].reshape(256, 8)[:G, 6:8]
print(f"  SPW: steps with the windows ready per block median {np.median(L7[:, 0]):.0f} of {K}, steps with no lane "
      f"jumping median {np.median(L7[:, 1]):.0f} (min over blocks {L7[:, 1].min()})")
st_k = a[:G, :min(K, 64), 0] * 10 - t0
print("  step k start, max over blocks (ns from first entry), k = 0..7:", [int(x) for x in st_k.max(0)[:8]])
env.set_profiling(True)
for _ in range(5):
    env.rollout(acts)
ms, nk = env.profile_read()
env.set_profiling(False)
print(f"  event-timed kernel: {ms / nk * 1e3:.1f} us per launch of K={K} ({ms / nk / K * 1e6:.0f} ns/step)")
if K < 8:
    sys.exit(0)
a = a[:G, 2:K - 2] * 10  # ns
def rep(name, d):
    per_step_max = d.max(0)
    print(f"{name:34s} median {np.median(d):7.0f} ns  p90 {np.percentile(d, 90):7.0f}  "
          f"max-over-blocks (median over steps) {np.median(per_step_max):7.0f}")
rep("transitions (0->1)", a[:, :, 1] - a[:, :, 0])
rep("B1 wait (1->2)", a[:, :, 2] - a[:, :, 1])
rep("B1 -> exchange done (2->7)", a[:, :, 7] - a[:, :, 2])
rep("exchange done -> B2 (7->4)", a[:, :, 4] - a[:, :, 7])
rep("resets (4->3)", a[:, :, 3] - a[:, :, 4])
rep("advance (3->5)", a[:, :, 5] - a[:, :, 3])
rep("step (0->next 0)", a[:, 1:, 0] - a[:, :-1, 0])
pub, done = a[:, :, 6], a[:, :, 7]
print(f"publish spread across blocks (max-min)   median {np.median(pub.max(0) - pub.min(0)):.0f} ns")
print(f"exchange done - last publish             median {np.median(done - pub.max(0)[None, :]):.0f} ns")
print(f"step start spread across blocks          median {np.median(a[:, :, 0].max(0) - a[:, :, 0].min(0)):.0f} ns")
slow = pub.argmax(0)
print("slowest publisher per step:", slow[:24].tolist())
t01 = (a[:, :, 1] - a[:, :, 0])
print("slowest transitions block per step:", t01.argmax(0)[:24].tolist())
b0 = 0
print("block 0 phases (ns) step 10:", np.diff(a[b0, 10, [0, 1, 2, 7, 4, 5]]).tolist())
bs = int(slow[10])
print(f"block {bs} phases (ns) step 10:", np.diff(a[bs, 10, [0, 1, 2, 7, 4, 5]]).tolist())
pd, dd = a[:, :, 8], a[:, :, 9]
print(f"poll done - last publish                 median {np.median(pd - pub.max(0)[None, :]):.0f} ns")
print(f"block0 gather done - last publish        median {np.median(a[0, :, 10] - pub.max(0)):.0f} ns")
print(f"draw cells (8->9)                        median {np.median(dd - pd):.0f} ns")
if (a[:, :, 14] > 0).all():
    print(f"  poll done -> lists ready (8->14)       median {np.median(a[:, :, 14] - pd):.0f} ns")
    print(f"  cell draw proper (14->9)               median {np.median(dd - a[:, :, 14]):.0f} ns")
print(f"publish_next etc (9->7)                  median {np.median(done - dd):.0f} ns")
e11, e12, e13 = a[:, :, 11], a[:, :, 12], a[:, :, 13]
rep("env: B1 -> resetters listed (2->11)", e11 - a[:, :, 2])
rep("env: staging written (11->12)", e12 - e11)
rep("env: J_B applied (12->13)", e13 - e12)
rep("env: B2 wait (13->4)", a[:, :, 4] - e13)
if (a[:, :, 15] > 0).all():
    rep("ctrl: lists ready -> jumps done (14->15)", a[:, :, 15] - a[:, :, 14])
    rep("ctrl: jumps done -> cells stored (15->9)", a[:, :, 9] - a[:, :, 15])
