"""Phase breakdown of the windowed numpy rollout (csrc/wgrid.hip) from a GP_STAMPS diagnostic build.

    python gym-po-taxi_amd/build.py --stamps && python tools/wstamps.py [B] [K]

Stamps are s_memrealtime (100 MHz, synchronous across XCDs), per block and step k:
  env wave 0: 0 step k-1's resetters: wait for the exchange starts, 1 exchange outcome seen, 2 transitions start
              (cells taken, window and staging ready), 3 transitions done, 4 coarse states done, 5 next window
              filled; env wave 7: 15 transitions done
  control:    6 S(x), S(y), next window base published, 7 transitions seen, 8 granule published, 9 all-gather done,
              10 exchange outcome published (cells_done), 12 next S(x) done
  store wave: 13 copy start, 14 copy issued
Launch stamps per block: 0 entry, 1 P1 passed (control), 3 step loop done, 4 kernel end.
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
NS = 256 * 64 * 16
buf = (ctypes.c_ulonglong * (NS + 256 * 8))()
fn(env._handle, buf, NS + 256 * 8)
raw = np.frombuffer(buf, dtype=np.uint64).astype(np.int64) * 10  # ns
a = raw[:NS].reshape(256, 64, 16)[:G]
ls = raw[NS:].reshape(256, 8)[:G]
t0 = ls[:, 0].min()
print(f"B={B} K={K} G={G} E={env.query('wgrid_block_envs')} H={env.query('wgrid_halo')}")
print(f"launch: entry spread {ls[:, 0].max() - t0} ns; P1 passed (max) {ls[:, 1].max() - t0}; loop done (max) {ls[:, 3].max() - t0}; kernel end (max) {ls[:, 4].max() - t0} ns")
env.set_profiling(True)
for _ in range(5):
    env.rollout(acts)
ms, nk = env.profile_read()
env.set_profiling(False)
print(f"event-timed kernel: {ms / nk * 1e3:.1f} us per launch ({ms / nk / K * 1e6:.0f} ns/step)")
if K < 8:
    sys.exit(0)
kk = min(K, 64)
x = a[:, 2:kk - 1]


def rep(name, d):
    print(f"  {name:44s} median {np.median(d):7.0f} ns  p90 {np.percentile(d, 90):7.0f}  max-over-blocks(median) "
          f"{np.median(d.max(0)):7.0f}")


n = kk - 3
A = a[:, 2:2 + n]          # step k
N = a[:, 3:3 + n]          # step k + 1
rep("step (transitions start -> next start)", N[:, :, 2] - A[:, :, 2])
rep("chain: transitions, wave 0 (2->3)", A[:, :, 3] - A[:, :, 2])
rep("chain: transitions, wave 7 (2->15)", A[:, :, 15] - A[:, :, 2])
rep("chain: ctrl sees transitions (wave-0 start->7)", A[:, :, 7] - A[:, :, 2])
rep("chain: ctrl publish (7->8)", A[:, :, 8] - A[:, :, 7])
rep("chain: all-gather (8->9)", A[:, :, 9] - A[:, :, 8])
rep("chain: R, offset, cells_done (9->10)", A[:, :, 10] - A[:, :, 9])
rep("chain: env sees cells_done (ctrl 10 -> env 1)", N[:, :, 1] - A[:, :, 10])
rep("chain: cells + waits (env 1 -> 2)", N[:, :, 2] - N[:, :, 1])
rep("off: coarse states (3->4)", A[:, :, 4] - A[:, :, 3])
rep("off: next window fill (4->5)", A[:, :, 5] - A[:, :, 4])
rep("off: slack, fill done -> exchange seen (5 -> next 1)", N[:, :, 1] - A[:, :, 5])
rep("ctrl: step start -> published (prev 12 -> 6)", N[:, :, 6] - A[:, :, 12])
pub = A[:, :, 8]
print(f"  publish spread across blocks (max-min)       median {np.median(pub.max(0) - pub.min(0)):.0f} ns")
print(f"  gather done - last publish                   median {np.median(A[:, :, 9] - pub.max(0)[None]):.0f} ns")
rep("store: copy issue (13->14)", A[:, :, 14] - A[:, :, 13])
print("block 0, step 10 (ns from transitions start):", (a[0, 10] - a[0, 10, 2]).tolist())
