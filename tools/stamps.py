"""Phase breakdown of the fused numpy rollout kernel from a GP_STAMPS diagnostic build.

    python gym-po-taxi_amd/build.py --stamps && GYM_PO_AMD_LIB=.../libgympo_amd_stamps.so python tools/stamps.py
Stamps: 0 step start, 1 transitions+stores issued, 2 granule published, 3 all-gather done,
4 resetters resolved, 5 next state broadcast. Reports median cycles per phase over blocks/steps.
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
K = 64
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
buf = (ctypes.c_ulonglong * (256 * 64 * 8))()
n = fn(env._handle, buf, 256 * 64 * 8)
a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 64, 8).astype(np.int64)
G = min(256, (B + 4095) // 4096)
a = a[:G, 1:K - 1]
d = np.diff(a[:, :, :6], axis=2)
names = ["transitions+stores", "scan+publish", "all-gather", "resolve", "next-state"]
for i, nm in enumerate(names):
    print(f"{nm:20s} median {np.median(d[:, :, i]):8.0f} cyc  p90 {np.percentile(d[:, :, i], 90):8.0f}")
step = a[:, 1:, 0] - a[:, :-1, 0]
print(f"{'step total':20s} median {np.median(step):8.0f} cyc")
# skew between blocks at publish time
pub = a[:, :, 2]
print(f"publish skew across blocks (max-min) median {np.median(pub.max(0) - pub.min(0)):.0f} cyc")
