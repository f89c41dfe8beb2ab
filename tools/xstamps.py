"""Phase breakdown of one C-ROOMS exact-mode step (csrc/crooms.hip xg_* kernels) from a GP_STAMPS build.

    python gym-po-taxi_amd/build.py --stamps && python tools/xstamps.py [B] [K] [reps]

Stamps (s_memrealtime, 100 MHz, chip-synchronous; thread 0 of blocks < 1024; the last launch of each kind):
  0 action noise normals: 0 entry, 1 stream state + n known, 2 base state, 3 words + slow attempts,
      4 on-chain bits, 5 count published, 6 prefix known, 7 writes done
  2 wall noise (one workgroup): 0 entry, 1 n known, 7 state set (extension covered), 6 drawn (not covered)
  1 dry step: 0 entry, 7 flags published     3 step: 0 entry, 1 wall-hit prefix, 2 flags published, 7 end
  4 choices: 0 entry, 4 a kernel argument read, 3 stream state read, 1 n known, 2 base state, 5 count published,
      6 prefix known, 7 writes done
  5 resets: 0 entry, 1 table staged
Stamps older than a launch's first entry are left-overs of earlier launches and are dropped.
"""
import ctypes
import os
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # as the package and bench.py
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-po-taxi_amd"))
os.environ.setdefault("GYM_PO_AMD_LIB", os.path.join(ROOT, "gym-po-taxi_amd", "gym_po_amd", "libgympo_amd_stamps.so"))
import torch  # noqa: E402
from gym_po_amd import CRoomsEnv, _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 3
NAMES = ["action normals", "dry step", "wall normals", "step", "choices", "resets"]

env = CRoomsEnv(B, obs_type="vector_mdp", rng_mode="numpy")
env.reset(seed=0)
a = torch.rand((K, B, 2), device=env.device) * 2 - 1
fn = _lib.lib().gp_debug_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
N = 6 * 1024 * 8
for rep in range(REPS):
    env.rollout(a)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * N)()
    got = fn(env._handle, buf, N)
    assert got == N, f"no stamps (got {got}): not a GP_STAMPS build or B <= 4096"
    st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(6, 1024, 8) * 10  # ns
    print(f"== B={B} K={K} rep {rep}: the last step of the rollout")
    t_first = st[0, :, 0][st[0, :, 0] > 0].min()
    prev_end = None
    for k in (0, 1, 2, 3, 4, 5):
        e = st[k, :, 0]
        ent = e[e > 0]
        e0 = ent.min()
        v = np.where(st[k] >= e0, st[k], 0)
        ends = v[v > 0]
        gap = "" if prev_end is None else f" gap after previous {e0 - prev_end:6d} ns;"
        line = [f"{NAMES[k]:15s} at {e0 - t_first:7d} ns;{gap} blocks {len(ent):4d}, entry spread {ent.max() - e0:6d}"]
        for i in range(1, 8):
            c = v[:, i]
            c = c[c > 0]
            if len(c):
                line.append(f"s{i} {np.median(c) - e0:6.0f}/{c.max() - e0:6d} ({len(c)})")
        print("  " + "; ".join(line))
        # per-block phase costs: median over blocks of (stamp i - the block's previous stamp)
        ords = {4: [0, 4, 3, 1, 2, 5, 6, 7]}.get(k, list(range(8)))
        d = []
        for i0, i1 in zip(ords, ords[1:]):
            m = (v[:, i0] > 0) & (v[:, i1] > 0)
            if m.sum():
                d.append(f"{i0}->{i1} {np.median(v[m, i1] - v[m, i0]):6.0f}")
        print("      per block (median ns): " + "; ".join(d))
        prev_end = ends.max()
    print(f"  step total {prev_end - t_first} ns (action normals entry -> last resets stamp)")
