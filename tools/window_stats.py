"""Reset-count statistics of the headline workload, to size the speculative word windows of the windowed fused
kernel (csrc/wgrid.hip): per step the total resets b_t, per block (4096 contiguous envs) its count and global
prefix, and the error of the predictors the kernel can use before the step's exchange.

    python tools/window_stats.py [B] [steps] [block_envs]

Runs the numpy oracle (test infrastructure; this is an offline sizing tool, nothing in the product imports it).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import gridworld  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
T = int(sys.argv[2]) if len(sys.argv) > 2 else 120
E = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
G = B // E
ora = gridworld.FourRoomsOracle(B, 1, obs_type="hansen")
ora.reset_seed(0)
rng = np.random.default_rng(1)
bs, pres = [], []
for t in range(T):
    o, r, d, tr = ora.step_seeded(rng.integers(0, 4, B))
    m = (d | tr).reshape(G, E).sum(1)
    bs.append(int(m.sum()))
    pres.append(np.concatenate(([0], np.cumsum(m)[:-1])))
bs = np.array(bs)
pres = np.array(pres)
print("b_t:", bs.tolist())
for name, pred in (("b[t-1]", bs[:-1]), ("mean of last 4", np.array([bs[max(0, t - 4):t].mean() for t in range(1, T)]))):
    err = bs[1:] - pred
    tail = err[40:]
    print(f"total predictor {name}: steady (t>=41) err sd {tail.std():.1f}, max |err| {np.abs(tail).max()}, "
          f"all-steps max |err| {np.abs(err).max()}")
# block prefix predicted as b[t-1] * beta / G
pp = bs[:-1, None] * np.arange(G)[None] / G
err = pres[1:] - pp
print(f"prefix predictor b[t-1]*beta/G: steady sd by block quartile "
      f"{[round(float(err[40:, q * G // 4:(q + 1) * G // 4].std()), 1) for q in range(4)]}, "
      f"max |err| steady {np.abs(err[40:]).max():.0f}, all {np.abs(err).max():.0f}")
