"""ORACLE / TEST INFRASTRUCTURE — numpy's standard normal sampler restated in Python.

The reference draws its C-ROOMS noise with `rng.normal(scale=...)` (gym_po/envs/rooms/crooms.py:175-178,
:324), i.e. numpy's Generator.standard_normal: random_standard_normal in
numpy/random/src/distributions/distributions.c (numpy 2.2.6 here, a third-party dependency absent from
/root/reference): a 256-layer ziggurat on 64-bit words (idx = low 8 bits, sign = bit 8, a 52-bit magnitude;
layer 0's tail by Marsaglia's exponential method; next_double = (word >> 11) * 2^-53). The tables are
tests/golden/ziggurat_tables.npz, generated with csrc/ziggurat_tables.h by tools/gen_ziggurat.py and pinned
to numpy's own outputs. `standard_normals` is checked bit for bit against numpy (tests/test_oracle_extra.py);
the device restatement (csrc/crooms.hip zig_normal) is checked against it and numpy on the GPU.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this module.
"""
import math
import os

import numpy as np

R = 3.6541528853610087963519472518
INV_R = 0.27366123732975827203338247596
_TABLES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                       "ziggurat_tables.npz")


def tables():
    z = np.load(_TABLES)
    return [int(x) for x in z["ki"]], [float(x) for x in z["wi"]], [float(x) for x in z["fi"]]


def standard_normals(words, n, tabs=None):
    """n normals from an iterable of uint64 words, consumed in numpy's order. Returns (values, words used)."""
    ki, wi, fi = tabs or tables()
    it = iter(words)
    used = 0

    def nxt():
        nonlocal used
        used += 1
        return int(next(it))

    def next_double():
        return (nxt() >> 11) * (1.0 / 9007199254740992.0)

    out = np.empty(n)
    for j in range(n):
        while True:
            r = nxt()
            idx = r & 0xFF
            r >>= 8
            sign = r & 1
            rabs = (r >> 1) & 0x000FFFFFFFFFFFFF
            x = rabs * wi[idx]
            if sign:
                x = -x
            if rabs < ki[idx]:
                break
            if idx == 0:
                while True:
                    xx = -INV_R * math.log1p(-next_double())
                    yy = -math.log1p(-next_double())
                    if yy + yy > xx * xx:
                        x = -(R + xx) if ((rabs >> 8) & 1) else R + xx
                        break
                break
            if ((fi[idx - 1] - fi[idx]) * next_double() + fi[idx]) < math.exp(-0.5 * x * x):
                break
        out[j] = x
    return out, used
