"""Generate csrc/ziggurat_tables.h: the 256-layer ziggurat of numpy's Generator.standard_normal
(numpy/random/src/distributions/distributions.c, random_standard_normal; numpy 2.2 here), the normal law the
reference's C-ROOMS draws its action and wall noise from (gym_po/envs/rooms/crooms.py:175-178, :324).

    python tools/gen_ziggurat.py      (CPU only, ~2 min; needs numpy + mpmath)

The layer edges x_i follow the Marsaglia-Tsang construction (r = 3.6541528853610087963519472518, each layer's
area v = r f(r) + int_r^inf f, f(x) = exp(-x^2/2)), evaluated at 60 digits: ki[i] = floor(2^52 x_{i-1}/x_i),
wi[i] = x_i / 2^52, fi[i] = f(x_i). numpy's published wi table differs from that evaluation in the last bits,
so each wi[i] is then pinned to numpy's own value: the double w that reproduces fl(rabs * w) for every
fast-path (or accepted) draw of layer i in 1.5M normals of a known PCG64 stream. The result is checked on
another seed: the restated algorithm over numpy's raw words must return numpy's standard_normal bit for bit.
"""
import math
import os
import struct

import mpmath
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "gym-po-taxi_amd", "csrc", "ziggurat_tables.h")
R = 3.6541528853610087963519472518
INV_R = 0.27366123732975827203338247596


def construct():
    mpmath.mp.dps = 60
    r = mpmath.mpf("3.6541528853610087963519472518")
    v = r * mpmath.exp(-r * r / 2) + mpmath.sqrt(mpmath.pi / 2) * mpmath.erfc(r / mpmath.sqrt(2))
    dn = r
    tn = dn
    m1 = mpmath.mpf(2) ** 52
    q = v / mpmath.exp(-dn * dn / 2)
    ki, wi, fi = [0] * 256, [0] * 256, [0] * 256
    ki[0] = int(mpmath.floor((dn / q) * m1))
    wi[0], wi[255] = q / m1, dn / m1
    fi[0], fi[255] = mpmath.mpf(1), mpmath.exp(-dn * dn / 2)
    for i in range(254, 0, -1):
        dn = mpmath.sqrt(-2 * mpmath.log(v / dn + mpmath.exp(-dn * dn / 2)))
        ki[i + 1] = int(mpmath.floor((dn / tn) * m1))
        tn = dn
        fi[i] = mpmath.exp(-dn * dn / 2)
        wi[i] = dn / m1
    return ki, [float(x) for x in wi], [float(x) for x in fi]


def standard_normals(words, n, ki, wi, fi):
    """numpy's random_standard_normal over a u64 word sequence (the restatement the device follows)."""
    out = []
    it = iter(words)

    def next_double():
        return (int(next(it)) >> 11) * (1.0 / 9007199254740992.0)

    while len(out) < n:
        r = int(next(it))
        idx = r & 0xFF
        r >>= 8
        sign = r & 1
        rabs = (r >> 1) & 0x000FFFFFFFFFFFFF
        x = rabs * wi[idx]
        if sign:
            x = -x
        if rabs < ki[idx]:
            out.append(x)
            continue
        if idx == 0:
            while True:
                xx = -INV_R * math.log1p(-next_double())
                yy = -math.log1p(-next_double())
                if yy + yy > xx * xx:
                    out.append(-(R + xx) if ((rabs >> 8) & 1) else R + xx)
                    break
        elif ((fi[idx - 1] - fi[idx]) * next_double() + fi[idx]) < math.exp(-0.5 * x * x):
            out.append(x)
    return np.array(out)


def pin_wi(ki, wi, fi, seed=2024, n=1500000):
    want = np.random.Generator(np.random.PCG64(seed)).standard_normal(n)
    W = [int(x) for x in np.random.PCG64(seed).random_raw(n + n // 20)]
    pairs = {i: [] for i in range(256)}
    it = 0

    def nd():
        nonlocal it
        x = (W[it] >> 11) * (1.0 / 9007199254740992.0)
        it += 1
        return x

    for j in range(n):  # walk numpy's word consumption, collecting (rabs, |x|) of every returned layer draw
        while True:
            r = W[it]
            it += 1
            idx = r & 0xFF
            r >>= 8
            rabs = (r >> 1) & 0x000FFFFFFFFFFFFF
            x = rabs * wi[idx]
            if rabs < ki[idx]:
                pairs[idx].append((rabs, abs(float(want[j]))))
                break
            if idx == 0:
                while True:
                    xx = -INV_R * math.log1p(-nd())
                    yy = -math.log1p(-nd())
                    if yy + yy > xx * xx:
                        break
                break
            if ((fi[idx - 1] - fi[idx]) * nd() + fi[idx]) < math.exp(-0.5 * x * x):
                pairs[idx].append((rabs, abs(float(want[j]))))
                break

    def step(x, d):
        b = struct.unpack("<q", struct.pack("<d", x))[0]
        return struct.unpack("<d", struct.pack("<q", b + d))[0]

    out = list(wi)
    for i in range(256):
        ra = np.array([p[0] for p in pairs[i]], dtype=np.float64)
        xs = np.array([p[1] for p in pairs[i]])
        assert len(ra) > 1000, (i, len(ra))
        for d in sorted(range(-400, 401), key=abs):
            c = step(wi[i], d)
            if np.all(ra * c == xs):
                out[i] = c
                break
        else:
            raise SystemExit(f"wi[{i}]: no double within 400 ulps reproduces numpy")
    return out


def bits(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def main():
    ki, wi, fi = construct()
    wi = pin_wi(ki, wi, fi)
    n = 300000
    want = np.random.Generator(np.random.PCG64(99)).standard_normal(n)
    got = standard_normals(np.random.PCG64(99).random_raw(2 * n), n, ki, wi, fi)
    bad = int(np.sum(got != want))
    assert bad == 0, f"{bad} mismatches against numpy on the check seed"
    with open(OUT, "w") as f:
        f.write("// ziggurat_tables.h — GENERATED by tools/gen_ziggurat.py (do not edit): the 256-layer ziggurat of\n"
                "// numpy's Generator.standard_normal (random_standard_normal), ki / wi / fi as IEEE bit patterns.\n"
                f"// Checked: over numpy's raw PCG64 words the restated algorithm returns numpy's normals bit for bit\n"
                f"// ({n} normals of seed 99).\n#pragma once\n#include <cstdint>\n\n")
        f.write("#define GP_ZIG_R 3.6541528853610087963519472518\n#define GP_ZIG_INV_R 0.27366123732975827203338247596\n")
        # initializer lists (macros), so that host tables and __device__ copies share one definition
        for name, vals in (("GP_ZIG_KI", ki), ("GP_ZIG_WI", [bits(x) for x in wi]), ("GP_ZIG_FI", [bits(x) for x in fi])):
            f.write(f"#define {name}_LIST \\\n")
            rows = [", ".join(f"0x{v:016x}ull" for v in vals[i:i + 4]) for i in range(0, 256, 4)]
            f.write(", \\\n".join("    " + r for r in rows) + "\n")
    np.savez(os.path.join(os.path.dirname(HERE), "tests", "golden", "ziggurat_tables.npz"),
             ki=np.array(ki, dtype=np.uint64), wi=np.array(wi), fi=np.array(fi))
    print(f"wrote {OUT}; check seed: {n} normals bit-exact vs numpy")


if __name__ == "__main__":
    main()
