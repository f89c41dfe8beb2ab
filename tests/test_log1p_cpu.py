"""The C-ROOMS exact mode's ziggurat tail log1p equals the C library's (no GPU needed).

numpy's random_standard_normal draws a tail normal as r + x with x = -log1p(-u1) / r, accepted when
-2 log1p(-u2) > x^2 (numpy/random/src/distributions/distributions.c); npy_log1p is libm's log1p (glibc here),
not the SIMD np.log1p ufunc (which differs from libm in ~1% of last bits). csrc/crooms.hip restates glibc's
__log1p (sysdeps/ieee754/dbl-64/s_log1p.c) operation for operation; its host copy (same source, gp_zig_log1p_neg)
is compared with libm's log1p bit for bit on the 2^-53 grid numpy's next_double produces, over every branch.
"""
import ctypes

import numpy as np


def _libm_log1p(x):
    libm = ctypes.CDLL("libm.so.6")
    f = libm.log1p
    f.restype, f.argtypes = ctypes.c_double, [ctypes.c_double]
    return np.array([f(float(v)) for v in x])


def _ours(u):
    from gym_po_amd import _lib as L
    u = np.ascontiguousarray(u, np.float64)
    out = np.empty_like(u)
    dp = ctypes.POINTER(ctypes.c_double)
    L.check(L.lib().gp_zig_log1p_neg(u.ctypes.data_as(dp), out.ctypes.data_as(dp), u.size), "gp_zig_log1p_neg")
    return out


def test_tail_log1p_equals_libm_bit_for_bit():
    rng = np.random.default_rng(7)
    k = rng.integers(1, 2 ** 53, 150_000, dtype=np.uint64) >> rng.integers(0, 53, 150_000).astype(np.uint64)
    grid = np.concatenate([
        k.astype(np.float64) * 2.0 ** -53,                        # log-uniform over [2^-53, 1)
        rng.integers(0, 2 ** 53, 50_000, dtype=np.uint64).astype(np.float64) * 2.0 ** -53,  # numpy's next_double
        np.arange(0, 3000) * 2.0 ** -53,                          # |x| < 2^-29 branch, incl. u = 0
        1.0 - np.arange(1, 3000) * 2.0 ** -53,                    # u -> 1
        0.5 + np.arange(-3000, 3000) * 2.0 ** -53,                # |f| < 2^-20 after reduction
        0.75 + np.arange(-3000, 3000) * 2.0 ** -53])
    hw = (np.uint64(0x3FD2BEC3) << np.uint64(32)) | rng.integers(0, 2 ** 32, 20_000, dtype=np.uint64)
    edge = np.round(hw.view(np.float64) * 2.0 ** 53) * 2.0 ** -53  # fdlibm's k = 0 / k != 0 boundary (0xbfd2bec3)
    u = np.concatenate([grid, edge])
    got, want = _ours(u), _libm_log1p(-u)
    bad = np.flatnonzero(got.view(np.uint64) != want.view(np.uint64))
    assert bad.size == 0, f"{bad.size} mismatches, e.g. u={u[bad[:3]]}"
