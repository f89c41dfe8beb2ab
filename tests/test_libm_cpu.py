"""The device restatement of the C library's exp (csrc/gp_libm.h) equals this machine's libm exp bit for bit.

numpy's random_binomial_inversion computes q^n as exp(n * log(q)) with libm (numpy/random/src/distributions/
distributions.c), and so does the ziggurat's wedge test with exp(-x^2 / 2); an exact-stream device path must get
the same doubles to take the same branches. glibc 2.35 (this image) runs __exp_fma on CPUs with FMA (ifunc), the
same e_exp.c built with -mfma. The host copy of the restatement (gp_exp_libm, the same header the kernels include)
is compared over the ranges those callers feed it, the whole normal range, and the special cases.
"""
import ctypes

import numpy as np
import pytest


def _libm_exp(x):
    libm = ctypes.CDLL("libm.so.6")
    f = libm.exp
    f.restype, f.argtypes = ctypes.c_double, [ctypes.c_double]
    return np.array([f(float(v)) for v in x])


def _ours(x, fma):
    from gym_po_amd import _lib as L
    x = np.ascontiguousarray(x, np.float64)
    out = np.empty_like(x)
    dp = ctypes.POINTER(ctypes.c_double)
    L.check(L.lib().gp_exp_libm(x.ctypes.data_as(dp), out.ctypes.data_as(dp), ctypes.c_int64(x.size), fma),
            "gp_exp_libm")
    return out


def _cpu_has_fma():
    try:
        return " fma " in " " + open("/proc/cpuinfo").read().replace("\n", " ") + " "
    except OSError:
        return False


@pytest.mark.skipif(not _cpu_has_fma(), reason="glibc selects its FMA build only on CPUs with FMA")
def test_exp_equals_libm_bit_for_bit():
    rng = np.random.default_rng(11)
    n = np.arange(1, 4097, dtype=np.float64)
    q = 1.0 - rng.uniform(0, 0.5, 4096)
    x = np.concatenate([
        n * np.log(q),                                   # binomial inversion: exp(n log q), p n <= 30
        rng.uniform(-60.0, 0.0, 150_000),
        -0.5 * rng.uniform(0, 3.7, 100_000) ** 2,        # ziggurat wedge: exp(-x^2 / 2)
        rng.uniform(-745.2, 709.78, 100_000),            # the whole finite range, incl. both special cases
        rng.uniform(-760.0, -708.0, 20_000),             # subnormal results
        np.array([0.0, -0.0, 1e-300, -1e-300, 2.0 ** -60, -(2.0 ** -55), 709.79, -746.0, np.inf, -np.inf]),
    ])
    got, want = _ours(x, 1), _libm_exp(x)
    bad = np.flatnonzero(got.view(np.uint64) != want.view(np.uint64))
    assert bad.size == 0, f"{bad.size} mismatches, e.g. x={x[bad[:3]]}"


def test_host_variant_detection():
    """gp_exp_host_variant() names the build this machine's libm runs (the exact-stream kernels use it): the FMA
    build on CPUs with FMA (glibc's ifunc), the plain build otherwise."""
    from gym_po_amd import _lib as L
    v = L.lib().gp_exp_host_variant()
    assert v in (0, 1)
    assert v == (1 if _cpu_has_fma() else 0)
    rng = np.random.default_rng(3)
    x = rng.uniform(-60.0, 20.0, 50_000)
    assert np.array_equal(_ours(x, v).view(np.uint64), _libm_exp(x).view(np.uint64))


def test_plain_variant_is_a_faithful_exp():
    """The non-FMA restatement (what a host without FMA runs) is self-consistent: within one ulp of the FMA build
    everywhere, differing from it on some inputs (so the two are really distinct code paths), and exact on the
    special cases."""
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(-745.0, 709.7, 200_000), -0.5 * rng.uniform(0, 3.7, 50_000) ** 2])
    a, b = _ours(x, 1), _ours(x, 0)
    ulp = np.abs(a.view(np.int64) - b.view(np.int64))
    assert ulp.max() <= 1
    assert (ulp == 1).sum() > 0
    sp = np.array([0.0, -0.0, np.inf, -np.inf, 709.79, -746.0])
    np.testing.assert_array_equal(_ours(sp, 0), _ours(sp, 1))
