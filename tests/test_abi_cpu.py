"""CPU tests of the C ABI library: it loads, exports every symbol include/gym_po_amd.h declares,
and its host-only logic (numpy seeding, taxi reset law) matches numpy / the oracle. No GPU
compute is issued here."""
import ctypes
import os
import re

import numpy as np
import pytest

from fixtures import GOLDEN_DIR, load_index

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gym_po_amd.h")


def _lib():
    from gym_po_amd import _lib as L
    return L


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gp_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = _lib()
    lib = L.lib()
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"{n} missing from libgympo_amd.so"
        assert n in L.SIGNATURES, f"{n} not bound in _lib.SIGNATURES"
    assert lib.gp_abi_version() == 1


def test_no_cpu_fallback_in_product():
    """The product package must not import the oracle or any CPU stand-in."""
    pkg = os.path.join(ROOT, "gym-po-taxi_amd", "gym_po_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r"#.*", "", src).replace('"""', ""), f


@pytest.mark.parametrize("seed,spawn", [(0, ()), (1, ()), (12345, ()), (2 ** 40 + 7, ()), (2 ** 100 + 3, ()),
                                        (7, (3,)), (9, (0, 5))])
def test_native_seeding_matches_numpy(seed, spawn):
    L = _lib()
    words = L.int_to_u32_words(seed)
    st = (ctypes.c_uint64 * 6)()
    w = (ctypes.c_uint32 * len(words))(*words)
    sk = (ctypes.c_uint32 * max(1, len(spawn)))(*(list(spawn) or [0]))
    assert L.lib().gp_pcg64_seed_state(w, len(words), sk, len(spawn), st) == 0
    ref = np.random.PCG64(np.random.SeedSequence(seed, spawn_key=spawn)).state
    assert (st[0] << 64 | st[1]) == ref["state"]["state"]
    assert (st[2] << 64 | st[3]) == ref["state"]["inc"]
    assert st[4] == ref["has_uint32"]


@pytest.mark.parametrize("m,n", [(300, 500), (660, 1280), (12, 20)])
def test_native_taxi_reset_law_matches_oracle(m, n):
    from oracle.taxi import argmax_multinomial_distribution
    L = _lib()
    out = (ctypes.c_double * m)()
    assert L.lib().gp_argmax_multinomial_distribution(m, n, out) == m
    q = np.array(out[:])
    p = argmax_multinomial_distribution(m, n)
    np.testing.assert_allclose(q, p, rtol=1e-10, atol=1e-16)
    assert abs(q.sum() - 1) < 1e-9


def test_taxi_reset_law_matches_reference_histogram():
    """Chi-square of the exact law against 2M reference resets (tests/golden/taxi_reset_hist.npz)."""
    from oracle.taxi import TaxiOracle, argmax_multinomial_distribution
    meta = load_index()["taxi_reset_hist"]
    h = np.load(os.path.join(GOLDEN_DIR, meta["file"]))
    for name in ("TAXI", "EXTENDED"):
        t = TaxiOracle(1, map=name)
        p = argmax_multinomial_distribution(len(t.valid_states), t.ns)
        cnt = h[name][t.valid_states]
        assert cnt.sum() == h[name].sum()  # invalid states never win the argmax
        e = p * cnt.sum()
        chi2 = float(((cnt - e) ** 2 / e).sum())
        dof = len(p) - 1
        assert chi2 < dof + 5 * np.sqrt(2 * dof), (name, chi2, dof)
