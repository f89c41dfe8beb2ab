"""oracle/philox.py's Philox4x32-R equals the device header's (gp_common.h philox4x32<R>, compiled for the host:
gp_philox_blocks) for R = 10 (every philox-mode kernel; also pinned to Random123's known-answer vectors,
tests/test_oracle_extra.py) and R = 7 (a C-ROOMS build option, csrc/crooms.hip CR_PHILOX_ROUNDS)."""
import ctypes

import numpy as np
import pytest

from oracle.philox import philox4x32


def _device_header(ctr, rounds):
    from gym_po_amd import _lib as L
    ctr = np.ascontiguousarray(ctr, np.uint32)
    out = np.empty((ctr.shape[0], 4), np.uint32)
    p = ctypes.POINTER(ctypes.c_uint32)
    L.check(L.lib().gp_philox_blocks(ctr.ctypes.data_as(p), rounds, out.ctypes.data_as(p), ctypes.c_int64(ctr.shape[0])),
            "gp_philox_blocks")
    return out


@pytest.mark.parametrize("rounds", [7, 10])
def test_oracle_equals_device_header(rounds):
    rng = np.random.default_rng(rounds)
    ctr = rng.integers(0, 1 << 32, (100000, 6), dtype=np.uint64).astype(np.uint32)
    ctr[::2, 2] = 0                                            # step_hi: 0 in practice
    ctr[1::3, 0] = np.arange(ctr[1::3].shape[0], dtype=np.uint32)  # env indices
    got = _device_header(ctr, rounds)
    # the oracle takes scalar keys: the first 2000 counters one by one, each with its own key
    want = np.array([np.asarray(philox4x32(*ctr[i, :4], int(ctr[i, 4]), int(ctr[i, 5]), rounds=rounds)).ravel()
                     for i in range(2000)], np.uint32)
    np.testing.assert_array_equal(got[:2000], want)
    # and vectorised over counters under one key
    k0, k1 = int(ctr[0, 4]), int(ctr[0, 5])
    ctr[:, 4], ctr[:, 5] = k0, k1
    got = _device_header(ctr, rounds)
    want = np.stack(philox4x32(*(ctr[:, j] for j in range(4)), k0, k1, rounds=rounds), 1)
    np.testing.assert_array_equal(got, want)


def test_seven_rounds_differ_from_ten():
    ctr = np.array([[1, 2, 0, 3, 4, 5]], np.uint32)
    assert not np.array_equal(_device_header(ctr, 7), _device_header(ctr, 10))
