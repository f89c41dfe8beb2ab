"""Host-side action validation (no GPU): out-of-range discrete actions given as host arrays raise exactly the
IndexError numpy raises in the reference's `action_matrix[action]` (msrooms.py:400, rooms.py:208) /
`ACTIONS_YX[actions]` (extended_taxi.py:248); negatives in [-n, 0) wrap and pass."""
import numpy as np
import pytest


def _env(n, dtype="int32"):
    from gym_po_amd.core import NativeVecEnv
    from gym_po_amd.spaces import Box, Discrete
    e = NativeVecEnv.__new__(NativeVecEnv)
    e.single_action_space = Discrete(n) if n else Box(-1.0, 1.0, (2,))
    e._action_dtype = dtype
    return e


@pytest.mark.parametrize("n", [4, 5, 8])
def test_out_of_range_host_actions_raise_numpys_index_error(n):
    e = _env(n)
    e._check_host_actions(np.array([-n, n - 1, 0]))
    table = np.zeros((n, n))
    for bad in (n, -n - 1, 10 * n):
        with pytest.raises(IndexError) as ours:
            e._check_host_actions(np.array([0, bad, 1]))
        with pytest.raises(IndexError) as ref:
            table[np.array([0, bad, 1])]
        assert str(ours.value) == str(ref.value)


def test_continuous_actions_not_range_checked():
    _env(None, "float32")._check_host_actions(np.array([[5.0, -7.0]]))


@pytest.mark.parametrize("n", [4, 8])
def test_first_offending_action_named_like_numpy(n):
    e = _env(n)
    table = np.zeros((n, n))
    a = np.array([0, -n - 3, 2 * n, 1])  # an early too-negative index, a later too-large one
    with pytest.raises(IndexError) as ours:
        e._check_host_actions(a)
    with pytest.raises(IndexError) as ref:
        table[a]
    assert str(ours.value) == str(ref.value)


def test_float_host_actions_raise_like_numpy():
    e = _env(4)
    table = np.zeros((4, 4))
    a = np.array([0.0, 1.0])
    with pytest.raises(IndexError) as ours:
        e._check_host_actions(a)
    with pytest.raises(IndexError) as ref:
        table[a]
    assert str(ours.value) == str(ref.value)
