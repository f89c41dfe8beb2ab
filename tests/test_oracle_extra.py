"""CPU checks of the oracle pieces that have no reference fixture: Philox4x32-10 (pinned to the
published Random123 known-answer vectors) and the build-defined grid Ant-Tag spec."""
import pytest
import numpy as np

from oracle.anttag import AntTagOracle
from oracle.philox import philox4x32_10, philox_key

# Random123 kat_vectors, philox4x32_10: (counter, key) -> output
KAT = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
       ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
       ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
        (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]


def test_philox_known_answers():
    for c, k, out in KAT:
        got = philox4x32_10(*c, *k)
        assert tuple(int(x) for x in got) == out


def test_philox_key_is_seed_sequence_word4():
    k0, k1 = philox_key(7)
    w = int(np.random.SeedSequence(7).generate_state(5, np.uint64)[4])
    assert (k0, k1) == (w & 0xFFFFFFFF, w >> 32)


def test_anttag_reset_law_and_rules():
    B = 1 << 16
    ora = AntTagOracle(B)
    key = philox_key(3)
    ora.reset(ora.philox_draws(0, key))
    ay, ax = np.divmod(ora.ant, 10)
    ty, tx = np.divmod(ora.target, 10)
    assert ((ay - ty) ** 2 + (ax - tx) ** 2 > 25).all()
    # ant cells uniform over the 100 cells
    c = np.bincount(ora.ant, minlength=100)
    assert c.min() > 0.8 * B / 100 and c.max() < 1.2 * B / 100
    rng = np.random.default_rng(0)
    for t in range(50):
        a0, t0 = ora.ant.copy(), ora.target.copy()
        o, r, d, tr = ora.step(rng.integers(0, 5, B), ora.philox_draws(t + 1, key))
        moved = ~(d | tr)
        # the target moves at most one (8-connected) cell and stays in the arena
        dy = np.abs(ora.target[moved] // 10 - t0[moved] // 10)
        dx = np.abs(ora.target[moved] % 10 - t0[moved] % 10)
        assert (dy <= 1).all() and (dx <= 1).all()
        # invisible targets are reported as -1
        vis = o[:, 2] >= 0
        d2 = (o[:, 0] - ora.target // 10) ** 2 + (o[:, 1] - ora.target % 10) ** 2
        assert (d2[vis] < 9).all() and (d2[~vis] >= 9).all()
        assert (r[d] == 1.0).all() and (r[~d] == 0.0).all()


@pytest.mark.parametrize("seed", [0, 99, 31337])
def test_ziggurat_oracle_matches_numpy(seed):
    """oracle.ziggurat restates numpy's random_standard_normal: over numpy's raw PCG64 words it returns
    numpy's normals bit for bit and consumes exactly the words numpy consumed."""
    from oracle.ziggurat import standard_normals
    n = 60000
    g = np.random.Generator(np.random.PCG64(seed))
    want = g.standard_normal(n)
    words = np.random.PCG64(seed).random_raw(2 * n)
    got, used = standard_normals(words, n)
    assert np.array_equal(got, want)
    ref = np.random.PCG64(seed)
    ref.advance(used)
    assert ref.state == g.bit_generator.state
