"""ORACLE / TEST INFRASTRUCTURE — Philox4x32-R and Lemire bounded draws in numpy (vectorised).

Restates the counter-based generator of the device's `rng_mode="philox"` (gym-po-taxi_amd/csrc/
gp_common.h: philox4x32<R>, philox4x32_10, lemire_value) so that build-defined envs (grid Ant-Tag) can be checked
bit-exactly in philox mode. Philox4x32-R is the published algorithm of Salmon et al. (SC'11,
"Parallel random numbers: as easy as 1, 2, 3"): R rounds of two 32x32->64 multiplies with the
multipliers 0xD2511F53 / 0xCD9E8D57 and the Weyl key increments 0x9E3779B9 / 0xBB67AE85. R = 10 (Random123's
default; pinned by its known-answer vectors, tests/test_oracle_extra.py) in every philox-mode kernel; R = 7 (the
paper's Crush-resistant minimum) is a build option of C-ROOMS (csrc/crooms.hip CR_PHILOX_ROUNDS): the same round
function with fewer iterations, both checked against the device header's host copy (tests/test_philox_cpu.py).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this module.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Counters (uint32 arrays / scalars, broadcast) and key -> 4 uint32 arrays."""
    return philox4x32(c0, c1, c2, c3, k0, k1, rounds=10)


def philox4x32(c0, c1, c2, c3, k0, k1, rounds=10):
    """Philox4x32-`rounds`: counters (uint32 arrays / scalars, broadcast) and key -> 4 uint32 arrays."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & MASK32 for c in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for _ in range(rounds):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        n0 = hi1 ^ c1 ^ np.uint64(k0)
        n2 = hi0 ^ c3 ^ np.uint64(k1)
        c0, c1, c2, c3 = n0, lo1, n2, lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return tuple(x.astype(np.uint32) for x in (c0, c1, c2, c3))


def lemire_value(word, n):
    """floor(word * n / 2^32) (the device's multiply-shift bounded draw)."""
    return ((np.asarray(word, dtype=np.uint64) * np.uint64(n)) >> np.uint64(32)).astype(np.int64)


def philox_key(seed, spawn_key=()):
    """The device key for a seed: SeedSequence(seed, spawn_key).generate_state(5, uint64)[4] split in
    two uint32 words (api.hip gp_seed_words)."""
    w = np.random.SeedSequence(seed, spawn_key=tuple(spawn_key)).generate_state(5, np.uint64)[4]
    w = int(w)
    return w & 0xFFFFFFFF, w >> 32


def env_step_words(B, step, tag, key):
    """The 4 words of counter (env, step, tag) for env = 0..B-1."""
    env = np.arange(B, dtype=np.uint64)
    return philox4x32_10(env, step & 0xFFFFFFFF, step >> 32, tag, *key)
