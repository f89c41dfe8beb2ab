"""ORACLE / TEST INFRASTRUCTURE — pure-Python restatement of the RNG arithmetic the reference's
hot path consumes. Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may
import anything under `oracle/`; the product (`gym-po-taxi_amd/`) never does.

The reference draws every random number from one `numpy.random.Generator(PCG64(SeedSequence(s)))`
per env object (gymnasium `seeding.np_random`, called from `Env.reset(seed=...)`;
`msrooms.py:376`, `rooms.py:184`, `crooms.py:246-249`, `extended_taxi.py:239`). numpy is an
un-vendored third-party dependency (`setup.py:39`, `numpy>=1.23`, container: 2.2.6); its published
algorithms restated here (NEP 19 gives no cross-version stream guarantee, so fixtures record the
version):

* SeedSequence (`numpy/random/bit_generator.pyx`): entropy -> uint32 words, hashmix pool of 4,
  generate_state(4, uint64).
* PCG64 = pcg_setseq_128 XSL-RR 128/64 (`numpy/random/src/pcg64/pcg64.h`): step, then output
  rotr64(hi ^ lo, state >> 122). Seeding: state=0; inc=(initseq<<1)|1; step; state+=initstate; step.
* next_uint32 buffering (`pcg64.h` pcg64_next32): if has_uint32 return the stored high half;
  else draw a u64, keep its high half, return the low half. next_uint64 does NOT touch the buffer.
* Generator.random(n) = ((next_u64 >> 11) * 2**-53) per element (`distributions.c` next_double).
* Generator.integers(0, m) / choice(m, b) with 32-bit range = Lemire bounded draw on next_uint32
  with rejection (`distributions.c` buffered_bounded_lemire_uint32).

Every function here is checked against numpy itself in tests/test_oracle_rng.py.
"""
MASK64 = (1 << 64) - 1
MASK128 = (1 << 128) - 1
PCG_MULT = (0x2360ED051FC65DA4 << 64) | 0x4385DF649FCCF645

# ---- SeedSequence (numpy/random/bit_generator.pyx) -------------------------------------------
_INIT_A = 0x43B0D7E5
_MULT_A = 0x931E8875
_INIT_B = 0x8B51F9DD
_MULT_B = 0x58F38DED
_MIX_MULT_L = 0xCA01F9DD
_MIX_MULT_R = 0x4973F715
_XSHIFT = 16
_M32 = 0xFFFFFFFF
POOL_SIZE = 4


def _int_to_u32_words(x):
    if x < 0:
        raise ValueError("negative entropy")
    words = []
    while True:
        words.append(x & _M32)
        x >>= 32
        if x == 0:
            break
    return words


def seed_sequence_pool(entropy, spawn_key=()):
    hash_const = _INIT_A

    def hashmix(value):
        nonlocal hash_const
        value = (value ^ hash_const) & _M32
        hash_const = (hash_const * _MULT_A) & _M32
        value = (value * hash_const) & _M32
        value ^= value >> _XSHIFT
        return value

    def mix(x, y):
        result = ((_MIX_MULT_L * x) & _M32) - ((_MIX_MULT_R * y) & _M32)
        result &= _M32
        result ^= result >> _XSHIFT
        return result

    run_entropy = _int_to_u32_words(entropy)
    if spawn_key:
        # numpy pads the entropy to the pool size before appending the spawn key
        if len(run_entropy) < POOL_SIZE:
            run_entropy = run_entropy + [0] * (POOL_SIZE - len(run_entropy))
        for k in spawn_key:
            run_entropy += _int_to_u32_words(k)
    mixer = [0] * POOL_SIZE
    n = len(run_entropy)
    for i in range(POOL_SIZE):
        mixer[i] = hashmix(run_entropy[i]) if i < n else hashmix(0)
    for i_src in range(POOL_SIZE):
        for i_dst in range(POOL_SIZE):
            if i_src != i_dst:
                mixer[i_dst] = mix(mixer[i_dst], hashmix(mixer[i_src]))
    for i_src in range(POOL_SIZE, n):
        for i_dst in range(POOL_SIZE):
            mixer[i_dst] = mix(mixer[i_dst], hashmix(run_entropy[i_src]))
    return mixer


def seed_sequence_generate_state_u64(entropy, n_words64, spawn_key=()):
    pool = seed_sequence_pool(entropy, spawn_key)
    hash_const = _INIT_B
    out32 = []
    for i in range(2 * n_words64):
        data_val = pool[i % POOL_SIZE]
        data_val ^= hash_const
        hash_const = (hash_const * _MULT_B) & _M32
        data_val = (data_val * hash_const) & _M32
        data_val ^= data_val >> _XSHIFT
        out32.append(data_val)
    return [out32[2 * i] | (out32[2 * i + 1] << 32) for i in range(n_words64)]


# ---- PCG64 ----------------------------------------------------------------------------------
def pcg_output(state):
    hi = state >> 64
    lo = state & MASK64
    x = (hi ^ lo) & MASK64
    rot = state >> 122
    return ((x >> rot) | (x << ((64 - rot) & 63))) & MASK64


def pcg_advance_params(delta, inc, mult=PCG_MULT):
    """(A, C) with state_{n+delta} = A*state_n + C (mod 2^128) — pcg_advance_lcg_128."""
    acc_mult, acc_plus = 1, 0
    cur_mult, cur_plus = mult, inc
    delta &= MASK128
    while delta > 0:
        if delta & 1:
            acc_mult = (acc_mult * cur_mult) & MASK128
            acc_plus = (acc_plus * cur_mult + cur_plus) & MASK128
        cur_plus = ((cur_mult + 1) * cur_plus) & MASK128
        cur_mult = (cur_mult * cur_mult) & MASK128
        delta >>= 1
    return acc_mult, acc_plus


class PCG64:
    """Python PCG64 with numpy's uint32 buffer. Checked bit-for-bit against numpy."""

    def __init__(self, state, inc, has_uint32=0, uinteger=0):
        self.state = state & MASK128
        self.inc = inc & MASK128
        self.has_uint32 = has_uint32
        self.uinteger = uinteger

    @classmethod
    def from_seed(cls, entropy, spawn_key=()):
        w = seed_sequence_generate_state_u64(entropy, 4, spawn_key)
        initstate = (w[0] << 64) | w[1]
        initseq = (w[2] << 64) | w[3]
        inc = ((initseq << 1) | 1) & MASK128
        state = 0
        state = (state * PCG_MULT + inc) & MASK128
        state = (state + initstate) & MASK128
        state = (state * PCG_MULT + inc) & MASK128
        return cls(state, inc)

    @classmethod
    def from_numpy(cls, bitgen):
        st = bitgen.state
        return cls(st["state"]["state"], st["state"]["inc"], st["has_uint32"], st["uinteger"])

    def to_numpy_state(self):
        return {"bit_generator": "PCG64", "state": {"state": self.state, "inc": self.inc},
                "has_uint32": self.has_uint32, "uinteger": self.uinteger}

    def next64(self):
        self.state = (self.state * PCG_MULT + self.inc) & MASK128
        return pcg_output(self.state)

    def next32(self):
        if self.has_uint32:
            self.has_uint32 = 0
            return self.uinteger
        v = self.next64()
        self.has_uint32 = 1
        self.uinteger = v >> 32
        return v & 0xFFFFFFFF

    def advance(self, delta):
        a, c = pcg_advance_params(delta, self.inc)
        self.state = (a * self.state + c) & MASK128

    def random_k53(self):
        """Integer k with Generator.random() == k * 2**-53."""
        return self.next64() >> 11

    def lemire32(self, rng_excl):
        """Generator.integers(0, rng_excl) for rng_excl <= 2**32 - 1 (one bounded draw)."""
        rng = rng_excl - 1
        m = self.next32() * rng_excl
        leftover = m & 0xFFFFFFFF
        if leftover < rng_excl:
            threshold = (0xFFFFFFFF - rng) % rng_excl
            while leftover < threshold:
                m = self.next32() * rng_excl
                leftover = m & 0xFFFFFFFF
        return m >> 32


def lemire_threshold(rng_excl):
    return (0xFFFFFFFF - (rng_excl - 1)) % rng_excl
