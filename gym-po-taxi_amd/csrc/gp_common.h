// gp_common.h — shared host/device helpers: 128-bit PCG64 arithmetic (numpy-compatible),
// Philox4x32-10, status packing for the decoupled-lookback reset scan, error plumbing.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned __int128 u128;

#define GP_HD __host__ __device__ __forceinline__

// ---------------------------------------------------------------- PCG64 (XSL-RR 128/64) ----
// numpy/random/src/pcg64/pcg64.h: state = state * MULT + inc; out = rotr64(hi ^ lo, state >> 122).
static constexpr uint64_t PCG_MULT_HI = 0x2360ED051FC65DA4ULL;
static constexpr uint64_t PCG_MULT_LO = 0x4385DF649FCCF645ULL;

GP_HD u128 pcg_mult() { return ((u128)PCG_MULT_HI << 64) | PCG_MULT_LO; }
GP_HD u128 mk128(uint64_t hi, uint64_t lo) { return ((u128)hi << 64) | lo; }
GP_HD uint64_t hi64(u128 x) { return (uint64_t)(x >> 64); }
GP_HD uint64_t lo64(u128 x) { return (uint64_t)x; }

GP_HD uint64_t pcg_output(u128 s) {
  uint64_t x = hi64(s) ^ lo64(s);
  unsigned r = (unsigned)(s >> 122);
  return (x >> r) | (x << ((64u - r) & 63u));
}

// An affine jump s -> A*s + C (mod 2^128). Jumps compose: (A2,C2)o(A1,C1) = (A2*A1, A2*C1 + C2).
struct PcgJump {
  uint64_t a_hi, a_lo, c_hi, c_lo;
};

GP_HD u128 apply_jump(const PcgJump& j, u128 s) { return mk128(j.a_hi, j.a_lo) * s + mk128(j.c_hi, j.c_lo); }

// pcg_advance_lcg_128: (A, C) for `delta` LCG steps with increment `inc`.
static inline PcgJump pcg_jump_params(u128 delta, u128 inc) {
  u128 acc_mult = 1, acc_plus = 0, cur_mult = pcg_mult(), cur_plus = inc;
  while (delta > 0) {
    if (delta & 1) {
      acc_mult *= cur_mult;
      acc_plus = acc_plus * cur_mult + cur_plus;
    }
    cur_plus = (cur_mult + 1) * cur_plus;
    cur_mult *= cur_mult;
    delta >>= 1;
  }
  return PcgJump{hi64(acc_mult), lo64(acc_mult), hi64(acc_plus), lo64(acc_plus)};
}

// Radix-64 jump tables: level L, digit d -> jump by d * 64^L. JT_LEVELS levels cover 2^30 steps.
#define JT_LEVELS 5
#define JT_RADIX_BITS 6
#define JT_RADIX 64

// Jump state s by n (< 2^30) LCG steps using the tables (gathers from global memory, L1/L2 hot), one level's
// entry at a time (few live registers: the grid kernels' rare paths call this inside register-tight loops).
__device__ __forceinline__ u128 pcg_jump(const PcgJump* __restrict__ jt, u128 s, uint32_t n) {
#pragma unroll
  for (int L = 0; L < JT_LEVELS; ++L) {
    const uint32_t d = (n >> (JT_RADIX_BITS * L)) & (JT_RADIX - 1);
    if (d) s = apply_jump(jt[L * JT_RADIX + d], s);
  }
  return s;
}
// The same with every level's entry loaded up front (independent loads in flight together, then applied in
// order): for kernels with registers to spare (the C-ROOMS exact mode's draw calls). In the fused grid kernel
// the 40 extra live VGPRs of this form made every step ~40% slower (K = 128: 4.72 -> 6.67 us/step).
__device__ __forceinline__ u128 pcg_jump_ilp(const PcgJump* __restrict__ jt, u128 s, uint32_t n) {
  PcgJump e[JT_LEVELS];
#pragma unroll
  for (int L = 0; L < JT_LEVELS; ++L) e[L] = jt[L * JT_RADIX + ((n >> (JT_RADIX_BITS * L)) & (JT_RADIX - 1))];
#pragma unroll
  for (int L = 0; L < JT_LEVELS; ++L)
    if ((n >> (JT_RADIX_BITS * L)) & (JT_RADIX - 1)) s = apply_jump(e[L], s);
  return s;
}

__device__ __forceinline__ u128 pcg_step(u128 s, u128 inc) { return s * pcg_mult() + inc; }

// Lemire 32-bit bounded draw acceptance (numpy distributions.c buffered_bounded_lemire_uint32):
// rejected iff (word * n mod 2^32) < (2^32 - n) % n.
GP_HD bool lemire_rejected(uint32_t word, uint32_t n, uint32_t threshold) {
  return (uint32_t)((uint64_t)word * n) < threshold;
}
GP_HD uint32_t lemire_value(uint32_t word, uint32_t n) { return (uint32_t)(((uint64_t)word * n) >> 32); }
static inline uint32_t lemire_threshold(uint32_t n) { return (uint32_t)((0xFFFFFFFFu - (n - 1)) % n); }

// ---------------------------------------------------------------- Philox4x32-10 ----
struct Philox4 {
  uint32_t x[4];
};
// a ^ b ^ c: ONE gfx950 v_bitop3_b32 (truth table 0x96) on the device, where the compiler emits two v_xor_b32
// (gfx950 has no v_xor3_b32); Philox4x32-10 spends 2 of its 3 VALU ops per output word per round here.
GP_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}
// Philox4x32-R (Salmon et al. 2011, "Parallel random numbers: as easy as 1, 2, 3"); R = 10 is Random123's default
// (every philox-mode kernel), R = 7 the fewest rounds the paper reports Crush-resistant (a C-ROOMS build option,
// csrc/crooms.hip CR_PHILOX_ROUNDS).
template <int R>
GP_HD Philox4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    uint64_t p0 = (uint64_t)M0 * c0, p1 = (uint64_t)M1 * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = xor3(hi1, c1, k0), n2 = xor3(hi0, c3, k1);
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += W0; k1 += W1;
  }
  Philox4 r; r.x[0] = c0; r.x[1] = c1; r.x[2] = c2; r.x[3] = c3;
  return r;
}
GP_HD Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  return philox4x32<10>(c0, c1, c2, c3, k0, k1);
}

// ---------------------------------------------------------------- lookback status words ----
// 64-bit status per block: [63:62] flag (0 = not ready, 1 = aggregate, 2 = inclusive prefix),
// [61] rejection-seen bit, [31:0] reset count. Written/read as agent-scope atomics: the word IS
// the hand-off (MI355X_MICROARCH.md, Guideline 16 R2 granule form: one aligned 8-B sc1 store).
#define ST_FLAG_X 0ull
#define ST_FLAG_A 1ull
#define ST_FLAG_P 2ull
GP_HD uint64_t st_pack(uint64_t flag, uint32_t rej, uint32_t count) {
  return (flag << 62) | ((uint64_t)(rej & 1u) << 61) | (uint64_t)count;
}
GP_HD uint64_t st_flag(uint64_t s) { return s >> 62; }
GP_HD uint32_t st_rej(uint64_t s) { return (uint32_t)(s >> 61) & 1u; }
GP_HD uint32_t st_count(uint64_t s) { return (uint32_t)s; }

// ---------------------------------------------------------------- error plumbing ----
// Per-handle device error word (GridCtl::err, the other kinds' `derr`): kernels OR bits into it,
// gp_check / gp_metrics turn a nonzero word into GP_E_DEVICE. Sticky until the handle is re-seeded.
#define GP_DERR_TIMEOUT 1u  // a persistent kernel's cross-block wait gave up (blocks not co-resident)
#define GP_DERR_ACTION 2u   // an action outside [-n, n): the reference raises IndexError
                            // (msrooms.py:400 action_matrix[action], extended_taxi.py:248 ACTIONS_YX[actions])
#define GP_DERR_STREAM 4u   // C-ROOMS exact mode: a numpy normal needed more words than one window holds
#define GP_DERR_OVERFLOW 8u // windowed grid kernel slow path: more rejected choice() words than it can list
#define GP_DERR_BTPE 16u    // Taxi numpy mode: a multinomial reset needed numpy's BTPE binomial (p n > 30) or an
                            // inversion did not end, neither of which the device walker restates
// numpy indexing of an n-row table accepts a in [-n, n) (negatives wrap); anything else raises.
__device__ __forceinline__ bool action_out_of_range(int a, int n) { return (uint32_t)(a + n) >= (uint32_t)(2 * n); }
__device__ __forceinline__ void flag_bad_action(uint32_t* derr) { atomicOr(derr, GP_DERR_ACTION); }
const char* gp_derr_text(uint32_t flags);  // api.hip: human-readable description of the set bits
void gp_set_error(const char* fmt, ...);
#define GP_HIP_CHECK(x)                                                                        \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      gp_set_error("%s:%d %s -> %s", __FILE__, __LINE__, #x, hipGetErrorString(e_));           \
      return GP_E_HIP;                                                                         \
    }                                                                                          \
  } while (0)
