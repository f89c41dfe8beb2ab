// wgrid.hip — the windowed numpy-exact fused rollout of the GRID envs with a fixed goal and random agent spawns
// (MultistoryFourRoomsEnv / RoomsEnv defaults; the BASELINE headline configs[1]), K steps in one persistent launch.
//
// The reference (msrooms.py:390-413, rooms.py:198-222, action_utils.py:84-90) draws everything from one numpy
// PCG64 stream: per step random(B) for the action failures, then choice(valid_agent, b) for the b envs that
// terminated or truncated, in ascending env order. Where step t+1's random(B) starts depends on how many words
// step t's choice() consumed, i.e. on the global reset count b_t: every step has one grid-wide exchange.
//
// Design (one workgroup of 11 waves per CU, block beta owns the E = 512 * NS consecutive envs [E beta, E beta + E);
// env slot i = k * 512 + 64 w + l of env wave w, lane l, slot k):
//  * The random(B) words a block needs at step t+1 depend on the stream only through the position x_{t+1} =
//    y_t + used_t (y_t = x_t + B). The words themselves can be computed before used_t is known: while step t's
//    exchange is in flight, the 8 env waves fill a WINDOW of E + 2H consecutive u64 draws around the predicted
//    position (used predicted from the previous step's b). After the exchange env i reads window word
//    i + rw_off, rw_off = H + used_t - used_pred; a prediction more than H off regenerates the window exactly
//    (measured miss rate: tools/window_stats.py). So the step's critical path is only
//      transitions (window word -> integer threshold compares -> LDS move table) -> granule publish ->
//      all-gather of the G granules -> the block's resetter cells -> barrier,
//    and the PCG64 work (~40 VALU per word) runs on the otherwise idle SIMDs during the exchange.
//  * choice() words: 512 COARSE STATES S(y + 1 + 32 j) (one per env lane, a per-lane constant jump) cover the
//    first 16384 draws after random(B); a resetter's word is one jump (<= 31 steps, LDS table) from a coarse state.
//  * Lemire rejections (p ~ 2.4e-8 per word for 104 cells): each block checks a 62-draw slice of the choice
//    stream before publishing (slices of all blocks cover 124 G half-words); the granule carries the count.
//    Any rejection, or more resets than the slices cover, takes the exact slow path: coverage rounds (one more
//    granule exchange each), the rejected positions listed, and every resetter's word placed exactly.
//  * Outputs: the env waves stage {cell, term, trunc, wall-bump} per env (4 B) in LDS; two store waves turn a
//    step's staging into obs (per-cell obs table), reward, terminated and truncated with 16-B non-temporal
//    stores while the next step runs (double-buffered staging).
// Synchronisation: one workgroup barrier per step (B2, after the exchange) plus LDS counters; cross-block only
// the tagged 8-B granules (agent-scope relaxed stores / polls, MI355X_MICROARCH.md "handoff" rows), each wait
// bounded by spin_limit (GridCtl::err flags a grid that cannot make progress).
#include <stdint.h>

#include "gp_internal.h"
#include "grid_shared.h"

namespace {

// GP_STAMPS diagnostic builds (tools/wstamps.py): s_memrealtime (100 MHz, chip-synchronous) stamps by one lane,
// kept in LDS during the launch and copied out at its end (a global store per stamp would be waited for by every
// later `s_waitcnt vmcnt(0)` of that wave, gfx950 counting stores in vmcnt, and stretch the phases it measures).
#ifdef GP_STAMPS
constexpr int ST_STEPS = 24, ST_SLOTS = 42;  // stamps of the first 24 steps, 42 per step (tools/wstamps.py)
__shared__ unsigned long long g_stamp[32 * 32 + 8];
#define WSTAMP(P, k, i)                                                                                  \
  do {                                                                                                   \
    if ((threadIdx.x & 63) == 0 && (k) < ST_STEPS) {                                                     \
      unsigned long long t_;                                                                             \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                     \
      g_stamp[(k) * ST_SLOTS + (i)] = t_;                                                                \
    }                                                                                                    \
  } while (0)
#define LSTAMP(P, i)                                                                                     \
  do {                                                                                                   \
    if ((threadIdx.x & 63) == 0) {                                                                       \
      unsigned long long t_;                                                                             \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                     \
      g_stamp[32 * 32 + (i)] = t_;                                                                       \
    }                                                                                                    \
  } while (0)
#else
#define WSTAMP(P, k, i) \
  do {                  \
  } while (0)
#define LSTAMP(P, i) \
  do {               \
  } while (0)
#endif

// Timing-study variants (WgParams::tmode, gp_debug_set "wg_tmode"; never set in production). TM_NOSTORE and TM_NOFILL
// drop work (results invalid: measurement only); the others are alternative schedules with exact results.
constexpr int TM_NOSTORE = 1;   // store waves skip the output copy
constexpr int TM_NOFILL = 2;    // env waves skip the window fill (stale words)
constexpr int TM_LATEACT = 4;   // env waves load the next step's actions after the transitions (default: before)
constexpr int TM_THROTTLE = 8;  // store waves drain their stores after every 16-env chunk (vmcnt(0))
constexpr int TM_BUSYPOLL = 16; // the all-gather polls without s_sleep
constexpr int TM_NOPRIO = 32;   // env waves keep priority 0 through their transitions (default: 2, above the store waves)
constexpr int TM_EAGERSTORE = 64; // store waves copy a step as soon as it is final (default: after the next transitions)
constexpr int TM_NOCAND = 128;  // no candidate cells during the all-gather (every resetter's cell drawn after it)
constexpr int TM_STORELOW = 256; // store waves at priority 0 (default 1)
constexpr int TM_ENVHIGH = 512; // env waves at priority 2 throughout (default: 2 for the transitions, 0 otherwise)
constexpr int TM_NOTABLES = 1024;  // no table staging at launch (stale LDS tables: measurement only)
constexpr int TM_NOFIRST = 2048;   // no first-window fill at launch (stale words: measurement only)
constexpr int TM_ACTSTART = 4096;  // env waves issue the next step's action loads at the step's start (default: loop top)
constexpr int TM_OLDPRO = 8192;    // round-5 prologue: the whole first window by rows, then the control wave's go-ahead
constexpr int TM_CELLSWAP = 16384; // blocks of <= 1,024 envs: the control wave places the resetters' cells (round 5)

constexpr int EW = 8;                 // env waves
#ifndef WG_SW
#define WG_SW 2
#endif
constexpr int SW = WG_SW;             // store waves (3: one on each SIMD without the control wave, 12 waves per CU)
constexpr int CWAVE = EW;             // the control wave
constexpr int NWAVES = EW + 1 + SW;
constexpr int TPB = NWAVES * 64;      // 704 threads
constexpr int NL = EW * 64;           // env lanes (512)
constexpr int SLICE = 62;             // u64 draws per rejection-check slice (124 half-words)
constexpr int MAXRP = 512;            // rejected half-word positions the slow path lists
constexpr int NCAND = 512;            // candidate resetter cells drawn during the all-gather (256 u64 draws)
constexpr uint32_t CAND_W = 192;      // half-words of them before the predicted block prefix

struct WgShared {
  uint64_t mask[8][EW];      // this step's resetter ballots by (slot k, env wave w)
  // monotone LDS counters: the waves never meet at a workgroup barrier inside the step loop
  uint32_t trans_done;       // env waves done with a step's transitions (EW per step)
  uint32_t cs_done;          // env waves done with a step's coarse states
  uint32_t r2s_done;         // env waves done listing a step's resetters in r2s
  uint32_t fill_done;        // env-wave window fills (and exact regenerations) completed
  uint32_t res_done;         // env waves done taking a step's resetter cells (the staging is final)
  uint32_t st_done;          // store-wave step copies completed (SW per step)
  uint32_t sx_ready;         // control wave: step k's S(x) published (k + 1)
  uint32_t sy_ready;         // control wave: step k's S(y) and step k+1's window base published (k + 1)
  uint32_t cells_done;       // control wave: step k's exchange finished, its resetters' cells staged (k + 1)
  uint32_t pro;              // prologue: the first window's base is published
  uint64_t sx[2][2];         // by step parity: S(x_t) (hi, lo), the state at the step's start
  uint64_t sy[2][2];         // by step parity: S(y_t) (hi, lo), the state after the step's random(B)
  uint64_t rw[2][2];         // by parity of the step a window serves: its base state (hi, lo)
  int32_t rw_off[2];         // by step parity: env i of that step reads window word i + rw_off
  uint32_t fix[2];           // by step parity: bit 0 slow path, bit 1 window regeneration
  uint32_t R, h, u, nrp;     // block prefix, has_uint32 / uinteger at the step start, # rejected positions (slow path)
  uint32_t cbase;            // half-word of cand[0] (env-wave cells)
  uint32_t rp[MAXRP];        // slow path: rejected half-word positions, ascending
  uint16_t r2s[4096];        // resetter rank in the block -> env slot
  uint16_t cand[NCAND];      // the cells of choice() half-words cbase .. cbase + NCAND - 1 (predicted block prefix)
};

// ------------------------------------------------------------------ small helpers ----
__device__ __forceinline__ void lds_barrier() {  // orders LDS only (no vmcnt(0) drain of the output stores)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
__device__ __forceinline__ void lds_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local"); }
__device__ __forceinline__ void lds_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); }
__device__ __forceinline__ uint32_t lds_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_add(uint32_t* p, uint32_t v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Wait (one wave) until an LDS counter reaches `want`. Every wave of the block is resident, so this ends; the
// bound (~2^26 polls) only turns a logic error into a flagged launch (GP_DERR_TIMEOUT) instead of a hung GPU.
__device__ __forceinline__ void lds_wait(const uint32_t* p, uint32_t want, uint32_t* err) {
  uint32_t n = 0;
  while (lds_load(p) < want) {
    __builtin_amdgcn_s_sleep(1);
    if (++n > (1u << 26)) {
      atomicOr(err, GP_DERR_TIMEOUT);
      break;
    }
  }
  lds_acquire();
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {  // DPP row shifts + broadcasts
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); // row_bcast:31
  return x;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(x), 63);
}
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {  // set bits of m below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot((int)p); }

// numpy next_uint32 bookkeeping after `wtot` 32-bit words: u64 draws used and the new buffer flag.
__device__ __forceinline__ void words_to_draws(uint32_t wtot, uint32_t h0, uint32_t& used, uint32_t& h) {
  if (wtot == 0) {
    used = 0; h = h0;
  } else if (h0) {
    used = wtot >> 1; h = (wtot - 1) & 1;  // ceil((wtot-1)/2)
  } else {
    used = (wtot + 1) >> 1; h = wtot & 1;  // ceil(wtot/2)
  }
}

// A 53-bit threshold t as a threshold on the full 64-bit draw x: (x >> 11) > t  <=>  x > (t << 11) | 0x7FF.
__host__ __device__ __forceinline__ uint64_t thr_on_u64(uint64_t t) {
  return t >= (1ull << 53) ? ~0ull : ((t << 11) | 0x7FFull);
}

// Action -> byte offset of its threshold row (numpy negative indexing; out-of-range actions, an IndexError in
// the reference (msrooms.py:400 action_matrix[action]), set GP_DERR_ACTION and are clamped).
template <int NA>
__device__ __forceinline__ int32_t action_row(int32_t a, uint32_t* derr) {
  if (action_out_of_range(a, NA)) flag_bad_action(derr);
  if (a < 0) a += NA;
  return min(max(a, 0), NA - 1) * NA * 8;
}

struct Tabs {  // the LDS copy of the tables (pointers resolved once per role)
  const PcgJump* j32p;   // [32] jump by d
  const PcgJump* jt8p;   // [2][256] jump by d, by 256 d
  const int32_t* ocp;    // [ncells] obs of the agent cell (fixed goal)
  const uint16_t* avp;   // [n_agent] valid agent cells
  const PcgJump* jt64;   // global radix-64 tables
  int32_t halo;
  __device__ __forceinline__ Tabs(const char* d, const WgParams& P)
      : j32p(reinterpret_cast<const PcgJump*>(d + P.lds.j32)), jt8p(reinterpret_cast<const PcgJump*>(d + P.lds.jt8)),
        ocp(reinterpret_cast<const int32_t*>(d + P.lds.ocell)), avp(reinterpret_cast<const uint16_t*>(d + P.lds.avalid)),
        jt64(P.jt64), halo(P.halo) {}
  __device__ __forceinline__ const PcgJump& j32(uint32_t i) const { return j32p[i]; }
  __device__ __forceinline__ const PcgJump& jt8(uint32_t i) const { return jt8p[i]; }
  __device__ __forceinline__ int32_t ocell(uint32_t c) const { return ocp[c]; }
  __device__ __forceinline__ uint32_t avalid(uint32_t v) const { return avp[v]; }
};

// Coarse state j (S(y + 1 + 32 j)) from its LDS slot (lo, hi).
__device__ __forceinline__ u128 load_cs(const uint64_t* CS, uint32_t j) {
  const ulonglong2 v = reinterpret_cast<const ulonglong2*>(CS)[j];
  return mk128(v.y, v.x);
}
// The state of 0-based choice-stream draw d (< 16384): one jump of d mod 32 from its coarse state.
__device__ __forceinline__ u128 draw_state(const Tabs& tb, const uint64_t* CS, uint32_t d) {
  return apply_jump(tb.j32(d & 31u), load_cs(CS, d >> 5));
}

// S jumped by n draws: two radix-256 LDS entries below 2^16, else the radix-64 tables in global memory.
__device__ __forceinline__ u128 jump_any(const Tabs& tb, u128 s, uint32_t n) {
  if (n < 65536u) {
    if (n & 255u) s = apply_jump(tb.jt8(n & 255u), s);
    if (n >> 8) s = apply_jump(tb.jt8(256u + (n >> 8)), s);
    return s;
  }
  return pcg_jump(tb.jt64, s, n);
}

// The base of the next step's window for block beta when the current step's choice() call uses `used` u64 draws:
// the state whose next output is window word 0, from S(x_t) (jb = jblk[beta][0] folds in random(B) and E beta - H),
// and heff = how many window words precede the block's first env word.
__device__ __forceinline__ u128 rw_base(const Tabs& tb, const PcgJump& jb, u128 Sx, uint32_t used, int beta,
                                        int32_t& heff) {
  const int32_t H = tb.halo;
  if (beta == 0) {
    heff = min(H, (int32_t)used + 1);
    return apply_jump(jb, jump_any(tb, Sx, used + 1u - (uint32_t)heff));
  }
  heff = H;
  return apply_jump(jb, jump_any(tb, Sx, used + 1u));
}

__device__ __forceinline__ bool spin_give_up(const WgParams& P, uint32_t& spins) {
  ++spins;
  if ((spins & 63u) == 0 &&
      (__hip_atomic_load(&P.ctl->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & GP_DERR_TIMEOUT))
    return true;
  if (spins > P.spin_limit) {
    atomicOr(&P.ctl->err, GP_DERR_TIMEOUT);
    return true;
  }
  return false;
}

// Granules: tag (32 bits: tag step << 6 | round) | rejection count (8 bits) | reset count (24 bits).
__device__ __forceinline__ uint64_t gran(uint32_t tag, uint32_t rej, uint32_t cnt) {
  return ((uint64_t)tag << 32) | ((uint64_t)min(rej, 255u) << 24) | (uint64_t)(cnt & 0xFFFFFFu);
}
// The control wave: publish this block's granule of (tag), then all-gather the G granules (lane l: blocks 4l..4l+3).
__device__ __forceinline__ void publish(const WgParams& P, uint64_t* slots, uint32_t tag, uint32_t rej, uint32_t cnt) {
  if ((threadIdx.x & 63) == 0 && (int)blockIdx.x != P.fault_block)
    __hip_atomic_store(&slots[blockIdx.x], gran(tag, rej, cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gather(const WgParams& P, const uint64_t* slots, uint32_t tag, uint64_t (&g)[4]) {
  const bool nap = !(P.tmode & TM_BUSYPOLL);
  const int lane = threadIdx.x & 63, G = (int)gridDim.x;
  uint32_t pend = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    g[j] = (uint64_t)tag << 32;  // blocks >= G: count 0
    if (lane * 4 + j < G) pend |= 1u << j;
  }
  uint32_t spins = 0;
  while (true) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (pend & (1u << j)) g[j] = __hip_atomic_load(&slots[lane * 4 + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((pend & (1u << j)) && (uint32_t)(g[j] >> 32) == tag) pend &= ~(1u << j);
    if (!__any((int)pend)) break;
    if (spin_give_up(P, spins)) {  // flagged (GP_E_DEVICE): counts read as 0 so that every wave drains
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (pend & (1u << j)) g[j] = (uint64_t)tag << 32;
      break;
    }
    if (nap) __builtin_amdgcn_s_sleep(1);
  }
}
__device__ __forceinline__ void exchange(const WgParams& P, uint64_t* slots, uint32_t tag, uint32_t rej, uint32_t cnt,
                                         uint64_t (&g)[4]) {
  publish(P, slots, tag, rej, cnt);
  gather(P, slots, tag, g);
}

__device__ __forceinline__ uint32_t gcnt(uint64_t g) { return (uint32_t)g & 0xFFFFFFu; }
__device__ __forceinline__ uint32_t grej(uint64_t g) { return (uint32_t)(g >> 24) & 0xFFu; }

// Per-launch view of the dynamic LDS (pointers resolved once) and the block geometry.
#ifndef WG_NSTG
#define WG_NSTG 3
#endif
#ifndef WG_EAGER_TAIL
#define WG_EAGER_TAIL 4
#endif
#ifndef WG_SUNROLL
#define WG_SUNROLL 2
#endif
constexpr int NSTG = WG_NSTG;  // staging buffers: the store waves may trail the env waves by up to NSTG - 1 steps
struct Lds {
  uint64_t* RW;   // [E + 2H] window words
  uint64_t* CS0;  // [2 step parities][512][2] coarse states (lo, hi)
  char* stg0;     // [NSTG][E] staged u32 per env: cell | term << 16 | trunc << 17 | wall bump << 18
  __device__ __forceinline__ Lds(char* dyn, const WgParams& P, int E)
      : RW(reinterpret_cast<uint64_t*>(dyn + P.lds.total)),
        CS0(reinterpret_cast<uint64_t*>(dyn + P.lds.total + (size_t)(E + 2 * P.halo) * 8)),
        stg0(dyn + P.lds.total + (size_t)(E + 2 * P.halo) * 8 + 2 * 512 * 16) {}
  __device__ __forceinline__ char* stg(int k, int E) const { return stg0 + (size_t)(k % NSTG) * E * 4; }
  __device__ __forceinline__ uint64_t* CS(int k) const { return CS0 + (size_t)(k & 1) * 1024; }
};

// Slow path, control wave: append the rejected half-word positions of choice-stream slice sigma (u64 draws
// 62 sigma + 1 .. 62 sigma + 62 after random(B), both halves; with a buffered half (h) slice 0 also owns hw 0).
__device__ __forceinline__ void list_slice(const WgParams& P, WgShared& sh, const Tabs& tb, const uint64_t* CS,
                                           uint32_t sigma, u128 Sy, uint32_t h, uint32_t u) {
  const int lane = threadIdx.x & 63;
  bool rlo = false, rhi = false;
  if (lane < SLICE) {
    const uint32_t d = 62u * sigma + (uint32_t)lane;  // 0-based draw after random(B): state S(y + 1 + d)
    const u128 s = d < 16384u ? draw_state(tb, CS, d) : pcg_jump(tb.jt64, Sy, d + 1u);
    const uint64_t x = pcg_output(s);
    rlo = lemire_rejected((uint32_t)x, (uint32_t)P.n_agent, P.thr_agent);
    rhi = lemire_rejected((uint32_t)(x >> 32), (uint32_t)P.n_agent, P.thr_agent);
  }
  const bool rb = sigma == 0 && h && lane == SLICE && lemire_rejected(u, (uint32_t)P.n_agent, P.thr_agent);
  const uint64_t mb = ballot(rb), mlo = ballot(rlo), mhi = ballot(rhi);
  const uint32_t n0 = sh.nrp;
  const uint32_t base = n0 + (mb ? 1u : 0u);
  const uint32_t ex = mbcnt(mlo) + mbcnt(mhi);
  const uint32_t pos = 124u * sigma + 2u * (uint32_t)lane + h;
  if (rb && n0 < (uint32_t)MAXRP) sh.rp[n0] = 0;
  if (rlo && base + ex < (uint32_t)MAXRP) sh.rp[base + ex] = pos;
  if (rhi && base + ex + (rlo ? 1u : 0u) < (uint32_t)MAXRP) sh.rp[base + ex + (rlo ? 1u : 0u)] = pos + 1u;
  const uint32_t n1 = base + (uint32_t)__builtin_popcountll(mlo) + (uint32_t)__builtin_popcountll(mhi);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    if (n1 > (uint32_t)MAXRP) atomicOr(&P.ctl->err, GP_DERR_OVERFLOW);
    sh.nrp = min(n1, (uint32_t)MAXRP);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// The slices with rejections among the gathered granules (lane l holds blocks 4l..4l+3 of round r), ascending.
__device__ __forceinline__ uint32_t list_flagged(const WgParams& P, WgShared& sh, const Tabs& tb, const uint64_t* CS,
                                                 const uint64_t (&g)[4], uint32_t r, u128 Sy, uint32_t h, uint32_t u) {
  const int G = (int)gridDim.x;
  uint32_t r4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) r4[j] = grej(g[j]);
  const uint32_t tot = wave_sum(r4[0] + r4[1] + r4[2] + r4[3]);
  uint64_t any = ballot((r4[0] | r4[1] | r4[2] | r4[3]) != 0);
  while (any) {
    const int l = __builtin_ctzll(any);
    any &= any - 1;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (__builtin_amdgcn_readlane((int)r4[j], l)) list_slice(P, sh, tb, CS, r * (uint32_t)G + (uint32_t)(4 * l + j), Sy, h, u);
  }
  return tot;
}

// Slow path, control wave (a Lemire rejection in the step's choice() words, or more resets than the slices
// cover): coverage rounds until every accepted word's position is known, the rejected positions listed in
// sh.rp (ascending). Returns the half-words consumed. The env waves then place their own resetters.
__device__ __forceinline__ uint32_t ctrl_slow(const WgParams& P, WgShared& sh, const Tabs& tb, const uint64_t* CS, u128 Sy,
                                              uint32_t h, uint32_t u, uint32_t b, uint32_t ts, const uint64_t (&g0)[4]) {
  const int lane = threadIdx.x & 63, G = (int)gridDim.x, beta = (int)blockIdx.x;
  if (lane == 0) sh.nrp = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  uint32_t rtot = list_flagged(P, sh, tb, CS, g0, 0u, Sy, h, u);
  // coverage rounds: slices sigma = r G + beta of the half-words beyond the first 124 G
  uint32_t covered = 124u * (uint32_t)G;
  uint64_t* slots = P.slots + (size_t)(ts & 1u) * 2 * G;
  for (uint32_t r = 1; covered < b + rtot && r < 64u; ++r) {
    const uint32_t sigma = r * (uint32_t)G + (uint32_t)beta;
    uint32_t rj = 0;
    if (lane < SLICE) {
      const uint64_t x = pcg_output(pcg_jump(tb.jt64, Sy, 62u * sigma + (uint32_t)lane + 1u));
      rj = (lemire_rejected((uint32_t)x, (uint32_t)P.n_agent, P.thr_agent) ? 1u : 0u) +
           (lemire_rejected((uint32_t)(x >> 32), (uint32_t)P.n_agent, P.thr_agent) ? 1u : 0u);
    }
    const uint32_t cnt = wave_sum(rj);
    uint64_t g[4];
    exchange(P, slots + (size_t)(r & 1u) * G, (ts << 6) | r, cnt, 0u, g);
    rtot += list_flagged(P, sh, tb, CS, g, r, Sy, h, u);
    covered += 124u * (uint32_t)G;
  }
  // half-words consumed: the position of accepted word b - 1, plus one
  uint32_t wtot = 0;
  if (b) {
    uint32_t p = b - 1u;
    const uint32_t n = sh.nrp;
    for (uint32_t q = 0; q < n; ++q) p += sh.rp[q] <= p ? 1u : 0u;
    wtot = p + 1u;
  }
  return wtot;
}

// ------------------------------------------------------------------ the control wave ----
// Per step: S(x) published (sx_ready: the env waves' coarse states), the rejection check of its slice, the block's
// reset count once the env waves' transitions are in, the granule published, S(y) and the next window's base
// (sy_ready), the all-gather, the resetters' cells (cells_done), then the next step's S(x) = J_used(S(y)). Every
// constant part of a jump (random(B), the block and lane offsets) is folded into per-lane / per-block tables, so
// the chain from one exchange to the next publish is two table jumps and one per-lane jump.
template <int NS, int NA>
__device__ __forceinline__ void wg_ctrl(const WgParams& P, WgShared& sh, const Tabs& tb, const Lds& L, int K) {
  const int lane = threadIdx.x & 63, beta = (int)blockIdx.x, G = (int)gridDim.x;
  constexpr int E = NS * 512;
  GridCtl* C = P.ctl;
  u128 Sx = mk128(C->s_hi, C->s_lo);
  uint32_t h = C->has_u32, u = C->uinteger;
  uint32_t bprev = C->fb_last;
  uint32_t Rprev = (uint32_t)(((uint64_t)bprev * (uint64_t)blockIdx.x) / (uint64_t)gridDim.x);  // a first guess
  const uint32_t ts0 = C->wstep + 1u;  // tag step of k = 0 (tags are never 0: the slots start zeroed)
  const PcgJump jr = P.jrej[(size_t)beta * 64 + lane];
  const PcgJump jb = P.jblk[2 * beta], jpro = P.jblk[2 * beta + 1];
  const PcgJump jB = P.jB;
  const uint32_t nag = (uint32_t)P.n_agent, thra = P.thr_agent;
  const int32_t H = P.halo;
  const uint32_t bias = (uint32_t)P.wg_bias;
  // small blocks (<= 1,024 envs): the env waves place their resetters' cells (their SIMDs have room; the control
  // wave's cells loop leaves the chain); 4,096-env blocks: the control wave (env waves' SIMD time bounds the step)
  const bool envcells = NS <= 2 && !(P.tmode & TM_CELLSWAP);
  uint32_t* derr = &C->err;
  lds_barrier();  // P1: tables staged, counters zeroed
  // round 5's prologue (TM_OLDPRO): the first window's offset for the env waves, which filled the window by rows
  if (lane == 0 && (P.tmode & TM_OLDPRO)) {
    const u128 s = apply_jump(jpro, Sx);
    sh.rw[0][0] = hi64(s);
    sh.rw[0][1] = lo64(s);
    sh.rw_off[0] = beta == 0 ? 1 : H;
    lds_release();
    __hip_atomic_store(&sh.pro, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  LSTAMP(P, 1);
  for (int k = 0; k < K; ++k) {
    const uint32_t ts = ts0 + (uint32_t)k;
    if (lane == 0) {
      sh.sx[k & 1][0] = hi64(Sx);
      sh.sx[k & 1][1] = lo64(Sx);
      lds_release();
      __hip_atomic_store(&sh.sx_ready, (uint32_t)k + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // Lemire check of this block's slice of the choice() stream (u64 draws 62 beta + 1 .. + 62 after random(B))
    uint32_t rj = 0;
    if (lane < SLICE) {
      const uint64_t x = pcg_output(apply_jump(jr, Sx));
      rj = (lemire_rejected((uint32_t)x, nag, thra) ? 1u : 0u) + (lemire_rejected((uint32_t)(x >> 32), nag, thra) ? 1u : 0u);
    } else if (lane == SLICE && beta == 0 && h) {
      rj = lemire_rejected(u, nag, thra) ? 1u : 0u;  // the buffered half is hw 0
    }
    const uint32_t rejc = wave_sum(rj);
    WSTAMP(P, k, 6);
    // this block's reset count, published
    lds_wait(&sh.trans_done, (uint32_t)EW * (uint32_t)(k + 1), derr);
    WSTAMP(P, k, 7);
    const uint32_t cb = wave_sum(lane < NS * EW ? (uint32_t)__builtin_popcountll(sh.mask[lane >> 3][lane & 7]) : 0u);
    uint64_t* slots = P.slots + (size_t)(ts & 1u) * 2 * G;
    publish(P, slots, ts << 6, rejc, cb);
    WSTAMP(P, k, 8);
    // while the granules travel: S(y) and the next step's window, around the used predicted from the last b
    const u128 Sy = apply_jump(jB, Sx);
    uint32_t used_p, hp;
    words_to_draws(bprev + bias, h, used_p, hp);
    int32_t heff_p;
    const u128 Srw = rw_base(tb, jb, Sx, used_p, beta, heff_p);
    if (lane == 0) {
      sh.sy[k & 1][0] = hi64(Sy);
      sh.sy[k & 1][1] = lo64(Sy);
      sh.rw[(k + 1) & 1][0] = hi64(Srw);
      sh.rw[(k + 1) & 1][1] = lo64(Srw);
      lds_release();
      __hip_atomic_store(&sh.sy_ready, (uint32_t)k + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // While the granules travel (the longest wait of a step): the cells of the choice() half-words around the block
    // prefix predicted by the last step's, so that the resetters' cells after the exchange are one LDS read each.
    // Candidate i is half-word cbase + i; cbase = 2 d0 + h, draws d0 .. d0 + NCAND / 2 - 1 (both halves each).
    const uint64_t* CS = L.CS(k);
    lds_wait(&sh.cs_done, (uint32_t)EW * (uint32_t)(k + 1), derr);
    const uint32_t d0 = min(Rprev > CAND_W + h ? (Rprev - CAND_W - h) >> 1 : 0u, 16384u - NCAND / 2);  // CS reach
    const uint32_t cbase = 2u * d0 + h;
    if (!(P.tmode & TM_NOCAND)) {
#pragma unroll
      for (int m = 0; m < NCAND / 128; ++m) {
        const uint32_t j = (uint32_t)(lane + 64 * m);
        const uint64_t x = pcg_output(draw_state(tb, CS, d0 + j));
        sh.cand[2 * j] = (uint16_t)tb.avalid(lemire_value((uint32_t)x, nag));
        sh.cand[2 * j + 1] = (uint16_t)tb.avalid(lemire_value((uint32_t)(x >> 32), nag));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    uint64_t g[4];
    gather(P, slots, ts << 6, g);
    WSTAMP(P, k, 9);
    const uint32_t bsum = gcnt(g[0]) + gcnt(g[1]) + gcnt(g[2]) + gcnt(g[3]);
    const uint32_t incl = wave_incl_scan(bsum);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    uint32_t R;
    {
      const int bl = beta >> 2, bj = beta & 3;
      uint32_t before = incl - bsum;  // the blocks of the lanes below
#pragma unroll
      for (int j = 0; j < 4; ++j) before += j < bj ? gcnt(g[j]) : 0u;
      R = (uint32_t)__builtin_amdgcn_readlane((int)before, bl);
    }
    const uint32_t rtot = wave_sum(grej(g[0]) + grej(g[1]) + grej(g[2]) + grej(g[3]));
    const bool slow = rtot != 0 || b > 124u * (uint32_t)G;
    uint32_t used, h2;
    // (also before cells_done when nothing is drawn: every env wave has read this step's masks)
    lds_wait(&sh.r2s_done, (uint32_t)EW * (uint32_t)(k + 1), derr);
    if (!slow) {
      words_to_draws(b, h, used, h2);
      if (envcells && lane == 0) {  // the env waves place their own resetters (rank q -> half-word R + q)
        sh.R = R;
        sh.h = h;
        sh.u = u;
        sh.cbase = cbase;
      }
      if (cb && !envcells) {  // this block's resetters' cells: rank q takes half-word R + q
        uint16_t* st = reinterpret_cast<uint16_t*>(L.stg(k, E));
        for (uint32_t q = (uint32_t)lane; q < cb; q += 64u) {
          const uint32_t hw = R + q;
          const uint32_t slot = sh.r2s[q];
          uint32_t cell;
          if (hw - cbase < (uint32_t)NCAND && !(P.tmode & TM_NOCAND)) {  // (hw >= cbase >= h: never the buffered half)
            cell = sh.cand[hw - cbase];
          } else {
            uint32_t word;
            if (h && hw == 0) {
              word = u;
            } else {
              const uint32_t hh = hw - h;
              const uint64_t x = pcg_output(draw_state(tb, CS, hh >> 1));
              word = (hh & 1u) ? (uint32_t)(x >> 32) : (uint32_t)x;
            }
            cell = tb.avalid(lemire_value(word, nag));
          }
          st[2 * slot] = (uint16_t)cell;  // the low half of the staged word
        }
      }
    } else {
      const uint32_t wtot = ctrl_slow(P, sh, tb, CS, Sy, h, u, b, ts, g);
      words_to_draws(wtot, h, used, h2);
      if (lane == 0) {
        sh.R = R;
        sh.h = h;
        sh.u = u;
      }
    }
    // the next step's window offset; a window more than H off is regenerated exactly by the env waves
    int32_t off = heff_p + (int32_t)used - (int32_t)used_p;
    uint32_t fix = slow ? 1u : 0u;
    if (k + 1 < K && (off < 0 || off > 2 * H)) {
      int32_t heff;
      const u128 s = rw_base(tb, jb, Sx, used, beta, heff);
      off = heff;
      fix |= 2u;
      if (lane == 0) {
        sh.rw[(k + 1) & 1][0] = hi64(s);
        sh.rw[(k + 1) & 1][1] = lo64(s);
      }
    }
    if (lane == 0) {
      sh.rw_off[(k + 1) & 1] = off;
      sh.fix[k & 1] = fix;
      lds_release();
      __hip_atomic_store(&sh.cells_done, (uint32_t)k + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    WSTAMP(P, k, 10);
    // the next step's state S(x_{t+1}) = S(y_t + used)
    Sx = jump_any(tb, Sy, used);
    if (used) u = (uint32_t)(pcg_output(Sx) >> 32);  // numpy keeps the last drawn high half in uinteger
    h = h2;
    bprev = b;
    Rprev = R;
    WSTAMP(P, k, 12);
  }
  LSTAMP(P, 3);
  if (beta == 0 && lane == 0) {
    C->s_hi = hi64(Sx);
    C->s_lo = lo64(Sx);
    C->has_u32 = h;
    C->uinteger = u;
    C->fb_last = bprev;
    C->wstep = ts0 + (uint32_t)K - 1u;  // (GridCtl::step is the fused kernel's own tag counter: not advanced here)
  }
}

// ------------------------------------------------------------------ the env waves ----
struct Acc {
  uint32_t eps = 0, ngoal = 0, nwall = 0, lens = 0;
};

// Slow path: place this lane's resetters exactly (ranks -> positions past the listed rejections -> words).
template <int NS>
__device__ __forceinline__ void wg_env_slow(const WgParams& P, WgShared& sh, const Tabs& tb, const uint64_t* CS,
                                            int k, char* stg, uint32_t dn, const uint32_t (&pre)[NS],
                                            const uint64_t (&bm)[NS], uint32_t (&ae)[NS]) {
  const int lg = threadIdx.x;
  const u128 Sy = mk128(sh.sy[k & 1][0], sh.sy[k & 1][1]);
  const uint32_t R = sh.R, h = sh.h, u = sh.u, n = sh.nrp;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (!((dn >> s) & 1u)) continue;
    uint32_t p = R + pre[s] + mbcnt(bm[s]);
    for (uint32_t q = 0; q < n; ++q) p += sh.rp[q] <= p ? 1u : 0u;
    uint32_t word;
    if (h && p == 0) {
      word = u;
    } else {
      const uint32_t hh = p - h, d = hh >> 1;
      const u128 st = d < 16384u ? draw_state(tb, CS, d) : pcg_jump(tb.jt64, Sy, d + 1u);
      const uint64_t x = pcg_output(st);
      word = (hh & 1u) ? (uint32_t)(x >> 32) : (uint32_t)x;
    }
    const uint32_t cell = tb.avalid(lemire_value(word, (uint32_t)P.n_agent));
    reinterpret_cast<uint16_t*>(stg)[2 * (s * 512 + lg)] = (uint16_t)cell;
    ae[s] = cell;
  }
}

// Fast path (no rejection in the step's choice() words), blocks of <= 1,024 envs: this lane's resetters take
// half-words R + rank, rank from the listing (pre + mbcnt); their cells are the control wave's candidates when inside
// its window, else drawn from the coarse states (the control wave publishes R, h, u, cbase with cells_done and draws
// nothing after the all-gather, so its cells loop is off the step's chain).
template <int NS>
__device__ __forceinline__ void wg_env_cells(const WgParams& P, WgShared& sh, const Tabs& tb, const uint64_t* CS,
                                             char* stg, uint32_t dn, const uint32_t (&pre)[NS], const uint64_t (&bm)[NS],
                                             uint32_t (&ae)[NS]) {
  if (!dn) return;
  const int lg = threadIdx.x;
  const uint32_t R = sh.R, h = sh.h, u = sh.u, cbase = sh.cbase;
  const bool nocand = (P.tmode & TM_NOCAND) != 0;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (!((dn >> s) & 1u)) continue;
    const uint32_t hw = R + pre[s] + mbcnt(bm[s]);
    uint32_t cell;
    if (hw - cbase < (uint32_t)NCAND && !nocand) {  // (hw >= cbase >= h: never the buffered half)
      cell = sh.cand[hw - cbase];
    } else {
      uint32_t word;
      if (h && hw == 0) {
        word = u;
      } else {
        const uint32_t hh = hw - h;
        const uint64_t x = pcg_output(draw_state(tb, CS, hh >> 1));
        word = (hh & 1u) ? (uint32_t)(x >> 32) : (uint32_t)x;
      }
      cell = tb.avalid(lemire_value(word, (uint32_t)P.n_agent));
    }
    reinterpret_cast<uint16_t*>(stg)[2 * (s * 512 + lg)] = (uint16_t)cell;
    ae[s] = cell;
  }
}

// Fill the window: env wave w writes rows fr0 .. fr0 + nrow - 1 of 64 words (word j = 64 r + lane): the lane's state
// is the base jumped by 64 fr0 + lane (its jlane entry), then by 64 per row. The rows per wave (WgParams::fill_rows)
// lean on the SIMD that hosts neither the control wave nor a store wave (round 6: its env waves finished their
// fills ~0.7 us before the others). (Two independent chains per lane, for the ILP of a wave whose SIMD partner
// has finished, measured no faster at 167 VGPRs: profiles/r06_fill_chains_ab.txt.)
__device__ __forceinline__ void fill_window(uint64_t* RW, const PcgJump& jl, const PcgJump& jrow, int fr0, int nrow,
                                            u128 base, int lane) {
  u128 s = apply_jump(jl, base);
  uint64_t* d = RW + fr0 * 64 + lane;
  for (int m = 0; m < nrow; ++m) {
    d[m * 64] = pcg_output(s);
    s = apply_jump(jrow, s);
  }
}

template <int NS, int NA>
__device__ __forceinline__ void wg_env(const WgParams& P, WgShared& sh, const Tabs& tb, const Lds& L, const char* dyn,
                                       const int32_t* __restrict__ act, int K, Acc& acc, int32_t* __restrict__ obs,
                                       float* __restrict__ rew, uint8_t* __restrict__ term,
                                       uint8_t* __restrict__ trunc) {
  const int lg = threadIdx.x, lane = lg & 63, w = lg >> 6;
  const int beta = (int)blockIdx.x, G = (int)gridDim.x;
  constexpr int E = NS * 512;
  const size_t B = (size_t)E * (size_t)G;
  const size_t e0 = (size_t)beta * E;
  const char* thr = dyn + P.lds.thr;
  const char* mv = dyn + P.lds.move;
  const uint32_t goal = (uint32_t)P.goal, tlim = (uint32_t)P.time_limit;
  uint32_t* derr = &P.ctl->err;
  uint32_t* aeg = P.ae;
  const bool envcells = NS <= 2 && !(P.tmode & TM_CELLSWAP);  // (as wg_ctrl)
  const int fr0 = P.fill_row0[w], nrow = P.fill_rows[w];  // this wave's window rows
  const int tmode = P.tmode;
  const PcgJump jrow = P.jrow;
  // per-lane constant jumps: to the lane's first window word (64 fill_row0[w] + lane) and by 32 lg + 1 (coarse state)
  const PcgJump jrw = P.jlane[2 * lg], jcs = P.jlane[2 * lg + 1];
  uint32_t ae[NS];
  int32_t arow[NS], anext[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    ae[k] = aeg[e0 + (size_t)k * 512 + lg];
    anext[k] = act[e0 + (size_t)k * 512 + lg];
  }
  // Step 0's words are exact (no prediction): env i = s 512 + lg of block beta draws S(x_0 + 1 + E beta + i). Each lane
  // computes its own NS words straight into the window slots its envs read (i + off0), from global data while the
  // control and store waves stage the tables (the window lies behind them in LDS), so step 0 waits for no other
  // wave's words and for no go-ahead: only for the tables (P1). (TM_OLDPRO: round 5's prologue, the whole window
  // by rows, then the control wave's offset.)
  const bool oldpro = (tmode & TM_OLDPRO) != 0;
  if (!(tmode & TM_NOFIRST)) {
    const GridCtl* C = P.ctl;
    const u128 S0 = mk128(C->s_hi, C->s_lo);
    if (oldpro) {
      fill_window(L.RW, jrw, jrow, fr0, nrow, apply_jump(P.jblk[2 * beta + 1], S0), lane);
    } else {
      const int32_t off0 = beta == 0 ? 1 : P.halo;
      u128 st = apply_jump(P.jfirst[(beta ? 512 : 0) + lg], apply_jump(P.jblk[2 * beta + 1], S0));
      const PcgJump j512 = P.j512;
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        L.RW[k * 512 + lg + off0] = pcg_output(st);
        if (k + 1 < NS) st = apply_jump(j512, st);
      }
      if (lg == 0) sh.rw_off[0] = off0;
    }
  }
  if (w == 0) LSTAMP(P, 2);
  lds_barrier();  // P1
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    arow[k] = action_row<NA>(anext[k], derr);
    acc.lens += ae[k] >> 16;  // episode lengths: + elapsed at the start - elapsed at the end + steps
  }
  if (oldpro) {
    lds_wait(&sh.pro, 1u, derr);  // the first window's offset
    if (lane == 0) lds_add(&sh.fill_done, 1u);
  }
  if (w == 0) LSTAMP(P, 7);
  uint32_t fill_target = EW;
  uint64_t bm[NS];
  uint32_t pre[NS];
  for (int k = 0; k < K; ++k) {
    char* stg = L.stg(k, E);
    if (w == 0) WSTAMP(P, k, 41);
    if (k + 1 < K && !(tmode & (TM_LATEACT | TM_ACTSTART))) {
#pragma unroll
      for (int s = 0; s < NS; ++s) anext[s] = act[(size_t)(k + 1) * B + e0 + (size_t)s * 512 + lg];
    }
    if (w == 0) WSTAMP(P, k, 40);
    lds_wait(&sh.fill_done, fill_target, derr);                  // every env wave's part of this step's window
    if (k >= NSTG) lds_wait(&sh.st_done, (uint32_t)SW * (uint32_t)(k - NSTG + 1), derr);  // this staging buffer copied out
    if (!(tmode & TM_NOPRIO)) __builtin_amdgcn_s_setprio(2);  // the transitions are on the critical path
    if (w == 0) WSTAMP(P, k, 0);
    WSTAMP(P, k, 32 + w);
    if (k + 1 < K && (tmode & TM_ACTSTART)) {
#pragma unroll
      for (int s = 0; s < NS; ++s) anext[s] = act[(size_t)(k + 1) * B + e0 + (size_t)s * 512 + lg];
    }
    // ---- transitions (the critical path) ----
    // Phased over the env slots so that their LDS round trips overlap: every slot's window word and threshold
    // row first, then the effective actions, the move-table entries, and the staged outputs last (a store to
    // the staging area between two slots' loads would order them: all of it is one LDS array to the compiler).
    const int32_t off = sh.rw_off[k & 1];
    uint32_t dn = 0;
    uint32_t mvo[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint64_t x = L.RW[s * 512 + lg + off];
      const char* t = thr + arow[s];
      uint32_t eb = 0;  // 2 x effective action: #{j : x > thr[a][j]} (integer form of action_utils.py:84-90)
#pragma unroll
      for (int j = 0; j + 1 < NA; j += 2) {
        const ulonglong2 tt = *reinterpret_cast<const ulonglong2*>(t + 8 * j);
        eb = x > tt.x ? (uint32_t)(2 * (j + 1)) : eb;
        if (j + 2 < NA) eb = x > tt.y ? (uint32_t)(2 * (j + 2)) : eb;
      }
      mvo[s] = (ae[s] & 0xFFFFu) * (2 * NA) + eb;
    }
    uint32_t mm[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) mm[s] = *reinterpret_cast<const uint16_t*>(mv + mvo[s]);
    uint32_t sv[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint32_t m = mm[s];
      const uint32_t nc = m & 0x7FFFu, blocked = m >> 15;
      const uint32_t el = (ae[s] >> 16) + 1u;
      const bool term = nc == goal, trunc = el > tlim, done = term || trunc;
      sv[s] = nc | ((uint32_t)term << 16) | ((uint32_t)trunc << 17) | (blocked << 18);
      ae[s] = done ? nc : (nc | (el << 16));
      bm[s] = ballot(done);
      dn |= (uint32_t)done << s;
      acc.ngoal += term ? 1u : 0u;
      acc.nwall += (blocked && !term) ? 1u : 0u;
    }
    if (lane == 0) {
#pragma unroll
      for (int s = 0; s < NS; ++s) sh.mask[s][w] = bm[s];
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) reinterpret_cast<uint32_t*>(stg)[s * 512 + lg] = sv[s];
    acc.eps += (uint32_t)__builtin_popcount(dn);
    lds_release();
    if (lane == 0) lds_add(&sh.trans_done, 1u);
    if (!(tmode & TM_NOPRIO) && !(tmode & TM_ENVHIGH)) __builtin_amdgcn_s_setprio(0);
    if (w == 0) WSTAMP(P, k, 1);
    WSTAMP(P, k, 16 + w);
    // the next step's actions (one step ahead)
    if (k + 1 < K && (tmode & TM_LATEACT)) {
#pragma unroll
      for (int s = 0; s < NS; ++s) anext[s] = act[(size_t)(k + 1) * B + e0 + (size_t)s * 512 + lg];
    }
    // ---- while the exchange runs: coarse states, resetter listing, the next step's window ----
    lds_wait(&sh.sx_ready, (uint32_t)k + 1u, derr);
    if (w == 0) WSTAMP(P, k, 2);
    {
      const u128 cs = apply_jump(jcs, mk128(sh.sx[k & 1][0], sh.sx[k & 1][1]));  // S(x + B + 32 lg + 1)
      reinterpret_cast<ulonglong2*>(L.CS(k))[lg] = ulonglong2{lo64(cs), hi64(cs)};
    }
    lds_release();
    if (lane == 0) lds_add(&sh.cs_done, 1u);
    if (w == 0) WSTAMP(P, k, 3);
    lds_wait(&sh.trans_done, (uint32_t)EW * (uint32_t)(k + 1), derr);  // every wave's masks; nobody reads the window now
    {
      const uint32_t c = lane < NS * EW ? (uint32_t)__builtin_popcountll(sh.mask[lane >> 3][lane & 7]) : 0u;
      const uint32_t ex = wave_incl_scan(c) - c;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        pre[s] = (uint32_t)__builtin_amdgcn_readlane((int)ex, s * EW + w);
        if ((dn >> s) & 1u) sh.r2s[pre[s] + mbcnt(bm[s])] = (uint16_t)(s * 512 + lg);
      }
    }
    lds_release();
    if (lane == 0) lds_add(&sh.r2s_done, 1u);
    if (w == 0) WSTAMP(P, k, 4);
    if (k + 1 < K) {
      lds_wait(&sh.sy_ready, (uint32_t)k + 1u, derr);
      const u128 Srw = mk128(sh.rw[(k + 1) & 1][0], sh.rw[(k + 1) & 1][1]);
      if (!(tmode & TM_NOFILL)) fill_window(L.RW, jrw, jrow, fr0, nrow, Srw, lane);
      lds_release();
      if (lane == 0) lds_add(&sh.fill_done, 1u);
      fill_target += EW;
#pragma unroll
      for (int s = 0; s < NS; ++s) arow[s] = action_row<NA>(anext[s], derr);
    }
    if (w == 0) WSTAMP(P, k, 5);
    if (w == EW - 1) WSTAMP(P, k, 15);
    WSTAMP(P, k, 24 + w);
    // ---- the exchange's outcome: the resetters' cells ----
    lds_wait(&sh.cells_done, (uint32_t)k + 1u, derr);
    if (w == 0) WSTAMP(P, k, 11);
    const uint32_t fix = sh.fix[k & 1];
    if (fix & 1u) {
      wg_env_slow<NS>(P, sh, tb, L.CS(k), k, stg, dn, pre, bm, ae);
    } else if (envcells) {
      wg_env_cells<NS>(P, sh, tb, L.CS(k), stg, dn, pre, bm, ae);
    } else {
#pragma unroll
      for (int s = 0; s < NS; ++s)
        if ((dn >> s) & 1u) ae[s] = reinterpret_cast<const uint16_t*>(stg)[2 * (s * 512 + lg)];
    }
    lds_release();
    if (lane == 0) lds_add(&sh.res_done, 1u);
    if (k == K - 1 && !(tmode & TM_NOSTORE)) {  // the launch's last step: its outputs straight from the env waves
      const uint32_t* st = reinterpret_cast<const uint32_t*>(stg);
      const size_t base = (size_t)k * B + e0 + (size_t)lg;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const uint32_t v = st[s * 512 + lg];
        const size_t e = base + (size_t)s * 512;
        obs[e] = tb.ocell(v & 0xFFFFu);
        rew[e] = (v & 0x10000u) ? P.r_goal : ((v & 0x40000u) ? P.r_wall : P.r_step);
        term[e] = (uint8_t)((v >> 16) & 1u);
        trunc[e] = (uint8_t)((v >> 17) & 1u);
      }
    }
    if ((fix & 2u) && k + 1 < K) {  // the prediction missed the window: regenerate it exactly
      fill_window(L.RW, jrw, jrow, fr0, nrow, mk128(sh.rw[(k + 1) & 1][0], sh.rw[(k + 1) & 1][1]), lane);
      lds_release();
      if (lane == 0) lds_add(&sh.fill_done, 1u);
      fill_target += EW;
    }
  }
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    aeg[e0 + (size_t)k * 512 + lg] = ae[k];
    acc.lens -= ae[k] >> 16;
  }
}

// ------------------------------------------------------------------ the store waves ----
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void nt_store(void* p, u32x4 v) { __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p)); }

// Step k's staging (final once every env wave has taken its resetters' cells) -> obs, reward, terminated,
// truncated in HBM, 16 envs per lane and chunk, while the env waves run the next steps.
template <int NS>
__device__ __forceinline__ void wg_store(const WgParams& P, WgShared& sh, const Tabs& tb, const Lds& L, int K,
                                         int32_t* __restrict__ obs, float* __restrict__ rew, uint8_t* __restrict__ term,
                                         uint8_t* __restrict__ trunc) {
  const int sl = (int)threadIdx.x - (EW + 1) * 64;  // 0..127
  const int lane = sl & 63;
  const int beta = (int)blockIdx.x, G = (int)gridDim.x;
  constexpr int E = NS * 512;
  const size_t B = (size_t)E * (size_t)G;
  const float rs = P.r_step, rwall = P.r_wall, rg = P.r_goal;
  const int tmode = P.tmode;
  uint32_t* derr = &P.ctl->err;
  lds_barrier();  // P1
  for (int k = 0; k + 1 < K; ++k) {  // (the env waves write the last step themselves)
    lds_wait(&sh.res_done, (uint32_t)EW * (uint32_t)(k + 1), derr);
    // and out of the way of the next step's transitions (the critical path): start once they are done, except for
    // a launch's last steps, whose copies are the launch's tail
    if (k + WG_EAGER_TAIL < K && !(tmode & TM_EAGERSTORE))
      lds_wait(&sh.trans_done, (uint32_t)EW * (uint32_t)(k + 2), derr);
    if (sl < 64) WSTAMP(P, k, 13);
    const uint32_t* st = reinterpret_cast<const uint32_t*>(L.stg(k, E));
    const size_t base = (size_t)k * B + (size_t)beta * E;
    // Lane-contiguous: in every store instruction consecutive lanes write consecutive 16 B (obs, reward) or 4 B
    // (terminated, truncated) of 4 envs each, whole cache lines per instruction (a lane-strided pattern left the
    // lines to be merged from partial writes and ran the output stream at a fraction of the HBM rate).
#if WG_SUNROLL == 4
#pragma unroll 4
#elif WG_SUNROLL == 1
#pragma unroll 1
#else
#pragma unroll 2
#endif
    for (int c = sl; c < E / 4 && !(tmode & TM_NOSTORE); c += SW * 64) {  // 4 envs per lane and iteration
      const uint4 x = reinterpret_cast<const uint4*>(st)[c];
      const uint32_t v[4] = {x.x, x.y, x.z, x.w};
      u32x4 o, r;
      uint32_t tm = 0, tr = 0;
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        o[z] = (uint32_t)tb.ocell(v[z] & 0xFFFFu);
        const float rr = (v[z] & 0x10000u) ? rg : ((v[z] & 0x40000u) ? rwall : rs);
        r[z] = __builtin_bit_cast(uint32_t, rr);
        tm |= ((v[z] >> 16) & 1u) << (8 * z);
        tr |= ((v[z] >> 17) & 1u) << (8 * z);
      }
      const size_t e = base + (size_t)c * 4;
      nt_store(obs + e, o);
      nt_store(rew + e, r);
      __builtin_nontemporal_store(tm, reinterpret_cast<uint32_t*>(term + e));
      __builtin_nontemporal_store(tr, reinterpret_cast<uint32_t*>(trunc + e));
      if (tmode & TM_THROTTLE) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // the staging buffer is free once its LDS reads are done (the stores' data left in registers)
    lds_release();
    if (lane == 0) lds_add(&sh.st_done, 1u);
    if (sl < 64) WSTAMP(P, k, 14);
  }
}

// ------------------------------------------------------------------ the kernel ----
template <int NS, int NA>
__global__ __launch_bounds__(TPB) void wgrid_rollout(const WgParams* __restrict__ Pp, int K, const int32_t* __restrict__ act,
                                                      int32_t* __restrict__ obs, float* __restrict__ rew,
                                                      uint8_t* __restrict__ term, uint8_t* __restrict__ trunc) {
  __shared__ WgShared sh;
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  // the step count in a scalar register for the whole launch (opaque to the compiler): the step loops would
  // otherwise re-read it from the kernarg segment, host memory unless HIP_FORCE_DEV_KERNARG
  asm volatile("" : "+s"(K));
  const WgParams& P = *Pp;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int E = NS * 512;
  if (tid == 0) LSTAMP(P, 0);
  // stage the table image (each thread's 16-B loads in flight before its LDS stores)
  // (the control and store waves; the env waves fill their first window meanwhile)
  if (wid >= EW && !(P.tmode & TM_NOTABLES)) {
    constexpr int CT = (NWAVES - EW) * 64;
    const int t = tid - EW * 64;
    const int n = P.lds.total >> 4;
    const uint4* s = reinterpret_cast<const uint4*>(P.limg);
    uint4* d = reinterpret_cast<uint4*>(dyn);
    for (int i0 = t; i0 < n; i0 += 4 * CT) {
      uint4 v0, v1, v2, v3;
      const bool a1 = i0 + CT < n, a2 = i0 + 2 * CT < n, a3 = i0 + 3 * CT < n;
      v0 = s[i0];
      if (a1) v1 = s[i0 + CT];
      if (a2) v2 = s[i0 + 2 * CT];
      if (a3) v3 = s[i0 + 3 * CT];
      d[i0] = v0;
      if (a1) d[i0 + CT] = v1;
      if (a2) d[i0 + 2 * CT] = v2;
      if (a3) d[i0 + 3 * CT] = v3;
    }
    if (wid == EW) LSTAMP(P, 5);
    if (wid == EW + 1) LSTAMP(P, 6);
  }
  if (tid == EW * 64) {
    sh.trans_done = sh.cs_done = sh.r2s_done = sh.fill_done = sh.res_done = sh.st_done = 0;
    sh.sx_ready = sh.sy_ready = sh.cells_done = sh.pro = 0;
    if (!(P.tmode & TM_OLDPRO)) sh.fill_done = EW;  // step 0's words: every env wave wrote its own before P1
    sh.fix[0] = sh.fix[1] = 0;
  }
  const Tabs tb(dyn, P);
  const Lds L(dyn, P, E);
  Acc acc;
  if (wid == CWAVE) {
    __builtin_amdgcn_s_setprio(3);  // the exchange is on every step's critical path
    wg_ctrl<NS, NA>(P, sh, tb, L, K);
  } else if (wid > CWAVE) {
    if (P.tmode & TM_STORELOW) __builtin_amdgcn_s_setprio(0);
    else __builtin_amdgcn_s_setprio(1);
    wg_store<NS>(P, sh, tb, L, K, obs, rew, term, trunc);
  } else {
    wg_env<NS, NA>(P, sh, tb, L, dyn, act, K, acc, obs, rew, term, trunc);
  }
  // episode statistics of the launch (env waves; the others contribute zeros)
  float rsum = 0.f;
  uint32_t nst = 0;
  if (wid < EW) {
    const uint32_t steps = (uint32_t)(NS * K);
    acc.lens += steps;
    nst = steps;
    rsum = (float)acc.ngoal * P.r_goal + (float)acc.nwall * P.r_wall + (float)(steps - acc.ngoal - acc.nwall) * P.r_step;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    rsum += __shfl_xor(rsum, d, 64);
    acc.eps += __shfl_xor(acc.eps, d, 64);
    acc.lens += __shfl_xor(acc.lens, d, 64);
    nst += __shfl_xor(nst, d, 64);
  }
  __shared__ float m_r[NWAVES];
  __shared__ uint32_t m_e[NWAVES], m_l[NWAVES], m_n[NWAVES];
  if (lane == 0) {
    m_r[wid] = rsum;
    m_e[wid] = acc.eps;
    m_l[wid] = acc.lens;
    m_n[wid] = nst;
  }
  __syncthreads();
  if (tid == 0) {
    float rr = 0;
    uint32_t e = 0, l = 0, n = 0;
    for (int w = 0; w < NWAVES; ++w) {
      rr += m_r[w];
      e += m_e[w];
      l += m_l[w];
      n += m_n[w];
    }
    MetricSlot& m = P.mslot[blockIdx.x];
    atomicAdd(&m.return_sum, (double)rr);
    atomicAdd(&m.episodes, (unsigned long long)e);
    atomicAdd(&m.length_sum, (unsigned long long)l);
    atomicAdd(&m.env_steps, (unsigned long long)n);
  }
#ifdef GP_STAMPS
  __syncthreads();
  for (int i = tid; i < 32 * 32; i += TPB) P.dbg[(size_t)blockIdx.x * 32 * 32 + i] = g_stamp[i];
  if (tid < 8 && tid != 4) P.dbg[(size_t)256 * 32 * 32 + (size_t)blockIdx.x * 8 + tid] = g_stamp[32 * 32 + tid];
  if (tid == 0) {  // kernel end (after the copy-out)
    unsigned long long t_;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
    P.dbg[(size_t)256 * 32 * 32 + (size_t)blockIdx.x * 8 + 4] = t_;
  }
#endif
}

template <int NS, int NA>
void launch_one(const WgArgs& a, int G, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL((wgrid_rollout<NS, NA>), dim3((unsigned)G), dim3(TPB), lds, s, a.P, a.K, a.act, a.obs, a.rew,
                     a.term, a.trunc);
}
template <int NS, int NA>
int fits_one(size_t lds) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, wgrid_rollout<NS, NA>, TPB, lds) != hipSuccess) return 0;
  return occ;
}

}  // namespace

int wgrid_launch(const WgArgs& a, int NS, int NA, int G, size_t lds, hipStream_t s) {
  switch (NS * 16 + NA) {
    case 1 * 16 + 4: launch_one<1, 4>(a, G, lds, s); break;
    case 2 * 16 + 4: launch_one<2, 4>(a, G, lds, s); break;
    case 4 * 16 + 4: launch_one<4, 4>(a, G, lds, s); break;
    case 8 * 16 + 4: launch_one<8, 4>(a, G, lds, s); break;
    case 1 * 16 + 8: launch_one<1, 8>(a, G, lds, s); break;
    case 2 * 16 + 8: launch_one<2, 8>(a, G, lds, s); break;
    case 4 * 16 + 8: launch_one<4, 8>(a, G, lds, s); break;
    case 8 * 16 + 8: launch_one<8, 8>(a, G, lds, s); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

int wgrid_fits(int NS, int NA, size_t lds) {
  switch (NS * 16 + NA) {
    case 1 * 16 + 4: return fits_one<1, 4>(lds);
    case 2 * 16 + 4: return fits_one<2, 4>(lds);
    case 4 * 16 + 4: return fits_one<4, 4>(lds);
    case 8 * 16 + 4: return fits_one<8, 4>(lds);
    case 1 * 16 + 8: return fits_one<1, 8>(lds);
    case 2 * 16 + 8: return fits_one<2, 8>(lds);
    case 4 * 16 + 8: return fits_one<4, 8>(lds);
    case 8 * 16 + 8: return fits_one<8, 8>(lds);
  }
  return 0;
}
