// grid.hip — GP_KIND_GRID: batched Multistory FourRooms (msrooms.py) and ROOMS (rooms.py).
//
// One env per lane-slot, 4 consecutive envs per thread (16-B vector loads/stores), 256 threads
// per block (1024 envs per block). State in HBM is one uint32 per env (agent cell | elapsed<<16)
// plus a uint16 goal cell when goals are random. Static tables (move table with the stair
// transit folded in, Hansen bases, obs windows, valid-cell lists) are built on the host once.
//
// RNG modes
//   GP_RNG_NUMPY  seed-identical to the reference's numpy Generator(PCG64):
//     step(): random(B) -> each env jumps the PCG64 state to its own stream position (radix-64
//     jump tables), the action-failure compare is done on integers (k > floor(cumsum*2^53));
//     resets: choice(valid, b) over the resetting envs in ascending order = Lemire-32 draws on
//     the buffered 32-bit halves. The resetting envs' ranks come from a single-pass
//     decoupled-lookback scan (ticket-ordered blocks, agent-scope status words). Lemire
//     rejections (p ~ 1e-8 per draw) are detected per word position in the same pass and take
//     an exact block-serial slow path. The last block publishes the next PCG64 state.
//   GP_RNG_PHILOX counter-based Philox4x32-10 keyed by (seed, env, global step): no scan, so K
//     steps fuse into one launch with the env state in registers (gp_rollout).
//   GP_RNG_REPLAY pre-decided per-env draws (parity harness for the Philox path).
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>

#include "gp_internal.h"
#include "grid_shared.h"

namespace {

constexpr int TPB = 256;
constexpr int EPT = 4;
constexpr int EPB = TPB * EPT;
constexpr uint32_t SPIN_LIMIT = 1u << 24;  // default polls before a persistent wait gives up (GP_SPIN_LIMIT)
constexpr int MAX_TPB2 = 1024;  // max tiles per K2 block (B <= 256 * 1024 * EPB)
// Longest launch on the windowed kernel (wgrid.hip); longer launches run the fused kernel (grid_rollout_numpy).
// In-call A/Bs on MI355X (profiles/r05_ab_kernel_by_K.txt).
#ifndef WG_KMAX
#define WG_KMAX 24
#endif
// Windowed kernel: window rows per env wave, per-SIMD deltas (wg_fill_simd's encoding; 0 = even rows).
// Per-wave deltas on top (wg_fill_wave's encoding): the first env wave of each SIMD (the older one, issued first at
// equal priority) +1 row, the second -1, so that the second does not fill alone at the end of the step.
#ifndef WG_FILL_WAVE
#define WG_FILL_WAVE 0xFFFF1111u
#endif
#ifndef WG_FILL_SIMD
#define WG_FILL_SIMD 0x3FFF  // SIMD 3 (no control or store wave) +3 rows per env wave, SIMDs 0-2 -1 (profiles/r06_prologue_fill_rows_ab.txt)
#endif

struct GridLdsTab {
  int32_t off, bytes;
};
struct GridLds {  // where the fused kernel stages the lookup tables in dynamic LDS
  int32_t total;
  GridLdsTab move, hbase, hvec, t1, t2, coords, window, gv, av, doff, jt, jt8, ofix, avo;
};

struct GridDev {
  int32_t B, nblk;
  int32_t nact, ncells;
  int32_t obs_kind, obs_dirs, obs_goal, obs_n, obs_width, ndim;
  int32_t fixed_goal, fixed_agent;  // -1 random
  int32_t goal_gz, goal_gy, goal_gx; // coordinates of the fixed goal (may be off-grid)
  int32_t n_goal_valid, n_agent_valid;
  uint32_t thr_goal, thr_agent;
  int32_t time_limit;
  float r_step, r_wall, r_goal;
  int32_t goal_code;
  const uint16_t* move;
  const uint64_t* thr;
  const uint16_t* goal_valid;
  const uint16_t* agent_valid;
  const uint32_t* hbase;
  const int32_t* doff;
  const uint8_t* hvec;
  const int32_t* t1;
  const int32_t* t2;
  const int16_t* coords;
  const uint8_t* window;
  const PcgJump* jt;
  const PcgJump* lt4;   // [256] jump by 4t  (per-thread action-draw offset inside a tile)
  const PcgJump* lt2;   // [256] jump by 2t  (per-thread word-check offset inside a tile)
  const PcgJump* tja;   // [nblk] jump by tile*EPB + 1      (tile base of the action draws)
  const PcgJump* tjw;   // [nblk] jump by B + tile*EPB/2     (tile base of the word checks)
  MetricSlot* mslot;
  uint32_t* ae;
  uint16_t* goal;
  GridCtl* ctl;
  uint32_t* tcount;  // [nblk] resets per tile (K1 -> K2)
  uint16_t* tlist;   // [nblk*EPB] local offsets of a tile's resetting envs, ascending
  uint32_t* rflag;   // [<=256] K2 per-block rejection flags, tagged with the epoch
  // fused numpy rollout
  int32_t fnt;              // fused tiles
  int32_t ftile, faw;       // envs per fused tile (512, 1024 or 2048 = FEPB) and the env waves that own them
                            // (ftile / 256; the other env waves of the block only join the barriers)
  const PcgJump* ftj;       // [fnt] jump by tau*ftile + 1
  const PcgJump* flt4;      // [FTPB] jump by 4t
  const PcgJump* fjB;       // [2] jump by B, jump by G * ftile (a block's tile stride)
  uint64_t* fslot;          // [2][3][G] tagged block granules, then [2][fnt] tile words
  unsigned long long* dbg;  // GP_STAMPS diagnostic builds: [G][64][8] s_memtime stamps
  GridLds lds;
  const char* limg;         // [lds.total] the tables laid out exactly as staged in LDS (one copy loop)
  const int32_t* ofix;      // Hansen obs of each agent cell for the fixed goal (empty otherwise)
  const uint32_t* avo;      // with ofix: {agent_valid[j], ofix[agent_valid[j]]} pairs (one load per drawn agent)
  const GridDev* self;      // device copy of this struct (for out-of-line slow-path helpers)
  const PcgJump* jt8;       // [2][256] radix-256 jumps: d and 256*d steps (fused kernel: jumps < 2^16)
  int32_t xmode;            // fused exchange: 0 = block-0 aggregator + per-tile words, 1 = all-gather
  uint32_t spin_limit;      // polls before a cross-block wait gives up and flags GridCtl::err
  int32_t fault_block;      // test knob (GP_FAULT_BLOCK): this block never publishes (forces the timeout); -1 off
  int32_t spw_on;           // staged fused kernel: the store waves precompute speculative word windows (SPW_*)
  // philox / replay
  uint32_t key0, key1;
  const uint64_t* rp_u;
  const int32_t* rp_goal;
  const int32_t* rp_agent;
};

// ------------------------------------------------------------------ cross-block waits ----
// Every cross-block wait of the persistent numpy-mode kernels polls through spin_give_up: it gives up
// after p.spin_limit polls (setting GridCtl::err bit 0, which the host turns into GP_E_DEVICE), and
// as soon as any other wave has flagged, so that a grid that cannot make progress (blocks not
// co-resident) still drains: every wave reaches the end of the kernel, the results are flagged invalid.
__device__ __forceinline__ bool spin_give_up(const GridDev& p, uint32_t& spins) {
  ++spins;
  if ((spins & 63u) == 0 &&
      (__hip_atomic_load(&p.ctl->err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & GP_DERR_TIMEOUT))
    return true;
  if (spins > p.spin_limit) {
    atomicOr(&p.ctl->err, GP_DERR_TIMEOUT);
    return true;
  }
  return false;
}

// ------------------------------------------------------------------ vector I/O helpers ----
__device__ __forceinline__ bool full_aligned(const void* p, int env0, int B, int esz) {
  return env0 + 3 < B && ((((uintptr_t)p) + (size_t)env0 * esz) & (size_t)(4 * esz - 1)) == 0;
}
template <class T>
__device__ __forceinline__ void load4(const T* __restrict__ p, int env0, int B, T (&v)[4]) {
  if (full_aligned(p, env0, B, sizeof(T))) {
    if constexpr (sizeof(T) == 4) {
      uint4 q = *reinterpret_cast<const uint4*>(p + env0);
      v[0] = __builtin_bit_cast(T, q.x); v[1] = __builtin_bit_cast(T, q.y);
      v[2] = __builtin_bit_cast(T, q.z); v[3] = __builtin_bit_cast(T, q.w);
    } else if constexpr (sizeof(T) == 2) {
      uint2 q = *reinterpret_cast<const uint2*>(p + env0);
      v[0] = (T)(q.x & 0xFFFF); v[1] = (T)(q.x >> 16); v[2] = (T)(q.y & 0xFFFF); v[3] = (T)(q.y >> 16);
    } else {
      uint32_t q = *reinterpret_cast<const uint32_t*>(p + env0);
      v[0] = (T)(q & 0xFF); v[1] = (T)((q >> 8) & 0xFF); v[2] = (T)((q >> 16) & 0xFF); v[3] = (T)(q >> 24);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (env0 + i < B) ? p[env0 + i] : (T)0;
  }
}
template <class T>
__device__ __forceinline__ void store4(T* __restrict__ p, int env0, int B, const T (&v)[4]) {
  if (full_aligned(p, env0, B, sizeof(T))) {
    if constexpr (sizeof(T) == 4) {
      uint4 q;
      q.x = __builtin_bit_cast(uint32_t, v[0]); q.y = __builtin_bit_cast(uint32_t, v[1]);
      q.z = __builtin_bit_cast(uint32_t, v[2]); q.w = __builtin_bit_cast(uint32_t, v[3]);
      *reinterpret_cast<uint4*>(p + env0) = q;
    } else if constexpr (sizeof(T) == 2) {
      uint2 q;
      q.x = (uint32_t)(uint16_t)v[0] | ((uint32_t)(uint16_t)v[1] << 16);
      q.y = (uint32_t)(uint16_t)v[2] | ((uint32_t)(uint16_t)v[3] << 16);
      *reinterpret_cast<uint2*>(p + env0) = q;
    } else {
      uint32_t q = (uint32_t)(uint8_t)v[0] | ((uint32_t)(uint8_t)v[1] << 8) | ((uint32_t)(uint8_t)v[2] << 16) |
                   ((uint32_t)(uint8_t)v[3] << 24);
      *reinterpret_cast<uint32_t*>(p + env0) = q;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (env0 + i < B) p[env0 + i] = v[i];
  }
}

// Fused-kernel variants: the host guarantees 16-B aligned base pointers (else the fused path is not
// taken), so only the last, partial quad of a ragged batch takes the per-element path.
template <class T>
__device__ __forceinline__ void load4f(const T* __restrict__ p, int env0, int B, T (&v)[4]) {
  if (env0 + 3 < B) {
    if constexpr (sizeof(T) == 4) {
      const uint4 q = *reinterpret_cast<const uint4*>(p + env0);
      v[0] = __builtin_bit_cast(T, q.x); v[1] = __builtin_bit_cast(T, q.y);
      v[2] = __builtin_bit_cast(T, q.z); v[3] = __builtin_bit_cast(T, q.w);
    } else {
      const uint2 q = *reinterpret_cast<const uint2*>(p + env0);
      v[0] = (T)(q.x & 0xFFFF); v[1] = (T)(q.x >> 16); v[2] = (T)(q.y & 0xFFFF); v[3] = (T)(q.y >> 16);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (env0 + i < B) ? p[env0 + i] : (T)0;
  }
}
template <class T>
__device__ __forceinline__ void store4f(T* __restrict__ p, int env0, int B, const T (&v)[4]) {
  if (env0 + 3 < B) {
    if constexpr (sizeof(T) == 4) {
      uint4 q;
      q.x = __builtin_bit_cast(uint32_t, v[0]); q.y = __builtin_bit_cast(uint32_t, v[1]);
      q.z = __builtin_bit_cast(uint32_t, v[2]); q.w = __builtin_bit_cast(uint32_t, v[3]);
      *reinterpret_cast<uint4*>(p + env0) = q;
    } else if constexpr (sizeof(T) == 2) {
      uint2 q;
      q.x = (uint32_t)(uint16_t)v[0] | ((uint32_t)(uint16_t)v[1] << 16);
      q.y = (uint32_t)(uint16_t)v[2] | ((uint32_t)(uint16_t)v[3] << 16);
      *reinterpret_cast<uint2*>(p + env0) = q;
    } else {
      *reinterpret_cast<uint32_t*>(p + env0) = (uint32_t)(uint8_t)v[0] | ((uint32_t)(uint8_t)v[1] << 8) |
                                               ((uint32_t)(uint8_t)v[2] << 16) | ((uint32_t)(uint8_t)v[3] << 24);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (env0 + i < B) p[env0 + i] = v[i];
  }
}

// ------------------------------------------------------------------ lookup-table access ----
// GTabs reads the tables from global memory (L1/L2 hot); LTabs from the fused kernel's LDS copy.
struct GTabs {
  const GridDev& p;
  __device__ __forceinline__ uint16_t move(int i) const { return p.move[i]; }
  __device__ __forceinline__ uint32_t hbase(int i) const { return p.hbase[i]; }
  __device__ __forceinline__ int32_t doff(int i) const { return p.doff[i]; }
  __device__ __forceinline__ uint8_t hvec(int i) const { return p.hvec[i]; }
  __device__ __forceinline__ int32_t t1(int i) const { return p.t1[i]; }
  __device__ __forceinline__ int32_t t2(int i) const { return p.t2[i]; }
  __device__ __forceinline__ bool has_t2() const { return p.t2 != nullptr; }
  __device__ __forceinline__ int16_t coords(int i) const { return p.coords[i]; }
  __device__ __forceinline__ uint8_t window(int i) const { return p.window[i]; }
  __device__ __forceinline__ uint16_t gv(int i) const { return p.goal_valid[i]; }
  __device__ __forceinline__ uint16_t av(int i) const { return p.agent_valid[i]; }
  __device__ __forceinline__ bool has_ofix() const { return p.ofix != nullptr; }
  __device__ __forceinline__ int32_t ofix(int i) const { return p.ofix[i]; }
};
struct LTabs {
  const GridDev& p;
  const char* dyn;
  template <class T>
  __device__ __forceinline__ T at(const GridLdsTab& t, int i) const {
    return reinterpret_cast<const T*>(dyn + t.off)[i];
  }
  __device__ __forceinline__ uint16_t move(int i) const { return at<uint16_t>(p.lds.move, i); }
  // move-table entry at byte offset `b` (= (cell * NA + action) * 2)
  __device__ __forceinline__ uint16_t move_b(uint32_t b) const {
    return *reinterpret_cast<const uint16_t*>(dyn + p.lds.move.off + b);
  }
  __device__ __forceinline__ uint32_t hbase(int i) const { return at<uint32_t>(p.lds.hbase, i); }
  __device__ __forceinline__ int32_t doff(int i) const { return at<int32_t>(p.lds.doff, i); }
  __device__ __forceinline__ uint8_t hvec(int i) const { return at<uint8_t>(p.lds.hvec, i); }
  __device__ __forceinline__ int32_t t1(int i) const { return at<int32_t>(p.lds.t1, i); }
  __device__ __forceinline__ int32_t t2(int i) const { return at<int32_t>(p.lds.t2, i); }
  __device__ __forceinline__ bool has_t2() const { return p.lds.t2.bytes > 0; }
  __device__ __forceinline__ int16_t coords(int i) const { return at<int16_t>(p.lds.coords, i); }
  __device__ __forceinline__ uint8_t window(int i) const { return at<uint8_t>(p.lds.window, i); }
  __device__ __forceinline__ uint16_t gv(int i) const { return at<uint16_t>(p.lds.gv, i); }
  __device__ __forceinline__ uint16_t av(int i) const { return at<uint16_t>(p.lds.av, i); }
  __device__ __forceinline__ const PcgJump* jt() const { return reinterpret_cast<const PcgJump*>(dyn + p.lds.jt.off); }
  __device__ __forceinline__ const PcgJump* jt8() const { return reinterpret_cast<const PcgJump*>(dyn + p.lds.jt8.off); }
  __device__ __forceinline__ bool has_ofix() const { return p.lds.ofix.bytes > 0; }
  __device__ __forceinline__ int32_t ofix(int i) const { return at<int32_t>(p.lds.ofix, i); }
  __device__ __forceinline__ bool has_avo() const { return p.lds.avo.bytes > 0; }
  __device__ __forceinline__ uint2 avo(int i) const { return at<uint2>(p.lds.avo, i); }
};

// ------------------------------------------------------------------ observation builders ----
// GP_OBS_HANSEN:     hbase[agent] * goal_mult (msrooms.py:162-189 ternary / observations.py:44-71 binary)
// GP_OBS_HANSEN_VEC: hvec[agent][i], goal -> goal_code    (msrooms.py:131-159 / observations.py:106-131)
// GP_OBS_TABLE:      t1[agent] + t2[goal]                 (mdp / room scalars: rooms.py:23-48, msrooms.py:217-235)
// GP_OBS_COORDS:     (z,)y,x of agent (+ goal)            (vector mdp: rooms.py:31-37, msrooms.py:218-224)
// GP_OBS_WINDOW:     n x n window, goal -> 2              (observations.py:74-103)
template <int OK, class TB>
__device__ __forceinline__ void write_obs(const GridDev& p, const TB& tb, int env, int agent, int goal,
                                          void* __restrict__ obs) {
  const bool gvalid = (unsigned)goal < (unsigned)p.ncells;
  if constexpr (OK == GP_OBS_HANSEN) {
    int mult = 1;
    if (gvalid) {
      int diff = goal - agent;
      for (int i = p.obs_dirs - 1; i >= 0; --i)
        if (diff == tb.doff(i)) mult = i + 1;
    }
    ((int32_t*)obs)[env] = (int32_t)tb.hbase(agent) * mult;
  } else if constexpr (OK == GP_OBS_HANSEN_VEC) {
    uint8_t* o = (uint8_t*)obs + (size_t)env * p.obs_width;
    int diff = goal - agent;
    for (int i = 0; i < p.obs_dirs; ++i) {
      uint8_t v = tb.hvec(agent * p.obs_dirs + i);
      if (p.obs_goal && gvalid && diff == tb.doff(i)) v = (uint8_t)p.goal_code;
      o[i] = v;
    }
  } else if constexpr (OK == GP_OBS_TABLE) {
    int32_t v = tb.t1(agent);
    if (tb.has_t2()) v += tb.t2(goal);
    ((int32_t*)obs)[env] = v;
  } else if constexpr (OK == GP_OBS_COORDS) {
    int32_t* o = (int32_t*)obs + (size_t)env * p.obs_width;
    int k = 0;
    if (p.ndim == 3) o[k++] = tb.coords(agent * 3);
    o[k++] = tb.coords(agent * 3 + 1);
    o[k++] = tb.coords(agent * 3 + 2);
    if (p.obs_goal) {
      int gz, gy, gx;
      if (gvalid) {
        gz = tb.coords(goal * 3); gy = tb.coords(goal * 3 + 1); gx = tb.coords(goal * 3 + 2);
      } else {
        gz = p.goal_gz; gy = p.goal_gy; gx = p.goal_gx;
      }
      if (p.ndim == 3) o[k++] = gz;
      o[k++] = gy;
      o[k++] = gx;
    }
  } else {  // GP_OBS_WINDOW
    const int n = p.obs_n, nn = n * n, h = n / 2;
    uint8_t* o = (uint8_t*)obs + (size_t)env * nn;
    for (int k = 0; k < nn; ++k) o[k] = tb.window(agent * nn + k);
    if (gvalid) {
      const int az = tb.coords(agent * 3), ay = tb.coords(agent * 3 + 1), ax = tb.coords(agent * 3 + 2);
      const int gz = tb.coords(goal * 3), gy = tb.coords(goal * 3 + 1), gx = tb.coords(goal * 3 + 2);
      int dy = gy - ay, dx = gx - ax;
      if (gz == az && dy >= -h && dy <= n - 1 - h && dx >= -h && dx <= n - 1 - h) o[(dy + h) * n + (dx + h)] = 2;
    }
  }
}

// Scalar obs of one env (GP_OBS_HANSEN / GP_OBS_TABLE), as write_obs4 computes it.
template <int OK, class TB>
__device__ __forceinline__ int32_t obs_value(const GridDev& p, const TB& tb, int a, int g) {
  if constexpr (OK == GP_OBS_HANSEN) {
    int mult = 1;
    if ((unsigned)g < (unsigned)p.ncells) {
      int diff = g - a;
      for (int d = p.obs_dirs - 1; d >= 0; --d)
        if (diff == tb.doff(d)) mult = d + 1;
    }
    return (int32_t)tb.hbase(a) * mult;
  } else {
    return tb.t1(a) + (tb.has_t2() ? tb.t2(g) : 0);
  }
}

// The same with the goal-direction offsets held in registers (dof[d] = doff(d) for d < obs_dirs, else a
// value no cell difference takes): no dependent LDS loads, just the hbase gather.
template <int OK, class TB>
__device__ __forceinline__ int32_t obs_value_r(const GridDev& p, const TB& tb, int a, int g, const int (&dof)[8]) {
  if constexpr (OK == GP_OBS_HANSEN) {
    if (tb.has_ofix()) return tb.ofix(a);  // fixed goal: the obs is a function of the agent cell (one lookup)
    int mult = 1;
    const int diff = g - a;
#pragma unroll
    for (int d = 7; d >= 0; --d) mult = diff == dof[d] ? d + 1 : mult;
    if ((unsigned)g >= (unsigned)p.ncells) mult = 1;
    return (int32_t)tb.hbase(a) * mult;
  } else {
    return tb.t1(a) + (tb.has_t2() ? tb.t2(g) : 0);
  }
}

template <int OK, class TB, bool ALIGNED = false>
__device__ __forceinline__ void write_obs4(const GridDev& p, const TB& tb, int env0, const int (&agent)[4],
                                           const int (&goal)[4], void* __restrict__ obs) {
  if constexpr (OK == GP_OBS_HANSEN || OK == GP_OBS_TABLE) {
    int32_t v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int a = agent[i], g = goal[i];
      if constexpr (OK == GP_OBS_HANSEN) {
        int mult = 1;
        if ((unsigned)g < (unsigned)p.ncells) {
          int diff = g - a;
          for (int d = p.obs_dirs - 1; d >= 0; --d)
            if (diff == tb.doff(d)) mult = d + 1;
        }
        v[i] = (int32_t)tb.hbase(a) * mult;
      } else {
        v[i] = tb.t1(a) + (tb.has_t2() ? tb.t2(g) : 0);
      }
    }
    if constexpr (ALIGNED)
      store4f<int32_t>((int32_t*)obs, env0, p.B, v);
    else
      store4<int32_t>((int32_t*)obs, env0, p.B, v);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (env0 + i < p.B) write_obs<OK>(p, tb, env0 + i, agent[i], goal[i], obs);
  }
}

// ------------------------------------------------------------------ numpy word stream ----
// Absolute 32-bit word index w (counted from the first word after the step's random(B)) ->
// the u64 draw index and half, honouring numpy's buffered half (has_uint32 at step start).
struct Stream {
  u128 s0, inc;
  uint32_t h0, u0;
  uint32_t U0;  // u64 draws consumed before the word stream starts (B for step, 0 for reset)
};

__device__ __forceinline__ uint32_t word_at(const GridDev& p, const Stream& st, uint32_t w) {
  if (st.h0 && w == 0) return st.u0;
  uint32_t ww = w - st.h0;
  uint32_t q = ww >> 1;
  uint64_t x = pcg_output(pcg_jump(p.jt, st.s0, st.U0 + q + 1));
  return (ww & 1) ? (uint32_t)(x >> 32) : (uint32_t)x;
}

// The 4 consecutive words w0..w0+3.
__device__ __forceinline__ void words4(const GridDev& p, const Stream& st, uint32_t w0, uint32_t (&out)[4]) {
  uint32_t k = 0;
  uint32_t w = w0;
  if (st.h0 && w == 0) {
    out[0] = st.u0;
    k = 1;
    w = 1;
  }
  uint32_t ww = w - st.h0;
  uint32_t q = ww >> 1;
  u128 s = pcg_jump(p.jt, st.s0, st.U0 + q + 1);
  uint64_t x = pcg_output(s);
  uint32_t half = ww & 1;
  for (; k < 4; ++k) {
    out[k] = half ? (uint32_t)(x >> 32) : (uint32_t)x;
    if (half) {
      s = pcg_step(s, st.inc);
      x = pcg_output(s);
    }
    half ^= 1;
  }
}

// Sequential reader of the 32-bit word stream from absolute word index w (numpy next_uint32
// semantics: buffered half first if present, then low/high halves of successive u64 draws).
struct WordIter {
  u128 s;
  uint64_t x;
  uint32_t half;
  bool buf;
  __device__ __forceinline__ void init(const GridDev& p, const Stream& st, uint32_t w) {
    if (st.h0 && w == 0) {
      buf = true;
      s = pcg_jump(p.jt, st.s0, st.U0);  // state before u64 #0
      x = 0;
      half = 0;
    } else {
      buf = false;
      const uint32_t ww = w - st.h0;
      s = pcg_jump(p.jt, st.s0, st.U0 + (ww >> 1) + 1);
      x = pcg_output(s);
      half = ww & 1;
    }
  }
  __device__ __forceinline__ uint32_t next(const Stream& st) {
    if (buf) {
      buf = false;
      s = pcg_step(s, st.inc);
      x = pcg_output(s);
      half = 0;
      return st.u0;
    }
    const uint32_t v = half ? (uint32_t)(x >> 32) : (uint32_t)x;
    if (half) {
      s = pcg_step(s, st.inc);
      x = pcg_output(s);
    }
    half ^= 1;
    return v;
  }
};

struct ResolveShared {
  uint32_t red[TPB / 64];
  uint32_t red2[TPB / 64];
  uint32_t tpre[MAX_TPB2 + 1];   // exclusive prefix of this block's tile counts
  uint32_t P, btot, n, anyrej, w1, bcast;
  uint32_t pos[EPB];              // slow path: accepted-word positions of one batch of ranks
  uint32_t pos2[EPB];
};

__device__ __forceinline__ uint32_t ld_flag(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <class T>
__device__ __forceinline__ T block_sum(T v, T* red) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int w = 0; w < TPB / 64; ++w) s += red[w];
  return s;
}

// Slow path (a Lemire rejection somewhere): wave 0 walks the word stream from `wbase`,
// recording the absolute positions of the accepted draws with rank in [jlo, jhi) into out.
// Returns (to wave 0) the position after the last recorded draw.
__device__ __noinline__ uint32_t scan_accepted(const GridDev* __restrict__ gp, const Stream st, uint32_t wbase, uint32_t n, uint32_t thr,
                                  uint32_t jlo, uint32_t jhi, uint32_t* out) {
  const GridDev& p = *gp;
  const int lane = threadIdx.x & 63;
  uint32_t acc = 0, pos = wbase, after = wbase;
  while (acc < jhi) {
    const uint32_t w = word_at(p, st, pos + lane);
    const bool ok = !lemire_rejected(w, n, thr);
    const unsigned long long m = __ballot(ok);
    const uint32_t below = (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
    const uint32_t j = acc + below;
    if (ok && j >= jlo && j < jhi) {
      if (out) out[j - jlo] = pos + lane;
      if (j == jhi - 1) after = pos + lane + 1;
    }
    acc += (uint32_t)__builtin_popcountll(m);
    pos += 64;
  }
  uint32_t a = after;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) a = max(a, __shfl_xor(a, d, 64));
  return a;
}

// Per-block metrics (episode count / return / length / env-steps) into the block's own slot.
__device__ void add_metrics(const GridDev& p, float rsum, uint32_t eps, uint32_t lens, uint32_t nsteps) {
  __shared__ float s_r[TPB / 64];
  __shared__ uint32_t s_e[TPB / 64], s_l[TPB / 64], s_n[TPB / 64];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    rsum += __shfl_xor(rsum, d, 64);
    eps += __shfl_xor(eps, d, 64);
    lens += __shfl_xor(lens, d, 64);
    nsteps += __shfl_xor(nsteps, d, 64);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { s_r[wid] = rsum; s_e[wid] = eps; s_l[wid] = lens; s_n[wid] = nsteps; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0; uint32_t e = 0, l = 0, n = 0;
    for (int w = 0; w < TPB / 64; ++w) { r += s_r[w]; e += s_e[w]; l += s_l[w]; n += s_n[w]; }
    MetricSlot& m = p.mslot[blockIdx.x];
    m.return_sum += (double)r;
    m.episodes += e;
    m.length_sum += l;
    m.env_steps += n;
  }
}

// ------------------------------------------------------------------ the env transition ----
// msrooms.py:398-411 / rooms.py:208-220 for one env, given its effective action.
struct Trans {
  int agent, goal, elapsed;
  float rew;
  uint8_t term, trunc;
};

__device__ __forceinline__ uint32_t effective_action(const uint64_t* __restrict__ thr, int nact, int a, uint64_t k) {
  // action_utils.py:84-90: #{j : cumsum(P[a])_j < k*2^-53}  <=>  #{j : k > floor(cumsum_j * 2^53)}
  uint32_t e = 0;
  const uint64_t* t = thr + a * nact;
  for (int j = 0; j < nact; ++j) e += (k > t[j]) ? 1u : 0u;
  return e;
}

template <class TB>
__device__ __forceinline__ Trans transition(const GridDev& p, const TB& tb, uint32_t ae, int goal, int a,
                                            uint64_t k53, const uint64_t* thr) {
  Trans t;
  const int agent = (int)(ae & 0xFFFF);
  t.elapsed = (int)(ae >> 16) + 1;
  if (action_out_of_range(a, p.nact)) flag_bad_action(&p.ctl->err);  // IndexError in the reference: flagged
  if (a < 0) a += p.nact;               // numpy negative indexing of action_matrix[action]
  a = min(max(a, 0), p.nact - 1);       // (clamped after flagging so the launch stays in bounds)
  const uint32_t eff = min(effective_action(thr, p.nact, a, k53), (uint32_t)p.nact - 1);
  const uint16_t m = tb.move(agent * p.nact + (int)eff);
  t.agent = m & 0x7FFF;
  const bool blocked = (m >> 15) != 0;
  t.goal = goal;
  t.term = (t.agent == goal) ? 1 : 0;
  t.rew = t.term ? p.r_goal : (blocked ? p.r_wall : p.r_step);
  t.trunc = (t.elapsed > p.time_limit) ? 1 : 0;
  return t;
}

// ------------------------------------------------------------------ kernels: numpy mode ----
// K1 — the streaming step (msrooms.py:398-411): random(B) action-failure draws, move, reward,
// terminated/truncated, and every output for every env. Envs that reset get elapsed = 0 and
// provisional agent/goal/obs; their indices go to a per-tile list for K2. No inter-block
// dependency: a pure load -> compute -> store kernel.
template <int OK>
__global__ __launch_bounds__(TPB) void grid_step_numpy(GridDev p, const int32_t* __restrict__ act,
                                                       void* __restrict__ obs, float* __restrict__ rew,
                                                       uint8_t* __restrict__ term, uint8_t* __restrict__ trunc) {
  __shared__ uint64_t s_thr[64];
  __shared__ uint32_t s_red[TPB / 64];
  if (threadIdx.x < p.nact * p.nact) s_thr[threadIdx.x] = p.thr[threadIdx.x];
  const GridCtl* C = p.ctl;
  const u128 s0 = mk128(C->s_hi, C->s_lo);
  const u128 inc = mk128(C->inc_hi, C->inc_lo);
  const int tile = blockIdx.x;
  const int env0 = tile * EPB + threadIdx.x * EPT;
  int32_t a4[4];
  uint32_t ae4[4];
  load4<int32_t>(act, env0, p.B, a4);
  load4<uint32_t>(p.ae, env0, p.B, ae4);
  int g4[4];
  if (p.fixed_goal < 0) {
    uint16_t gg[4];
    load4<uint16_t>(p.goal, env0, p.B, gg);
#pragma unroll
    for (int i = 0; i < 4; ++i) g4[i] = gg[i];
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) g4[i] = p.fixed_goal;
  }
  // random(B): env e draws the u64 at stream position e+1 (action_utils.py:84). Lane state =
  // (jump by 4t) o (jump by tile*EPB + 1) applied to s0, both tables precomputed per seed.
  uint64_t k4[4];
  {
    u128 s = apply_jump(p.lt4[threadIdx.x], apply_jump(p.tja[tile], s0));
    k4[0] = pcg_output(s) >> 11;
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      s = pcg_step(s, inc);
      k4[i] = pcg_output(s) >> 11;
    }
  }
  __syncthreads();  // s_thr
  float r[4];
  uint8_t tm[4], tr[4];
  uint32_t nae[4];
  int ag[4], gl[4];
  uint32_t c = 0, fm = 0;
  float rsum = 0.f;
  uint32_t eps = 0, lens = 0, nst = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const Trans t = transition(p, GTabs{p}, ae4[i], g4[i], a4[i], k4[i], s_thr);
    const bool valid = env0 + i < p.B;
    const bool f = valid && (t.term | t.trunc);
    r[i] = t.rew;
    tm[i] = t.term;
    tr[i] = t.trunc;
    ag[i] = f && p.fixed_agent >= 0 ? p.fixed_agent : t.agent;
    gl[i] = t.goal;
    nae[i] = (uint32_t)ag[i] | ((uint32_t)(f ? 0 : t.elapsed) << 16);
    c += f;
    fm |= (f ? 1u : 0u) << i;
    if (valid) {
      rsum += t.rew;
      nst += 1;
      if (f) { eps += 1; lens += (uint32_t)t.elapsed; }
    }
  }
  store4<float>(rew, env0, p.B, r);
  store4<uint8_t>(term, env0, p.B, tm);
  store4<uint8_t>(trunc, env0, p.B, tr);
  store4<uint32_t>(p.ae, env0, p.B, nae);
  write_obs4<OK>(p, GTabs{p}, env0, ag, gl, obs);
  // compact this tile's resetters (ascending env order) for K2
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_red[wid] = x;
  __syncthreads();
  uint32_t off = x - c, tot = 0;
#pragma unroll
  for (int w = 0; w < TPB / 64; ++w) {
    if (w < wid) off += s_red[w];
    tot += s_red[w];
  }
  if (c) {
    uint16_t* lst = p.tlist + (size_t)tile * EPB;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (fm & (1u << i)) lst[off++] = (uint16_t)(threadIdx.x * EPT + i);
  }
  if (threadIdx.x == 0) p.tcount[tile] = tot;
  add_metrics(p, rsum, eps, lens, nst);
}

// K2 — choice(valid, b) for the b resetting envs in ascending env order (goal call, then agent
// call; msrooms.py:383-388 / rooms.py:191-196), and the next PCG64 state. Block i owns tiles
// [i*T, (i+1)*T): its resetters have ranks [P_i, P_i + n_i), P_i = resets in earlier tiles.
// Fast path: the j-th resetter of a call takes word (call base + j). Every block checks its own
// words for Lemire rejections and publishes a flag; a block whose range or any predecessor's
// range holds a rejection recomputes exact positions by walking the stream (rare: p ~ 1e-8
// per word). The last block publishes the next RNG state (it waited on every other block).
#define RM_RESET 1  // every env resets (reset()); U0 = 0, no random(B) before the words

template <int OK>
__global__ __launch_bounds__(TPB) void grid_resolve_numpy(GridDev p, void* __restrict__ obs, int mode, uint32_t U0) {
  __shared__ ResolveShared sh;
  GridCtl* C = p.ctl;
  Stream st;
  st.s0 = mk128(C->s_hi, C->s_lo);
  st.inc = mk128(C->inc_hi, C->inc_lo);
  st.h0 = C->has_u32;
  st.u0 = C->uinteger;
  st.U0 = U0;
  const uint32_t epoch = C->epoch;
  const bool reset_all = mode & RM_RESET;
  const bool rgoal = p.fixed_goal < 0, ragent = p.fixed_agent < 0;
  const int ncalls = (int)rgoal + (int)ragent;
  const int T = (p.nblk + (int)gridDim.x - 1) / (int)gridDim.x;
  const int t0 = min((int)blockIdx.x * T, p.nblk), t1 = min(t0 + T, p.nblk);
  auto count_of = [&](int k) -> uint32_t {
    return reset_all ? (uint32_t)min(EPB, p.B - k * EPB) : p.tcount[k];
  };
  // prefix of the tile counts before my tiles, and the total
  uint32_t pre = 0, all = 0;
  for (int k = threadIdx.x; k < p.nblk; k += TPB) {
    const uint32_t v = count_of(k);
    all += v;
    if (k < t0) pre += v;
  }
  const uint32_t P = block_sum(pre, sh.red);
  const uint32_t btot = block_sum(all, sh.red2);
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int k = t0; k < t1; ++k) {
      sh.tpre[k - t0] = acc;
      acc += count_of(k);
    }
    sh.tpre[t1 - t0] = acc;
    sh.n = acc;
  }
  __syncthreads();
  const uint32_t n = sh.n;
  // pass A: Lemire rejections among my words (fast-path positions)
  uint32_t rj = 0;
  if (n) {
    const uint32_t m = (n + TPB - 1) / TPB;
    const uint32_t q0 = threadIdx.x * m, q1 = min(q0 + m, n);
    for (int cidx = 0; cidx < ncalls; ++cidx) {
      const bool goal_call = rgoal && cidx == 0;
      const uint32_t nv = goal_call ? (uint32_t)p.n_goal_valid : (uint32_t)p.n_agent_valid;
      const uint32_t th = goal_call ? p.thr_goal : p.thr_agent;
      if (q0 < q1) {
        WordIter it;
        it.init(p, st, (uint32_t)cidx * btot + P + q0);
        for (uint32_t q = q0; q < q1; ++q) rj |= lemire_rejected(it.next(st), nv, th) ? 1u : 0u;
      }
    }
  }
  const uint32_t myrej = __syncthreads_or((int)rj) ? 1u : 0u;
  if (threadIdx.x == 0 && (int)blockIdx.x != p.fault_block)
    st_flag32(&p.rflag[blockIdx.x], ((epoch + 1u) << 1) | myrej);
  // wait for every predecessor block's flag (all K2 blocks are resident: gridDim <= 256)
  uint32_t prej = 0;
  for (int j = threadIdx.x; j < (int)blockIdx.x; j += TPB) {
    uint32_t f = ld_flag(&p.rflag[j]);
    uint32_t spins = 0;
    while ((f >> 1) != epoch + 1u) {
      __builtin_amdgcn_s_sleep(1);
      f = ld_flag(&p.rflag[j]);
      if (spin_give_up(p, spins)) break;
    }
    prej |= f & 1u;
  }
  const bool slow = __syncthreads_or((int)(prej | myrej)) != 0;
  // exact call-2 base when a rejection is anywhere before or in call 1
  uint32_t w1 = btot;
  if (slow && ncalls == 2 && btot) {
    if (threadIdx.x < 64) {
      const uint32_t a = scan_accepted(p.self, st, 0, (uint32_t)p.n_goal_valid, p.thr_goal, btot - 1, btot, nullptr);
      if (threadIdx.x == 0) sh.w1 = a;
    }
    __syncthreads();
    w1 = sh.w1;
  }
  // pass B: resolve my resetters, in batches of EPB ranks
  for (uint32_t b0 = 0; b0 < n; b0 += EPB) {
    const uint32_t bl = min((uint32_t)EPB, n - b0);
    if (slow) {
      if (threadIdx.x < 64) {
        if (rgoal)
          scan_accepted(p.self, st, 0, (uint32_t)p.n_goal_valid, p.thr_goal, P + b0, P + b0 + bl, sh.pos);
        if (ragent)
          scan_accepted(p.self, st, rgoal ? w1 : 0, (uint32_t)p.n_agent_valid, p.thr_agent, P + b0, P + b0 + bl,
                        rgoal ? sh.pos2 : sh.pos);
      }
      __syncthreads();
    }
    for (uint32_t q = b0 + threadIdx.x; q < b0 + bl; q += TPB) {
      int kt = 0;
      while (sh.tpre[kt + 1] <= q) ++kt;  // my tile holding flattened resetter q (T is small)
      const int k = t0 + kt;
      const uint32_t local = q - sh.tpre[kt];
      const int env = k * EPB + (reset_all ? (int)local : (int)p.tlist[(size_t)k * EPB + local]);
      const uint32_t j = P + q;
      int goal = p.fixed_goal, agent = p.fixed_agent;
      if (rgoal) {
        const uint32_t w = slow ? sh.pos[q - b0] : j;
        goal = p.goal_valid[lemire_value(word_at(p, st, w), (uint32_t)p.n_goal_valid)];
      } else if (goal < 0) {
        goal = 0;
      }
      if (ragent) {
        const uint32_t w = slow ? (rgoal ? sh.pos2[q - b0] : sh.pos[q - b0]) : (rgoal ? btot : 0u) + j;
        agent = p.agent_valid[lemire_value(word_at(p, st, w), (uint32_t)p.n_agent_valid)];
      }
      if (rgoal) p.goal[env] = (uint16_t)goal;
      p.ae[env] = (uint32_t)agent;  // elapsed = 0
      write_obs<OK>(p, GTabs{p}, env, agent, goal, obs);
    }
    __syncthreads();
  }
  // the last block has seen every flag: publish the next RNG state
  if (blockIdx.x == gridDim.x - 1) {
    uint32_t wtot = 0;
    if (btot && ncalls) {
      if (!slow) {
        wtot = (uint32_t)ncalls * btot;
      } else {
        if (threadIdx.x < 64) {
          uint32_t a = ncalls == 2 ? w1 : 0u;
          const bool last_goal = ncalls == 1 && rgoal;
          a = scan_accepted(p.self, st, a, last_goal ? (uint32_t)p.n_goal_valid : (uint32_t)p.n_agent_valid,
                            last_goal ? p.thr_goal : p.thr_agent, btot - 1, btot, nullptr);
          if (threadIdx.x == 0) sh.bcast = a;
        }
        __syncthreads();
        wtot = sh.bcast;
      }
    }
    if (threadIdx.x == 0) {
      uint32_t used, h, u = st.u0;
      if (wtot == 0) {
        used = 0; h = st.h0;
      } else if (st.h0) {
        used = wtot >> 1;          // ceil((wtot-1)/2)
        h = (wtot - 1) & 1;
      } else {
        used = (wtot + 1) >> 1;    // ceil(wtot/2)
        h = wtot & 1;
      }
      const u128 s = pcg_jump(p.jt, st.s0, st.U0 + used);
      // numpy keeps the last buffered half in `uinteger` even after it has been consumed
      if (used) u = (uint32_t)(pcg_output(s) >> 32);
      C->s_hi = hi64(s);
      C->s_lo = lo64(s);
      C->has_u32 = h;
      C->uinteger = u;
      C->b_total = btot;
      C->epoch = epoch + 1u;
    }
  }
}

// reset(): elapsed = 0 and the fixed parts (msrooms.py:376-381 / rooms.py:184-189).
__global__ __launch_bounds__(TPB) void grid_reset_init(GridDev p) {
  const int env = blockIdx.x * TPB + threadIdx.x;
  if (env >= p.B) return;
  p.ae[env] = p.fixed_agent >= 0 ? (uint32_t)p.fixed_agent : 0u;
  if (p.fixed_goal < 0) p.goal[env] = 0;
}

// ------------------------------------------------------------------ kernel: fused numpy rollout ----
// K numpy-exact steps in ONE persistent launch, one block per CU (G <= 256). Block b owns the 2048-env
// tiles tau = q*G + b (q < QPT); env state lives in registers for the whole launch and the lookup tables
// in LDS. Waves: 8 env waves (4 envs per thread per tile), 1 control wave, 2 store waves. Per step
// (s0 = PCG64 state at the step start):
//   1. env waves: every env e draws u64 #e of random(B) from its lane state S_e = jump(s0, e+1) and
//      transitions (critical path); per-wave reset counts by ballot bit-planes -> LDS -> barrier B1.
//   2. control wave: publishes ONE tagged 8-B granule per block {tag, Lemire-rejection bit, 12-bit
//      reset count per tile} (the rejection bit covers a speculative window of RCOV choice() words per
//      tile, checked before B1), all-gathers the G granules (4 per lane, the only inter-block exchange;
//      xmode 0: block 0 aggregates and publishes per-tile words instead), scans them (DPP) into this
//      block's tile prefixes, the total b and the rejection flag, and in the common case draws the
//      resetters' cells and the next state s0' = J_used(J_B(s0)) with one jump chain per lane.
//      Meanwhile (STG) the env waves list their resetters and write the step's outputs into the LDS
//      staging area (no global stores during the exchange); without STG they store directly.
//   3. barrier B2; env waves take their resetters' cells (slow cases: extra check rounds extend the
//      rejection coverage for mass resets or a second reset call; a rejection anywhere switches to the
//      exact stream walk, p ~ 1e-8/word) and advance every lane state by J_used.
//   4. store waves (STG): copy the staged outputs to HBM while the env waves advance and run the next
//      step's VALU-bound transitions.
// Granule tags = ((global step + 1) * 4 + round) mod 2^15; slots alternate by step parity (a
// block publishes step t+2 only after every block has published step t+1, i.e. finished
// reading step t's slots), so a stale granule never carries the expected tag.
constexpr int FENVW = 8;                 // env waves per block (2 per SIMD)
constexpr int FSTW = 2;                  // store waves (LDS-staged outputs -> HBM)
constexpr int FWAVES = FENVW + 1 + FSTW; // + one control wave + the store waves
constexpr int FTPB = FWAVES * 64;
constexpr int FEPB = FENVW * 64 * EPT;   // 2048 envs per fused tile
constexpr int RCOV = 62;                 // speculative rejection-check words per tile per step (32 u64 lanes)
constexpr int FMAXG = 256;        // blocks: wave 0 gathers 4 granules per lane
constexpr int FMAXQ = 4;          // tiles per block (12-bit counts: 4 per granule)
constexpr int FMAXT = FMAXG * FMAXQ;
constexpr int LDS_TABLE_BUDGET = 96 * 1024;
// Output staging (scalar obs kinds, <= 2 tiles per block): per tile obs int32[FEPB], reward f32[FEPB],
// terminated u8[FEPB], truncated u8[FEPB], in dynamic LDS after the tables.
constexpr int STG_TILE_BYTES = FEPB * 10;
// Speculative word windows of the staged fused kernel. A step's resetter words sit at stream positions that are
// only known once the all-gather has delivered the tile prefixes; but the words themselves depend only on the
// post-random(B) state SB, known at the step's start. So while the exchange is in flight the (otherwise idle) store
// waves evaluate, per tile, the u64 outputs of a window of SPW_NJ draws centred on the tile's predicted position
// (the previous step's reset total b spread over the tiles in proportion), and SPW_NU candidates for the next
// step's state J_used(SB) and J_used's coefficients centred on the predicted used = b / 2. After the gather the
// control wave reads its resetters' words and J_used from LDS instead of evaluating two dependent radix-256 jumps
// per lane; lanes whose position falls outside a window (or a window not ready) take the jump path as before.
constexpr int SPW_NJ = 384;  // u64 draws per tile window (768 words: +-4 sigma of the prefix prediction at 1M envs)
constexpr int SPW_NU = 256;  // next-state candidates (+-128 u64 draws around the predicted J_used)
constexpr int SPW_CAND_U64 = 6;  // a_hi, a_lo, c_hi, c_lo, s_hi, s_lo
__host__ __device__ constexpr int spw_bytes(int qpt) { return (qpt * SPW_NJ + SPW_NU * SPW_CAND_U64) * 8; }
constexpr int R_ENV = 0, R_CTRL = 1, R_PASS = 2;  // fused_resets roles: env wave, control wave, store wave
template <int OK, int QPT>
constexpr bool fused_staged() { return QPT <= 2 && (OK == GP_OBS_HANSEN || OK == GP_OBS_TABLE); }
constexpr uint32_t TAG_MASK = 0x7FFFu;
// Tuning switches of the fused kernel (A/B builds: tools/build_variant.sh):
//  GP_TRIMS 1: VALU trims of the transitions (thresholds pre-shifted so the full 64-bit draw is compared,
//    actions turned into threshold-row offsets while waiting at B2).
//  GP_ALIGNBIT 1: the draw's 64-bit rotate as two v_alignbit_b32.
//  GP_ACC 1: the episode statistics from the step's masks (popcounts) and, for the episode lengths, from
//    the elapsed counters at the launch's start and end, instead of per-env accumulations.
#ifndef GP_TRIMS
#define GP_TRIMS 1
#endif
#ifndef GP_ACC
#define GP_ACC 1
#endif
//  GP_VPIN 1: the stream increment and the goal-direction offsets pinned to VGPRs (SGPR pressure).
//  GP_ILV 1: the transitions loop runs env-slot-major (the tiles' independent draw chains interleave).
//  GP_CELLENV 1 (staged kernel): resetter cells stored by env slot, taken with one 16-B LDS load per tile.
#ifndef GP_ILV
#define GP_ILV 1
#endif
#ifndef GP_CELLENV
#define GP_CELLENV 1
#endif
//  GP_STORE_PRIO: scheduling priority of the store waves (1: above the env waves).
#ifndef GP_STORE_PRIO
#define GP_STORE_PRIO 1
#endif
#ifndef GP_VPIN
#define GP_VPIN 1
#endif
#ifndef GP_ALIGNBIT
#define GP_ALIGNBIT 0
#endif
//  GP_PRO2 1: the launch prologue pays ONE global-load latency: the env waves issue their state / action /
//    tile-jump loads first and copy only the small lookup tables (everything before the PCG jump tables,
//    ~3.5 KB for FourRooms) into LDS before the block barrier; the store waves, idle until the first step's
//    B1, copy the jump tables (26 KB) behind it, and the control wave sets up from the global copies.
#ifndef GP_PRO2
#define GP_PRO2 1
#endif

struct FusedShared {
  uint32_t wcnt[FMAXQ][FENVW];   // per-env-wave reset counts of each tile
  uint32_t wrej;                 // speculative-check rejection (control wave)
  uint32_t tpre[FMAXQ];          // global exclusive prefix of this block's tiles
  uint32_t btot, anyrej, known, flag, w1;
  uint64_t ju[4];                // this step's J_used (a_hi, a_lo, c_hi, c_lo)
  uint64_t jB[4];                // J_B: jump by num_envs
  uint64_t ns_hi, ns_lo;         // next step's s0
  uint32_t nh, nu;               // next step's has_uint32 / uinteger
  uint32_t drawn;                // the control wave drew this step's resetter cells before B2
  uint32_t rdone;                // env waves done listing their resetters in renv (monotone)
  int32_t dof[8];                // goal-direction cell offsets (Hansen goal multiplier)
  uint64_t spw_sb[2];            // SPW: this step's post-random(B) state (control wave, before B1)
  uint32_t spw_h0, spw_b;        // SPW: has_uint32 at the step start, the previous step's reset words
  uint32_t spw_done;             // SPW: store waves done with their windows (monotone, FSTW per step)
  uint32_t spw_n0[FMAXQ];        // SPW: first draw number of each tile's window (0: no window)
  uint32_t spw_u0;               // SPW: first candidate's used
  uint16_t renv[2][FEPB];        // STG: env (in tile) of resetter rank r of tile q
  uint32_t pos[FEPB];            // slow path: accepted-word positions of one tile's resetters
  uint32_t pos2[FEPB];
  alignas(16) uint32_t cell[FMAXQ * FEPB];  // resetter cells (goal | agent << 16) by tile and rank (or env slot)
};

__device__ __forceinline__ uint64_t bgran(uint32_t tag, uint32_t rej, uint64_t counts) {
  return ((uint64_t)(tag & TAG_MASK) << 49) | ((uint64_t)(rej & 1u) << 48) | counts;
}
__device__ __forceinline__ uint32_t gcount(uint64_t g, int q) { return (uint32_t)(g >> (12 * q)) & 0xFFFu; }
// Per-tile word published by the aggregator: {tag, rejection bit, b (24 bits), tile prefix (24 bits)}.
__device__ __forceinline__ uint64_t tword(uint32_t tag, uint32_t rej, uint32_t b, uint32_t pre) {
  return ((uint64_t)(tag & TAG_MASK) << 49) | ((uint64_t)(rej & 1u) << 48) | ((uint64_t)(b & 0xFFFFFFu) << 24) |
         (uint64_t)(pre & 0xFFFFFFu);
}

// Wave-64 inclusive prefix sum (DPP row shifts + row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); // row_bcast:31
  return x;
}

// Exclusive wave prefix and wave total of a per-lane count in [0, 7] (three ballot bit-planes).
__device__ __forceinline__ void wave_count_prefix(uint32_t c, uint32_t& excl, uint32_t& tot) {
  const uint64_t b0 = __ballot(c & 1u), b1 = __ballot(c & 2u), b2 = __ballot(c & 4u);
  const uint32_t lt0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b0, 0u));
  const uint32_t lt1 = __builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b1, 0u));
  const uint32_t lt2 = __builtin_amdgcn_mbcnt_hi((uint32_t)(b2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b2, 0u));
  excl = lt0 + 2u * lt1 + 4u * lt2;
  tot = (uint32_t)__builtin_popcountll(b0) + 2u * (uint32_t)__builtin_popcountll(b1) +
        4u * (uint32_t)__builtin_popcountll(b2);
}

// Orders a wave's own LDS writes before its later LDS reads by other lanes (no block barrier).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}


// Wave 0: poll the G block granules of one round (lane l holds blocks 4l..4l+3) until every one
// carries `tag`. Granules of blocks >= G read as 0. `full`: the coverage rounds' granules carry the whole 32-bit
// tag in their (otherwise unused) count bits too, so that a round-1/2 slot last written 8192 steps earlier
// (same 15-bit tag, same parity) is never taken for this step's.
__device__ __forceinline__ void gather_blocks(const GridDev& p, const uint64_t* slots, int G, uint32_t tag,
                                              uint64_t (&g)[4], bool full = false) {
  const int lane = threadIdx.x & 63;
  const uint64_t want = (uint64_t)(tag & TAG_MASK);
  uint32_t pend = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    g[j] = 0;
    if (lane * 4 + j < G) pend |= 1u << j;
  }
  uint32_t spins = 0;
  while (true) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (pend & (1u << j))
        g[j] = __hip_atomic_load(&slots[lane * 4 + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((pend & (1u << j)) && (g[j] >> 49) == want && (!full || (uint32_t)g[j] == tag)) pend &= ~(1u << j);
    if (!__any((int)pend)) break;
    if (spin_give_up(p, spins)) {  // flagged: the results of this launch are invalid (GP_E_DEVICE)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (pend & (1u << j)) g[j] = want << 49;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Lemire check of `cnt` consecutive words from `w0` (one thread).
__device__ __noinline__ uint32_t check_words(const GridDev* __restrict__ gp, const Stream st, uint32_t w0, uint32_t cnt,
                                                uint32_t n, uint32_t thr) {
  const GridDev& p = *gp;
  if (!cnt) return 0;
  WordIter it;
  it.init(p, st, w0);
  uint32_t r = 0;
  for (uint32_t i = 0; i < cnt; ++i) r |= lemire_rejected(it.next(st), n, thr) ? 1u : 0u;
  return r;
}

// An extra coverage round: tile tau checks words [base + tau*R, base + (tau+1)*R) (R =
// ceil(total / nt)) with wave q checking tile q of the block; returns whether any word in
// [base, base + total) is rejected (grid-wide, via one more granule exchange).
__device__ __noinline__ uint32_t coverage_round(const GridDev* __restrict__ gp, const Stream st, uint64_t* slots, int nt, int G, int QPT,
                                   uint32_t tag, uint32_t base, uint32_t total, uint32_t n, uint32_t thr,
                                   FusedShared& sh) {
  const GridDev& p = *gp;
  const uint32_t R = (total + nt - 1) / nt;
  const uint32_t per = (R + 63) / 64;  // words per checking lane (64 lanes per tile)
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t r = 0;
  if (wid < QPT) {
    const int tau = wid * G + (int)blockIdx.x;
    if (tau < nt) {
      const uint32_t lo = tau * R + lane * per, hi = min(min(lo + per, (uint32_t)(tau + 1) * R), total);
      if (lo < hi) r = check_words(gp, st, base + lo, hi - lo, n, thr);
    }
  }
  const uint32_t any = __syncthreads_or((int)r) ? 1u : 0u;
  if (threadIdx.x == 0 && (int)blockIdx.x != p.fault_block)
    __hip_atomic_store(&slots[blockIdx.x], bgran(tag, any, (uint64_t)tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (wid == FENVW) {  // the control wave
    uint64_t g[4];
    gather_blocks(p, slots, G, tag, g, true);
    uint32_t rj = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) rj |= (uint32_t)(g[j] >> 48) & 1u;
    const bool a = __any((int)rj);
    if (lane == 0) sh.flag = a ? 1u : 0u;
  }
  __syncthreads();
  return sh.flag;
}

__device__ __forceinline__ PcgJump compose_jump(const PcgJump& j2, const PcgJump& j1) {  // j2 o j1
  const u128 a = mk128(j2.a_hi, j2.a_lo) * mk128(j1.a_hi, j1.a_lo);
  const u128 c = mk128(j2.a_hi, j2.a_lo) * mk128(j1.c_hi, j1.c_lo) + mk128(j2.c_hi, j2.c_lo);
  return PcgJump{hi64(a), lo64(a), hi64(c), lo64(c)};
}

// Jump parameters for n steps from the radix tables (composition of <= JT_LEVELS entries).
__device__ __forceinline__ PcgJump jump_params(const PcgJump* jt, uint32_t n) {
  PcgJump j{0, 1, 0, 0};
  bool first = true;
#pragma unroll
  for (int L = 0; L < JT_LEVELS; ++L) {
    const uint32_t d = (n >> (JT_RADIX_BITS * L)) & (JT_RADIX - 1);
    if (d) {
      j = first ? jt[L * JT_RADIX + d] : compose_jump(jt[L * JT_RADIX + d], j);
      first = false;
    }
  }
  return j;
}

// Jump by n steps: two radix-256 entries (both loads issued up front) for n < 2^16, else the
// radix-64 tables.
__device__ __forceinline__ u128 jump_small(const PcgJump* t8, const PcgJump* t64, u128 s, uint32_t n) {
  if (n < 65536u) {
    const PcgJump j0 = t8[n & 255u], j1 = t8[256u + (n >> 8)];
    return apply_jump(j1, apply_jump(j0, s));
  }
  return pcg_jump(t64, s, n);
}
__device__ __forceinline__ PcgJump jparams_small(const PcgJump* t8, const PcgJump* t64, uint32_t n) {
  if (n < 65536u) return compose_jump(t8[256u + (n >> 8)], t8[n & 255u]);
  return jump_params(t64, n);
}

// The choice() draws of one resetter: Lemire values of word wg (goal call, mode bit 0, n = ng)
// and word wa (agent call, mode bit 1, n = na) -> goal index | agent index << 16. Out of line:
// it is the only place the fused kernel needs a full jump from s0 per lane.
__device__ __forceinline__ uint32_t draw_cells(const PcgJump* jt8, const PcgJump* jt, u128 SB, uint32_t h0,
                                            uint32_t u0, uint32_t wg, uint32_t wa, uint32_t mode, uint32_t ng,
                                            uint32_t na) {
  auto word = [&](uint32_t w) -> uint32_t {
    if (h0 && w == 0) return u0;
    const uint32_t ww = w - h0;
    const uint64_t x = pcg_output(jump_small(jt8, jt, SB, (ww >> 1) + 1));
    return (ww & 1) ? (uint32_t)(x >> 32) : (uint32_t)x;
  };
  uint32_t v = 0;
  if (mode & 1u) v |= lemire_value(word(wg), ng);
  if (mode & 2u) v |= lemire_value(word(wa), na) << 16;
  return v;
}

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

// Publish (to LDS) the next step's state: s0' = J_used(SB), buffered half. One lane writes.
__device__ __forceinline__ void publish_next(const LTabs& tb, FusedShared& sh, const u128 SB, uint32_t wtot,
                                            uint32_t h0, uint32_t u0, bool writer) {
  uint32_t used, h;
  words_to_draws(wtot, h0, used, h);
  const PcgJump ju = jparams_small(tb.jt8(), tb.jt(), used);
  const u128 s = jump_small(tb.jt8(), tb.jt(), SB, used);
  // numpy keeps the last buffered half in `uinteger` even after it has been consumed
  const uint32_t u = used ? (uint32_t)(pcg_output(s) >> 32) : u0;
  if (writer) {
    sh.ju[0] = ju.a_hi; sh.ju[1] = ju.a_lo; sh.ju[2] = ju.c_hi; sh.ju[3] = ju.c_lo;
    sh.ns_hi = hi64(s); sh.ns_lo = lo64(s);
    sh.nh = h; sh.nu = u;
  }
}

#ifdef GP_STAMPS
#define STAMP(i)                                                                                  \
  do {                                                                                            \
    if (threadIdx.x == 0 && k < 64) {                                                             \
      unsigned long long t_;                                                                      \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
      p_in.dbg[((size_t)blockIdx.x * 64 + k) * 16 + (i)] = t_;                                    \
    }                                                                                             \
  } while (0)
// wall-clock (100 MHz, chip-synchronous) stamp by the calling lane
#define RSTAMP(i)                                                                                 \
  do {                                                                                            \
    if (k < 64) {                                                                                 \
      unsigned long long t_;                                                                      \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
      p_in.dbg[((size_t)blockIdx.x * 64 + k) * 16 + (i)] = t_;                                    \
    }                                                                                             \
  } while (0)
// launch-level stamps (block, slot): 0 entry, 1 tables staged, 2 step loop done, 3 kernel end
#define LSTAMP(i)                                                                                 \
  do {                                                                                            \
    if (threadIdx.x == 0) {                                                                       \
      unsigned long long t_;                                                                      \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
      p_in.dbg[(size_t)256 * 64 * 16 + (size_t)blockIdx.x * 8 + (i)] = t_;                        \
    }                                                                                             \
  } while (0)
#else
#define LSTAMP(i) \
  do {            \
  } while (0)
#define RSTAMP(i) \
  do {            \
  } while (0)
#define STAMP(i) \
  do {           \
  } while (0)
#endif

// Workgroup barrier that orders LDS only: __syncthreads() also drains every outstanding global
// store of the wave (s_waitcnt vmcnt(0)), which would put the obs/reward store latency on the
// fused kernel's per-step critical path. All fused-kernel barriers below guard LDS (sh.*) only.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Stage the first `bytes` (a multiple of 16) of the LDS table image: every thread issues all of its
// 16-B loads before its first LDS store, so the block pays ONE global-load latency for all the
// tables (one copy loop per table paid one each: ≈4-5 µs of launch prologue).
__device__ __forceinline__ void lds_image_copy(char* dyn, const char* src, int bytes) {
  const int n = bytes >> 4, bd = (int)blockDim.x;
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(dyn);
  // rounds of up to 8 chunks per thread; named registers (an array here was placed in scratch)
  for (int i0 = (int)threadIdx.x; i0 < n; i0 += 8 * bd) {
    uint4 v0, v1, v2, v3, v4, v5, v6, v7;
    const bool a1 = i0 + bd < n, a2 = i0 + 2 * bd < n, a3 = i0 + 3 * bd < n, a4 = i0 + 4 * bd < n,
               a5 = i0 + 5 * bd < n, a6 = i0 + 6 * bd < n, a7 = i0 + 7 * bd < n;
    v0 = s[i0];
    if (a1) v1 = s[i0 + bd];
    if (a2) v2 = s[i0 + 2 * bd];
    if (a3) v3 = s[i0 + 3 * bd];
    if (a4) v4 = s[i0 + 4 * bd];
    if (a5) v5 = s[i0 + 5 * bd];
    if (a6) v6 = s[i0 + 6 * bd];
    if (a7) v7 = s[i0 + 7 * bd];
    d[i0] = v0;
    if (a1) d[i0 + bd] = v1;
    if (a2) d[i0 + 2 * bd] = v2;
    if (a3) d[i0 + 3 * bd] = v3;
    if (a4) d[i0 + 4 * bd] = v4;
    if (a5) d[i0 + 5 * bd] = v5;
    if (a6) d[i0 + 6 * bd] = v6;
    if (a7) d[i0 + 7 * bd] = v7;
  }
}

// Copy image bytes [b0, b1) (multiples of 16) to the same LDS offsets with threads t0 .. t0 + nt - 1, every
// thread's 16-B loads in flight before its first LDS store.
__device__ __forceinline__ void lds_image_copy_range(char* dyn, const char* src, int b0, int b1, int t, int nthr) {
  const int c0 = b0 >> 4, n = (b1 - b0) >> 4;
  const uint4* s = reinterpret_cast<const uint4*>(src) + c0;
  uint4* d = reinterpret_cast<uint4*>(dyn) + c0;
  for (int i0 = t; i0 < n; i0 += 8 * nthr) {
    uint4 v0, v1, v2, v3, v4, v5, v6, v7;
    const bool a1 = i0 + nthr < n, a2 = i0 + 2 * nthr < n, a3 = i0 + 3 * nthr < n, a4 = i0 + 4 * nthr < n,
               a5 = i0 + 5 * nthr < n, a6 = i0 + 6 * nthr < n, a7 = i0 + 7 * nthr < n;
    v0 = s[i0];
    if (a1) v1 = s[i0 + nthr];
    if (a2) v2 = s[i0 + 2 * nthr];
    if (a3) v3 = s[i0 + 3 * nthr];
    if (a4) v4 = s[i0 + 4 * nthr];
    if (a5) v5 = s[i0 + 5 * nthr];
    if (a6) v6 = s[i0 + 6 * nthr];
    if (a7) v7 = s[i0 + 7 * nthr];
    d[i0] = v0;
    if (a1) d[i0 + nthr] = v1;
    if (a2) d[i0 + 2 * nthr] = v2;
    if (a3) d[i0 + 3 * nthr] = v3;
    if (a4) d[i0 + 4 * nthr] = v4;
    if (a5) d[i0 + 5 * nthr] = v5;
    if (a6) d[i0 + 6 * nthr] = v6;
    if (a7) d[i0 + 7 * nthr] = v7;
  }
}

// Phase 4 of a fused step (both roles; every barrier here is block-uniform): the resetters'
// choice() draws. ROLE: R_CTRL = the control wave (coverage exchanges, stream walks, J_used of the
// unusual cases); R_ENV = an env wave with its env state; R_PASS = a store wave (barriers only).
// Control wave: the cells (goal | agent << 16) of this block's resetters, rank r of tile q ->
// sh.cell[q*FEPB + r]. Word positions: fast path P_q + r (goal call) and w1 + P_q + r (agent
// call); slow path (only_q >= 0: one tile) from the stream walk's position lists pg / pa.
// Control wave, common case (one reset call, no rejected word, b within the speculative window):
// the next PCG64 state and the block's resetter cells in ONE straight-line block so that their
// dependent jump chains overlap. tq / pre: lane q < QPT holds tile q's reset count / prefix.
// STG: the final obs of resetter rank r of tile q (new cells goal | agent << 16) into the staging area.
template <int OK, bool STG>
__device__ __forceinline__ void stage_reset_obs(const GridDev& p, const FusedShared& sh, const LTabs& tb, char* stg,
                                                int q, uint32_t r, uint32_t cell) {
  if constexpr (STG) {
    int dof[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) dof[d] = (OK == GP_OBS_HANSEN && d < p.obs_dirs) ? sh.dof[d] : 0x7FFFFFFF;
    reinterpret_cast<int32_t*>(stg + q * STG_TILE_BYTES)[sh.renv[q][r]] =
        obs_value_r<OK>(p, tb, (int)(cell >> 16), (int)(cell & 0xFFFFu), dof);
  }
}
// The same with the slot (renv) and the direction offsets already in registers.
template <int OK, bool STG>
__device__ __forceinline__ void stage_reset_obs_r(const GridDev& p, const LTabs& tb, char* stg, int q, int slot,
                                                  uint32_t cell, const int (&dof)[8]) {
  if constexpr (STG)
    reinterpret_cast<int32_t*>(stg + q * STG_TILE_BYTES)[slot] =
        obs_value_r<OK>(p, tb, (int)(cell >> 16), (int)(cell & 0xFFFFu), dof);
}

template <int OK, int QPT, bool STG>
__device__ __forceinline__ uint32_t ctrl_fast_finish(const GridDev& p, FusedShared& sh, const LTabs& tb, const u128 SB,
                                                 const Stream& st, uint32_t b, uint32_t tq, uint32_t pre, char* stg,
                                                 const int (&dof)[8], const uint64_t* spw = nullptr, int kstamp = 64) {
  const int lane = threadIdx.x & 63;
  // SPW (spw != nullptr: the store waves' windows for this step are complete): the windows' bases
  uint32_t sn0[QPT], su0 = 0xFFFFFFFFu;
  if (spw) {
#pragma unroll
    for (int q = 0; q < QPT; ++q) sn0[q] = sh.spw_n0[q];
    su0 = sh.spw_u0;
  }
  const bool rgoal = p.fixed_goal < 0;
  const uint32_t nsel = rgoal ? (uint32_t)p.n_goal_valid : (uint32_t)p.n_agent_valid;
  uint32_t tc[QPT], P[QPT], cum[QPT + 1];
  cum[0] = 0;
#pragma unroll
  for (int q = 0; q < QPT; ++q) {
    tc[q] = (uint32_t)__builtin_amdgcn_readlane((int)tq, q);
    P[q] = (uint32_t)__builtin_amdgcn_readlane((int)pre, q);
    cum[q + 1] = cum[q] + tc[q];
  }
  uint32_t used, h;
  words_to_draws(b, st.h0, used, h);
  // Every lane evaluates ONE two-level jump X = J2(J1(X0)) from the radix-256 tables (all jumps here
  // are < 2^16: b <= nt * RCOV). Cell lanes: SB jumped to their choice() word. In the first pass
  // lanes 61..63 produce the next step's state instead: J_used = J_hi o J_lo as its multiplier
  // a_hi * a_lo (lane 61) and increment a_hi * c_lo + c_hi (lane 62), and s0' = J_used(SB) (lane 63),
  // so that the whole wave pays for one jump chain instead of four.
  constexpr uint32_t XL = 61;
  uint32_t jumped = 0;  // some lane took the jump path (diagnostics)
  const uint32_t ncell = cum[QPT];
  const uint32_t npass = ncell <= XL ? 1u : 1u + (ncell - XL + 63u) / 64u;
  const PcgJump* t8 = tb.jt8();
  for (uint32_t it = 0; it < npass; ++it) {  // wave-uniform
    const uint32_t idx = it == 0 ? (uint32_t)lane : XL + (it - 1u) * 64u + (uint32_t)lane;
    const bool extra = it == 0 && (uint32_t)lane >= XL;
    const bool cellj = !extra && idx < ncell;
    int q = 0;
#pragma unroll
    for (int j = 1; j < QPT; ++j) q += idx >= cum[j] ? 1 : 0;
    const uint32_t r = idx - cum[q];
    const uint32_t w = P[q] + r;
    const bool buffered = st.h0 && w == 0;  // numpy's buffered half-word
    const uint32_t ww = w - st.h0;
    const uint32_t n = extra ? used : (cellj && !buffered ? (ww >> 1) + 1u : 0u);
    // the env slot of this resetter (STG), loaded alongside the jump tables, off the dependent chain
    const int slot = STG ? (int)sh.renv[q][min(r, (uint32_t)FEPB - 1u)] : 0;
    u128 X = 0;
    uint64_t x = 0;
    bool have = false, xout = false;  // X (and x) from a window: no jump
    if (spw) {
      if (extra) {
        const uint32_t d = used - su0;
        if (su0 != 0xFFFFFFFFu && d < (uint32_t)SPW_NU) {  // (0xFFFFFFFF: the store waves built no candidates)
          const uint64_t* c = spw + QPT * SPW_NJ + (size_t)d * SPW_CAND_U64 + (lane == 61 ? 0 : (lane == 62 ? 2 : 4));
          X = mk128(c[0], c[1]);
          have = true;
        }
      } else if (!cellj || buffered) {
        have = xout = true;  // nothing to jump
      } else {
        const uint32_t d = n - sn0[q];
        if (sn0[q] && d < (uint32_t)SPW_NJ) {
          x = spw[q * SPW_NJ + d];
          have = xout = true;
        }
      }
    }
    if (!have) {  // a lane outside the windows (or no windows): the two dependent radix-256 jumps
      const PcgJump jlo = t8[n & 255u], jhi = t8[256u + ((n >> 8) & 255u)];
      PcgJump J1 = jlo, J2 = jhi;
      u128 X0 = SB;
      if (extra && lane == 61) {
        J1 = PcgJump{0, 1, 0, 0};
        J2.c_hi = 0; J2.c_lo = 0;
        X0 = mk128(jlo.a_hi, jlo.a_lo);
      } else if (extra && lane == 62) {
        J1 = PcgJump{0, 1, 0, 0};
        X0 = mk128(jlo.c_hi, jlo.c_lo);
      }
      X = apply_jump(J2, apply_jump(J1, X0));
      jumped = 1u;
    }
    if (!xout) x = pcg_output(X);
#ifdef GP_STAMPS
    if (it == 0 && kstamp < 64) {  // stamps slot 15: the first pass's jumps are done (diagnostic build only)
      unsigned long long t_;
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_) : "v"(x) : "memory");
      if (lane == 0) p.dbg[((size_t)blockIdx.x * 64 + kstamp) * 16 + 15] = t_;
    }
#endif
    if (cellj) {
      const uint32_t word = buffered ? st.u0 : ((ww & 1u) ? (uint32_t)(x >> 32) : (uint32_t)x);
      const uint32_t v = lemire_value(word, nsel);
      if (OK == GP_OBS_HANSEN && STG && !rgoal && tb.has_avo()) {  // uniform: agent and its obs in one load
        const uint2 e = tb.avo((int)v);
        sh.cell[q * FEPB + (GP_CELLENV ? (uint32_t)slot : r)] = (uint32_t)p.fixed_goal | (e.x << 16);
        reinterpret_cast<int32_t*>(stg + q * STG_TILE_BYTES)[slot] = (int32_t)e.y;
      } else {
        const uint32_t goal = rgoal ? (uint32_t)tb.gv((int)v) : (uint32_t)p.fixed_goal;
        const uint32_t agent = rgoal ? (uint32_t)p.fixed_agent : (uint32_t)tb.av((int)v);
        sh.cell[q * FEPB + ((STG && GP_CELLENV) ? (uint32_t)slot : r)] = goal | (agent << 16);
        stage_reset_obs_r<OK, STG>(p, tb, stg, q, slot, goal | (agent << 16), dof);
      }
    } else if (extra) {
      if (lane == 61) { sh.ju[0] = hi64(X); sh.ju[1] = lo64(X); }
      if (lane == 62) { sh.ju[2] = hi64(X); sh.ju[3] = lo64(X); }
      if (lane == 63) {
        sh.ns_hi = hi64(X); sh.ns_lo = lo64(X);
        sh.nh = h;
        sh.nu = used ? (uint32_t)(x >> 32) : st.u0;
      }
    }
  }
  return __any((int)jumped) ? 1u : 0u;
}

template <int OK, int QPT, bool STG>
__device__ __forceinline__ void ctrl_draw_cells(const GridDev& p, FusedShared& sh, const LTabs& tb, const u128 SB,
                                                const Stream& st, uint32_t w1, const uint32_t* pg, const uint32_t* pa,
                                                int only_q, char* stg) {
  const int lane = threadIdx.x & 63;
  const bool rgoal = p.fixed_goal < 0, ragent = p.fixed_agent < 0;
  const uint32_t mode = (rgoal ? 1u : 0u) | (ragent ? 2u : 0u);
  const uint32_t ng = (uint32_t)p.n_goal_valid, na = (uint32_t)p.n_agent_valid;
  uint32_t tc[QPT], cum[QPT + 1];
  cum[0] = 0;
#pragma unroll
  for (int q = 0; q < QPT; ++q) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < FENVW; ++w) t += sh.wcnt[q][w];
    const int tau = q * (int)gridDim.x + (int)blockIdx.x;
    tc[q] = (tau < p.fnt && (only_q < 0 || only_q == q)) ? t : 0u;
    cum[q + 1] = cum[q] + tc[q];
  }
  for (uint32_t idx = lane; idx < cum[QPT]; idx += 64) {
    int q = 0;
#pragma unroll
    for (int j = 1; j < QPT; ++j) q += idx >= cum[j] ? 1 : 0;
    const uint32_t r = idx - cum[q];
    uint32_t wg, wa;
    if (pg) {
      wg = pg[r];
      wa = pa[r];
    } else {
      wg = sh.tpre[q] + r;
      wa = (rgoal ? w1 : 0u) + wg;
    }
    const uint32_t v = draw_cells(tb.jt8(), tb.jt(), SB, st.h0, st.u0, wg, wa, mode, ng, na);
    const uint32_t goal = rgoal ? (uint32_t)tb.gv((int)(v & 0xFFFFu)) : (uint32_t)p.fixed_goal;
    const uint32_t agent = ragent ? (uint32_t)tb.av((int)(v >> 16)) : (uint32_t)p.fixed_agent;
    sh.cell[q * FEPB + ((STG && GP_CELLENV) ? (uint32_t)sh.renv[q][r] : r)] = goal | (agent << 16);
    stage_reset_obs<OK, STG>(p, sh, tb, stg, q, r, goal | (agent << 16));
  }
}


template <int OK, int QPT, int ROLE, bool STG = false>
__device__ __forceinline__ void fused_resets(const GridDev& p, FusedShared& sh, const LTabs& tb, const Stream& st,
                                             const u128 SB, const PcgJump& jB, uint64_t* slots, uint32_t tag0,
                                             uint32_t (&ae)[QPT][4], int (&gl)[QPT][4], const uint32_t (&fm)[QPT],
                                             const uint32_t (&excl)[QPT], uint32_t (&pc)[QPT][4],
                                             uint32_t (&pfm)[QPT], char* stg = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int G = (int)gridDim.x, nt = p.fnt;
  const bool rgoal = p.fixed_goal < 0, ragent = p.fixed_agent < 0;
  const int ncalls = (int)rgoal + (int)ragent;
  const uint32_t n1 = rgoal ? (uint32_t)p.n_goal_valid : (uint32_t)p.n_agent_valid;
  const uint32_t thr1 = rgoal ? p.thr_goal : p.thr_agent;
  const uint32_t b = sh.btot;
  if (!(ncalls && b)) return;
  // env waves: take the resetters' cells the control wave drew for tile q
  auto consume = [&](int q) {
    if constexpr (ROLE == R_ENV) {
      // the resetters' new cells (independent LDS loads); their obs are written in the next step's
      // output phase, off the critical path (pc / pfm)
      // (STG: the control wave wrote their final obs into the LDS staging area when it drew them)
      uint32_t c[4];
      if constexpr (STG && GP_CELLENV) {  // by env slot: this thread's 4 envs in one 16-B load
        const uint4 v = reinterpret_cast<const uint4*>(sh.cell + q * FEPB)[threadIdx.x];
        c[0] = v.x; c[1] = v.y; c[2] = v.z; c[3] = v.w;
      } else {
        uint32_t r = excl[q];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t bit = (fm[q] >> i) & 1u;
          c[i] = sh.cell[q * FEPB + min(r, (uint32_t)FEPB - 1u)];
          r += bit;
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if ((fm[q] >> i) & 1u) {
          gl[q][i] = (int)(c[i] & 0xFFFFu);
          ae[q][i] = c[i] >> 16;
        }
      }
      if constexpr (!STG) {
#pragma unroll
        for (int i = 0; i < 4; ++i) pc[q][i] = c[i];
        pfm[q] = fm[q];
      }
    }
  };
  if (sh.drawn) {  // common case: drawn before B2
#pragma unroll
    for (int q = 0; q < QPT; ++q) consume(q);
    return;
  }
  uint32_t slow = sh.anyrej;
  if (!slow && b > (uint32_t)nt * RCOV)  // mass reset: extend call-1 coverage
    slow = coverage_round(p.self, st, slots + G, nt, G, QPT, tag0 + 1, (uint32_t)nt * RCOV, b - nt * RCOV, n1, thr1,
                          sh);
  if (!slow && ncalls == 2)  // agent words start right after the b goal words
    slow = coverage_round(p.self, st, slots + 2 * G, nt, G, QPT, tag0 + 2, b, b, (uint32_t)p.n_agent_valid,
                          p.thr_agent, sh);
  uint32_t w1 = b;
  if (slow && ncalls == 2) {
    if constexpr (ROLE == R_CTRL) {
      const uint32_t a = scan_accepted(p.self, st, 0, n1, thr1, b - 1, b, nullptr);
      if (lane == 0) sh.w1 = a;
    }
    lds_barrier();
    w1 = sh.w1;
  }
  if (!slow) {
    if constexpr (ROLE == R_CTRL) ctrl_draw_cells<OK, QPT, STG>(p, sh, tb, SB, st, w1, nullptr, nullptr, -1, stg);
    lds_barrier();
#pragma unroll
    for (int q = 0; q < QPT; ++q) consume(q);
  } else {
    // slow path (a rejection somewhere): the control wave walks the stream tile by tile
#pragma unroll
    for (int q = 0; q < QPT; ++q) {
      const int tau = q * G + (int)blockIdx.x;
      if (tau >= nt) continue;  // block-uniform
      if constexpr (ROLE == R_CTRL) {
        const uint32_t P = sh.tpre[q];
        uint32_t tc = 0;
#pragma unroll
        for (int w = 0; w < FENVW; ++w) tc += sh.wcnt[q][w];
        if (tc) {
          if (rgoal) scan_accepted(p.self, st, 0, n1, p.thr_goal, P, P + tc, sh.pos);
          if (ragent)
            scan_accepted(p.self, st, rgoal ? w1 : 0, (uint32_t)p.n_agent_valid, p.thr_agent, P, P + tc,
                          rgoal ? sh.pos2 : sh.pos);
        }
        ctrl_draw_cells<OK, QPT, STG>(p, sh, tb, SB, st, w1, sh.pos, rgoal ? sh.pos2 : sh.pos, q, stg);
      }
      lds_barrier();
      consume(q);
    }
  }
  if (!sh.known) {  // block-uniform: the slow / multi-call / extended cases
    if constexpr (ROLE == R_CTRL) {
      uint32_t wtot;
      if (!slow) {
        wtot = (uint32_t)ncalls * b;
      } else {
        const bool last_goal = ncalls == 1 && rgoal;
        wtot = scan_accepted(p.self, st, ncalls == 2 ? w1 : 0u, last_goal ? n1 : (uint32_t)p.n_agent_valid,
                             last_goal ? p.thr_goal : p.thr_agent, b - 1, b, nullptr);
      }
      publish_next(tb, sh, SB, wtot, st.h0, st.u0, lane == 0);
    }
    lds_barrier();
  }
}


// Effective action of env with action a and 53-bit uniform k: min(#{j : k > thr[a][j]}, NA - 1) (integer
// form of action_utils.py:84-90 with the reference's cumsum thresholds). The thresholds of a row are
// non-decreasing (a cumulative sum), so the count is the first j with k <= thr[j]: NA - 1 compares as a
// select chain (the last threshold never matters: k > thr[NA-2] already gives NA - 1 after the clamp).
// A (uniform) value pinned to a VGPR: the opaque move keeps the compiler from re-materialising it in the
// SGPR file, whose pressure spills values to VGPR lanes in the fused loop.
__device__ __forceinline__ uint32_t vgpr_u32(uint32_t x) {
#if GP_VPIN
  uint32_t v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"(x));
  return v;
#else
  return __builtin_amdgcn_readfirstlane(x);
#endif
}
__device__ __forceinline__ int32_t vgpr_u32(int32_t x) { return (int32_t)vgpr_u32((uint32_t)x); }

// PCG64 XSL-RR output with the 64-bit rotate as two v_alignbit_b32 (same value as pcg_output).
__device__ __forceinline__ uint64_t pcg_output_ab(u128 s) {
  const uint64_t hi = hi64(s), lo = lo64(s);
  const uint32_t xh = (uint32_t)(hi >> 32) ^ (uint32_t)(lo >> 32), xl = (uint32_t)hi ^ (uint32_t)lo;
  const uint32_t r = (uint32_t)(hi >> 58);
  const bool sw = (r & 32u) != 0;  // a rotate by >= 32 first swaps the halves
  const uint32_t H = sw ? xl : xh, L = sw ? xh : xl;
  const uint32_t olo = __builtin_amdgcn_alignbit(H, L, r), ohi = __builtin_amdgcn_alignbit(L, H, r);
  return ((uint64_t)ohi << 32) | olo;
}
// A 53-bit threshold t as a threshold on the full 64-bit draw x: (x >> 11) > t  <=>  x > (t << 11) | 0x7FF
// (t >= 2^53, a cumulative sum of 1.0, is never exceeded: saturate).
__host__ __device__ __forceinline__ uint64_t thr_on_u64(uint64_t t) {
  return t >= (1ull << 53) ? ~0ull : ((t << 11) | 0x7FFull);
}
// Sanitised action -> byte offset of its threshold row in s_thr (numpy negative indexing; out-of-range
// actions, which raise IndexError in the reference, set GP_DERR_ACTION and are clamped).
template <int NA>
__device__ __forceinline__ int32_t action_row(int32_t a, uint32_t* derr) {
  if (action_out_of_range(a, NA)) flag_bad_action(derr);
  if (a < 0) a += NA;
  return min(max(a, 0), NA - 1) * NA * 8;
}
// Effective action x 2 (the byte offset of its entry in a move-table row) from the 64-bit draw x and the
// pre-shifted thresholds of row `boff` (16-B loads: rows are 32/64-B aligned).
template <int NA>
__device__ __forceinline__ uint32_t fused_effx_row(const uint64_t* s_thr, int boff, uint64_t x) {
  const ulonglong2* t = reinterpret_cast<const ulonglong2*>(reinterpret_cast<const char*>(s_thr) + boff);
  uint64_t th[NA];
#pragma unroll
  for (int j = 0; j < NA / 2; ++j) {
    const ulonglong2 v = t[j];
    th[2 * j] = v.x;
    th[2 * j + 1] = v.y;
  }
  uint32_t e = 0;
#pragma unroll
  for (int j = 0; j < NA - 1; ++j) e = x > th[j] ? (uint32_t)(2 * (j + 1)) : e;
  return e;
}

template <int NA>
__device__ __forceinline__ uint32_t fused_effective_action(const uint64_t* s_thr, int a, uint64_t k) {
  const uint64_t* t = s_thr + a * NA;
  uint32_t e = 0;
#pragma unroll
  for (int j = 0; j < NA - 1; ++j) e = k > t[j] ? (uint32_t)(j + 1) : e;
  return e;
}

// The obs of the previous step's resetters (their provisional obs were stored with the step's
// outputs): written during the next step's exchange wait.
template <int OK, int QPT, bool SMALL>
__device__ __forceinline__ void flush_reset_obs(const GridDev& p, const LTabs& tb, void* ob, int tid,
                                                const uint32_t (&pc)[QPT][4], uint32_t (&pfm)[QPT]) {
#pragma unroll
  for (int q = 0; q < QPT; ++q) {
    if (!pfm[q]) continue;
    const int env0 = (q * (int)gridDim.x + (int)blockIdx.x) * (SMALL ? p.ftile : FEPB) + tid * EPT;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if ((pfm[q] >> i) & 1u) write_obs<OK>(p, tb, env0 + i, (int)(pc[q][i] >> 16), (int)(pc[q][i] & 0xFFFFu), ob);
    pfm[q] = 0;
  }
}

// The env waves of the fused kernel.
template <int OK, int QPT, int NA, bool STG, bool SMALL>
__device__ __forceinline__ void fused_env(const GridDev& p_in, FusedShared& sh, const uint64_t* s_thr,
                                          const LTabs& tb, char* stg, int K, const int32_t* __restrict__ act,
                                          void* __restrict__ obs, float* __restrict__ rew,
                                          uint8_t* __restrict__ term, uint8_t* __restrict__ trunc, float& rsum,
                                          uint32_t& eps, uint32_t& lens, uint32_t& nst) {
  const GridDev& p = p_in;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const GridCtl* C = p.ctl;
  const int G = (int)gridDim.x;
  const int nt = p.fnt;
  const int B = p.B;
  const bool rgoal = p.fixed_goal < 0;
  const int ncalls = (int)rgoal + (int)(p.fixed_agent < 0);
  const int fixed_agent = p.fixed_agent, fixed_goal = p.fixed_goal, tlim = p.time_limit;
  const float r_step = p.r_step, r_wall = p.r_wall, r_goal = p.r_goal;
  Stream st;
  st.s0 = mk128(C->s_hi, C->s_lo);
  st.inc = mk128(C->inc_hi, C->inc_lo);
  st.h0 = C->has_u32;
  st.u0 = C->uinteger;
  st.U0 = (uint32_t)B;
  const uint32_t step_base = C->step;
  const size_t ow = (size_t)p.obs_width * ((OK == GP_OBS_HANSEN_VEC || OK == GP_OBS_WINDOW) ? 1 : 4);
  const PcgJump jB_unused{0, 1, 0, 0};
  constexpr bool TRIMS = GP_TRIMS;
  const int TILE = SMALL ? p.ftile : FEPB;  // envs per tile (compile-time 2048 unless SMALL)
  uint32_t ae[QPT][4];
  int gl[QPT][4];
  int32_t a_cur[QPT][4];  // TRIMS: threshold-row byte offsets (action_row) instead of raw actions
  // GP_ACC: valid-env masks (partial tiles), goal / wall-bump counts; rewards and lengths at the end
  uint32_t vmask[QPT], ngoal = 0, nwall = 0;
  u128 S[QPT];  // lane draw state: jump(s0, e0 + 1)
  uint32_t pc[QPT][4], pfm[QPT];  // previous step's resetters: new cells (goal | agent << 16), masks
  int dof[8];                     // goal-direction offsets (uniform, in VGPRs) for the staged Hansen obs
  const PcgJump jl = p.flt4[tid];
  PcgJump jtile[QPT];
#pragma unroll
  for (int q = 0; q < QPT; ++q) {
    const int tau = q * G + (int)blockIdx.x;
    const int env0 = tau * TILE + tid * EPT;
    pfm[q] = 0;
    load4f<uint32_t>(p.ae, env0, B, ae[q]);
    if (rgoal) {
      uint16_t gg[4];
      load4f<uint16_t>(p.goal, env0, B, gg);
#pragma unroll
      for (int i = 0; i < 4; ++i) gl[q][i] = gg[i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) gl[q][i] = fixed_goal;
    }
    load4f<int32_t>(act, env0, B, a_cur[q]);
    jtile[q] = p.ftj[min(tau, nt - 1)];
  }
  const PcgJump jstride = p.fjB[1];
  if constexpr (GP_PRO2) {
    // keep the state / action / jump loads above ahead of the table copy's (the compiler otherwise sinks them
    // below it, and their latency lands after the barrier): their latencies overlap
    asm volatile("" ::: "memory");
    // the small lookup tables and shared words while the loads above are in flight, then the block barrier
    char* dyn = const_cast<char*>(tb.dyn);
    if (tid < NA * NA) const_cast<uint64_t*>(s_thr)[tid] = GP_TRIMS ? thr_on_u64(p.thr[tid]) : p.thr[tid];
    if (tid < 4) sh.jB[tid] = (&p.fjB->a_hi)[tid];
    if (tid < 8) sh.dof[tid] = (OK == GP_OBS_HANSEN && p.doff && tid < p.obs_dirs) ? p.doff[tid] : 0x7FFFFFFF;
    if (tid == 0) {
      sh.rdone = 0;
      sh.spw_done = 0;
    }
    lds_image_copy_range(dyn, p.limg, 0, p.lds.jt.off, tid, FENVW * 64);
    __syncthreads();
    LSTAMP(1);
  }
#pragma unroll
  for (int q = 0; q < QPT; ++q) {
    const int tau = q * G + (int)blockIdx.x;
    const int env0 = tau * TILE + tid * EPT;
    if constexpr (TRIMS) {
#pragma unroll
      for (int i = 0; i < 4; ++i) a_cur[q][i] = action_row<NA>(a_cur[q][i], &p.ctl->err);
    }
    vmask[q] = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) vmask[q] |= (STG || env0 + i < B) ? 1u << i : 0u;
    if constexpr (GP_ACC) {
      // episode lengths ended in this launch = steps taken + elapsed at the start - elapsed at the end
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((vmask[q] >> i) & 1u) lens += ae[q][i] >> 16;
    }
  }
  LSTAMP(4);
#pragma unroll
  for (int d = 0; d < 8; ++d)
    dof[d] = (OK == GP_OBS_HANSEN && d < p.obs_dirs) ? vgpr_u32(tb.doff(d)) : 0x7FFFFFFF;
  // The stream increment as VGPR operands: uniform, but SGPRs are the scarce file in this loop (kept there,
  // it was spilled to VGPR lanes and re-read by v_readlane + v_mov in every draw).
  const u128 incv = mk128(((uint64_t)vgpr_u32((uint32_t)(hi64(st.inc) >> 32)) << 32) | vgpr_u32((uint32_t)hi64(st.inc)),
                          ((uint64_t)vgpr_u32((uint32_t)(lo64(st.inc) >> 32)) << 32) | vgpr_u32((uint32_t)lo64(st.inc)));
  // lane draw states jump(s0, e0 + 1): tile 0 by its tile base then this thread's offset (two affine maps, no
  // composition), the block's further tiles by the tile stride from the previous one
  S[0] = apply_jump(jl, apply_jump(jtile[0], st.s0));
#pragma unroll
  for (int q = 1; q < QPT; ++q) S[q] = apply_jump(jstride, S[q - 1]);
  LSTAMP(5);
  for (int k = 0; k < K; ++k) {
    STAMP(0);
    const uint32_t tag0 = (step_base + (uint32_t)k + 1u) * 4u;
    uint64_t* slots = p.fslot + (size_t)((step_base + (uint32_t)k) & 1u) * 3 * G;
    int32_t a_nxt[QPT][4];
    if (k + 1 < K) {
#pragma unroll
      for (int q = 0; q < QPT; ++q)
      {
        const int e0 = (q * G + (int)blockIdx.x) * TILE + tid * EPT;
        if constexpr (STG) {  // complete tiles: one unconditional 16-B load
          const int4 v = *reinterpret_cast<const int4*>(act + (size_t)(k + 1) * B + e0);
          a_nxt[q][0] = v.x; a_nxt[q][1] = v.y; a_nxt[q][2] = v.z; a_nxt[q][3] = v.w;
        } else {
          load4f<int32_t>(act + (size_t)(k + 1) * B, e0, B, a_nxt[q]);
        }
      }
    }
    // ---- 1. draws + transitions (the critical path) ----
    uint32_t fm[QPT], tmm[QPT], trm[QPT], bkm[QPT], excl[QPT], wex[QPT], wt[QPT];
    u128 sd[QPT];  // draw states of the tiles' current env slots
#pragma unroll
    for (int q = 0; q < QPT; ++q) {
      fm[q] = tmm[q] = trm[q] = bkm[q] = 0;
      sd[q] = S[q];
    }
#pragma unroll
    for (int o = 0; o < QPT * 4; ++o) {
      // GP_ILV: slot-major (q fastest) so that the tiles' dependent draw chains interleave
      const int q = GP_ILV ? o % QPT : o / 4, i = GP_ILV ? o / QPT : o % 4;
      const int env0 = (q * G + (int)blockIdx.x) * TILE + tid * EPT;
      {
        u128& s = sd[q];
        if (i) s = pcg_step(s, incv);
        const uint32_t s_ae = ae[q][i];
        uint32_t m;
        if constexpr (TRIMS) {
          const uint32_t effx =
              fused_effx_row<NA>(s_thr, a_cur[q][i], GP_ALIGNBIT ? pcg_output_ab(s) : pcg_output(s));
          m = tb.move_b(((s_ae & 0xFFFFu) << (NA == 4 ? 3 : 4)) + effx);
        } else {
          const uint64_t k53 = pcg_output(s) >> 11;
          int a = a_cur[q][i];
          if (action_out_of_range(a, NA)) flag_bad_action(&p.ctl->err);
          if (a < 0) a += NA;                 // numpy negative indexing of action_matrix[action]
          a = min(max(a, 0), NA - 1);         // (out-of-range actions raise in the reference; clamped here)
          const uint32_t eff = fused_effective_action<NA>(s_thr, a, k53);
          m = tb.move((int)(s_ae & 0xFFFFu) * NA + (int)eff);
        }
        const int na_ = (int)__builtin_amdgcn_ubfe(m, 0, 15);
        const bool blocked = (m >> 15) != 0;
        const uint32_t el = (s_ae >> 16) + 1u;
        const bool tm_ = na_ == gl[q][i];
        const bool tr_ = el > (uint32_t)tlim;
        const bool valid = STG || env0 + i < B;  // STG launches have only complete tiles
        const bool f = valid && (tm_ || tr_);
        const float rw = tm_ ? r_goal : (blocked ? r_wall : r_step);
        tmm[q] |= (uint32_t)tm_ << i;
        bkm[q] |= (uint32_t)blocked << i;
        trm[q] |= (uint32_t)tr_ << i;
        fm[q] |= (uint32_t)f << i;
        const int ag = f && fixed_agent >= 0 ? fixed_agent : na_;
        ae[q][i] = (uint32_t)ag | ((f ? 0u : el) << 16);
        if (f && fixed_goal >= 0) gl[q][i] = fixed_goal;
        if constexpr (!GP_ACC) {
          if (valid) {
            rsum += rw;
            nst += 1;
          }
          if (f) {
            eps += 1;
            lens += el;
          }
        }
      }
    }
    if constexpr (GP_ACC) {
#pragma unroll
      for (int q = 0; q < QPT; ++q) {
        const uint32_t vm = STG ? 0xFu : vmask[q];
        eps += (uint32_t)__builtin_popcount(fm[q]);
        ngoal += (uint32_t)__builtin_popcount(tmm[q] & vm);
        nwall += (uint32_t)__builtin_popcount(bkm[q] & ~tmm[q] & vm);
      }
    }
    // the per-wave reset counts after both tiles' transitions (their VALU chains interleave: -2.5% per step)
#pragma unroll
    for (int q = 0; q < QPT; ++q) {
      wave_count_prefix((uint32_t)__builtin_popcount(fm[q]), wex[q], wt[q]);
      if (lane == 0) sh.wcnt[q][wid] = wt[q];
    }
    STAMP(1);
    lds_barrier();  // B1: per-wave reset counts are in LDS
    STAMP(2);
#pragma unroll
    for (int q = 0; q < QPT; ++q) {
      uint32_t woff = 0;
#pragma unroll
      for (int w = 0; w < FENVW; ++w) woff += w < wid ? sh.wcnt[q][w] : 0u;
      excl[q] = wex[q] + woff;
    }
    if constexpr (STG) {
      // list this wave's resetters (rank -> env in tile) for the control wave, which writes their
      // final obs into the staging area once it has drawn their cells
#pragma unroll
      for (int q = 0; q < QPT; ++q) {
        uint32_t r = excl[q];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if ((fm[q] >> i) & 1u) {
            sh.renv[q][min(r, (uint32_t)FEPB - 1u)] = (uint16_t)(tid * EPT + i);
            ++r;
          }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      if (lane == 0) __hip_atomic_fetch_add(&sh.rdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    STAMP(11);
    // ---- 3. this step's outputs (overlap the exchange) ----
    size_t off = (size_t)k * B;
#ifdef GP_STAMPS
    if (p.xmode & 8) off = 0;  // diagnostic: every step writes the first step's slice
#endif
    void* ob = (uint8_t*)obs + off * ow;
    if constexpr (STG) {
      // into the LDS staging area; the store waves move it to HBM during the next VALU phases, so
      // no global store competes with the exchange (resetters' obs: written by the control wave)
      int32_t obv[QPT][4];
      if (OK == GP_OBS_HANSEN && tb.has_ofix()) {  // uniform: the fixed-goal table, all loads in flight together
#pragma unroll
        for (int q = 0; q < QPT; ++q)
#pragma unroll
          for (int i = 0; i < 4; ++i) obv[q][i] = tb.ofix((int)(ae[q][i] & 0xFFFFu));
      } else {
#pragma unroll
        for (int q = 0; q < QPT; ++q)
#pragma unroll
          for (int i = 0; i < 4; ++i) obv[q][i] = obs_value_r<OK>(p, tb, (int)(ae[q][i] & 0xFFFFu), gl[q][i], dof);
      }
#pragma unroll
      for (int q = 0; q < QPT; ++q) {
        char* t = stg + q * STG_TILE_BYTES;
        int4 ov;
        ov.x = obv[q][0];
        ov.y = obv[q][1];
        ov.z = obv[q][2];
        ov.w = obv[q][3];
        const uint32_t drawm = ncalls ? fm[q] : 0u;  // resetters whose cells the control wave draws
        if (!drawm) {
          reinterpret_cast<int4*>(t)[tid] = ov;
        } else {
          int32_t* o = reinterpret_cast<int32_t*>(t) + tid * EPT;
          if (!(drawm & 1u)) o[0] = ov.x;
          if (!(drawm & 2u)) o[1] = ov.y;
          if (!(drawm & 4u)) o[2] = ov.z;
          if (!(drawm & 8u)) o[3] = ov.w;
        }
        float rw[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          rw[i] = ((tmm[q] >> i) & 1u) ? r_goal : (((bkm[q] >> i) & 1u) ? r_wall : r_step);
        reinterpret_cast<float4*>(t + FEPB * 4)[tid] = make_float4(rw[0], rw[1], rw[2], rw[3]);
        uint32_t tmw = 0, trw = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          tmw |= ((tmm[q] >> i) & 1u) << (8 * i);
          trw |= ((trm[q] >> i) & 1u) << (8 * i);
        }
        reinterpret_cast<uint32_t*>(t + FEPB * 8)[tid] = tmw;
        reinterpret_cast<uint32_t*>(t + FEPB * 9)[tid] = trw;
      }
    } else {
#pragma unroll
      for (int q = 0; q < QPT; ++q) {
#ifdef GP_STAMPS
        if (p.xmode & 4) break;  // diagnostic: no output stores
#endif
        const int env0 = (q * G + (int)blockIdx.x) * TILE + tid * EPT;
        uint8_t tm[4], tr[4];
        int ag[4];
        float rw[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          tm[i] = (uint8_t)((tmm[q] >> i) & 1u);
          tr[i] = (uint8_t)((trm[q] >> i) & 1u);
          ag[i] = (int)(ae[q][i] & 0xFFFFu);
          rw[i] = tm[i] ? r_goal : (((bkm[q] >> i) & 1u) ? r_wall : r_step);
        }
        store4f<float>(rew + off, env0, B, rw);
        store4f<uint8_t>(term + off, env0, B, tm);
        store4f<uint8_t>(trunc + off, env0, B, tr);
        // one vector store for all 4 envs (uniform store count per step: no vmcnt(0) at merges);
        // a resetter's obs is provisional here and rewritten in phase 4
        write_obs4<OK, LTabs, true>(p, tb, env0, ag, gl[q], ob);
      }
    }
    STAMP(12);
    if (!STG && k > 0) flush_reset_obs<OK, QPT, SMALL>(p, tb, (uint8_t*)obs + (off ? off - B : 0) * ow, tid, pc, pfm);
    {
      const PcgJump jB{sh.jB[0], sh.jB[1], sh.jB[2], sh.jB[3]};
#pragma unroll
      for (int q = 0; q < QPT; ++q) S[q] = apply_jump(jB, S[q]);  // first half of the advance (J_B)
    }
    if constexpr (TRIMS) {  // the next step's actions -> threshold rows, while the exchange runs
      if (k + 1 < K) {
#pragma unroll
        for (int q = 0; q < QPT; ++q)
#pragma unroll
          for (int i = 0; i < 4; ++i) a_nxt[q][i] = action_row<NA>(a_nxt[q][i], &p.ctl->err);
      }
    }
    STAMP(13);
    lds_barrier();  // B2: the exchange result is in LDS
    STAMP(4);
    // ---- 4. the resetters' draws ----
    fused_resets<OK, QPT, R_ENV, STG>(p, sh, tb, st, st.s0, jB_unused, slots, tag0, ae, gl, fm, excl, pc, pfm, stg);
    STAMP(3);
    // ---- 5. advance: lane states jump by J_used (J_B was applied while waiting for the exchange) ----
    {
      const PcgJump jt{sh.ju[0], sh.ju[1], sh.ju[2], sh.ju[3]};
      st.s0 = mk128(sh.ns_hi, sh.ns_lo);
      st.h0 = sh.nh;
      st.u0 = sh.nu;
#pragma unroll
      for (int q = 0; q < QPT; ++q) S[q] = apply_jump(jt, S[q]);
    }
    if (k + 1 < K) {
#pragma unroll
      for (int q = 0; q < QPT; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) a_cur[q][i] = a_nxt[q][i];
    }
    STAMP(5);
  }
  if (!STG && K > 0) flush_reset_obs<OK, QPT, SMALL>(p, tb, (uint8_t*)obs + (size_t)(K - 1) * B * ow, tid, pc, pfm);
  if constexpr (GP_ACC) {
    uint32_t nv = 0;
#pragma unroll
    for (int q = 0; q < QPT; ++q) {
      nv += (uint32_t)__builtin_popcount(vmask[q]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((vmask[q] >> i) & 1u) lens -= ae[q][i] >> 16;
    }
    const uint32_t steps = nv * (uint32_t)K;
    lens += steps;
    nst += steps;
    rsum += (float)ngoal * r_goal + (float)nwall * r_wall + (float)(steps - ngoal - nwall) * r_step;
  }
#pragma unroll
  for (int q = 0; q < QPT; ++q) {
    const int env0 = (q * G + (int)blockIdx.x) * TILE + tid * EPT;
    store4f<uint32_t>(p.ae, env0, B, ae[q]);
    if (rgoal) {
      uint16_t gg[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) gg[i] = (uint16_t)gl[q][i];
      store4f<uint16_t>(p.goal, env0, B, gg);
    }
  }
}

// The control wave of the fused kernel: speculative rejection checks, the granule exchange, the
// next PCG64 state; publishes the RNG state at the end (block 0).
template <int OK, int QPT, bool STG, bool SMALL>
__device__ __forceinline__ void fused_ctrl(const GridDev& p_in, FusedShared& sh, const LTabs& tb, char* stg, int K) {
  constexpr int NC = (QPT + 1) / 2;  // checker states per lane (32 lanes per tile)
  const GridDev& p = p_in;
  const int tid = threadIdx.x, lane = tid & 63;
  GridCtl* C = p.ctl;
  const int G = (int)gridDim.x;
  const int nt = p.fnt;
  const bool rgoal = p.fixed_goal < 0, ragent = p.fixed_agent < 0;
  const int ncalls = (int)rgoal + (int)ragent;
  const uint32_t n1 = rgoal ? (uint32_t)p.n_goal_valid : (uint32_t)p.n_agent_valid;
  const uint32_t thr1 = rgoal ? p.thr_goal : p.thr_agent;
  Stream st;
  st.s0 = mk128(C->s_hi, C->s_lo);
  st.inc = mk128(C->inc_hi, C->inc_lo);
  st.h0 = C->has_u32;
  st.u0 = C->uinteger;
  st.U0 = (uint32_t)p.B;
  const uint32_t step_base = C->step;
  const PcgJump jB = *p.fjB;
  uint32_t bprev = C->fb_last;  // SPW: the reset words of the previous step (window centres)
  uint32_t d_ready = 0, d_nojump = 0;  // GP_STAMPS diagnostics: steps with the windows ready / with no lane jumping
  // lane l checks tile q = 2c + (l >> 5); lane ll = l & 31 holds u64 #(tau*31 - 1 + ll) of the
  // post-random(B) stream, i.e. jump(s0, B + tau*31 + ll)
  u128 CS[NC];
  bool chk[NC];
  int ctau[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int q = 2 * c + (lane >> 5);
    ctau[c] = q * G + (int)blockIdx.x;
    chk[c] = ncalls && q < QPT && ctau[c] < nt;
    CS[c] = chk[c] ? pcg_jump(GP_PRO2 ? p.jt : tb.jt(), st.s0,
                              (uint32_t)p.B + (uint32_t)ctau[c] * (RCOV / 2) + (uint32_t)(lane & 31))
                   : (u128)0;
  }
  if constexpr (GP_PRO2) __syncthreads();  // the prologue barrier (the env waves staged the small tables)
  uint32_t dummy_u[QPT][4];
  int dummy_i[QPT][4];
  const uint32_t dummy_c[QPT] = {};
  uint32_t dummy_p[QPT] = {};
  for (int k = 0; k < K; ++k) {
    const uint32_t tag0 = (step_base + (uint32_t)k + 1u) * 4u;
    uint64_t* slots = p.fslot + (size_t)((step_base + (uint32_t)k) & 1u) * 3 * G;
    int cdof[8];  // goal-direction offsets for the resetters' staged obs (read long before they are used)
#pragma unroll
    for (int d = 0; d < 8; ++d) cdof[d] = sh.dof[d];
    // speculative Lemire check of the RCOV-word windows of this block's tiles (call 1)
    uint32_t crej = 0;
    const uint32_t ll = lane & 31;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (!chk[c]) continue;
      const uint64_t x = pcg_output(CS[c]);
      const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
      bool rj;
      if (!st.h0) {
        rj = ll >= 1 && (lemire_rejected(lo, n1, thr1) || lemire_rejected(hi, n1, thr1));
      } else if (ll == 0) {
        rj = lemire_rejected(ctau[c] == 0 ? st.u0 : hi, n1, thr1);
      } else if (ll < 31) {
        rj = lemire_rejected(lo, n1, thr1) || lemire_rejected(hi, n1, thr1);
      } else {
        rj = lemire_rejected(lo, n1, thr1);
      }
      crej |= rj ? 1u : 0u;
    }
    const uint32_t wrej = __any((int)crej) ? 1u : 0u;
    const u128 SB = apply_jump(jB, st.s0);  // state after random(B): base of the word stream
    if (STG && p.spw_on && lane == 0) {  // what the store waves build this step's windows from (after B1)
      sh.spw_sb[0] = hi64(SB);
      sh.spw_sb[1] = lo64(SB);
      sh.spw_h0 = st.h0;
      sh.spw_b = bprev;
    }
    lds_barrier();  // B1
    // ---- 2. publish this block's granule ----
    uint32_t tq = 0;
    if (lane < QPT) {
#pragma unroll
      for (int w = 0; w < FENVW; ++w) tq += sh.wcnt[lane][w];
    }
    uint64_t counts = 0;
#pragma unroll
    for (int q = 0; q < QPT; ++q) counts |= (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)tq, q) << (12 * q);
    if (lane == 0 && (int)blockIdx.x != p.fault_block) {
      __hip_atomic_store(&slots[blockIdx.x], bgran(tag0, wrej, counts), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      RSTAMP(6);
    }
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (chk[c]) CS[c] = apply_jump(jB, CS[c]);
    // ---- 3. exchange: block 0 aggregates and publishes one tagged word per tile
    // {rejection, b, tile prefix}; every other block polls only its own QPT words ----
    uint64_t* tw = p.fslot + (size_t)6 * G + (size_t)((step_base + (uint32_t)k) & 1u) * nt;
    uint32_t b, anyr, mypre = 0;  // lane q < QPT: global prefix of tile q
    if (blockIdx.x == 0 || (p.xmode & 3) == 1) {
      uint64_t g[4];
      gather_blocks(p, slots, G, tag0, g);
      if (lane == 0) RSTAMP(10);
      uint32_t rj = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) rj |= (uint32_t)(g[j] >> 48) & 1u;
      anyr = __any((int)rj) ? 1u : 0u;
      uint32_t pre[QPT][4];
      uint32_t acc = 0;
#pragma unroll
      for (int q = 0; q < QPT; ++q) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) v += gcount(g[j], q);
        const uint32_t incl = wave_incl_scan(v);
        uint32_t run = acc + incl - v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pre[q][j] = run;
          run += gcount(g[j], q);
        }
        acc += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      }
      b = acc;
      if ((p.xmode & 3) == 0) {
#pragma unroll
        for (int q = 0; q < QPT; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int blk = lane * 4 + j, tau = q * G + blk;
            if (blk < G && tau < nt)
              __hip_atomic_store(&tw[tau], tword(tag0, anyr, b, pre[q][j]), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
          }
      }
      const int bl = (int)blockIdx.x >> 2, bj = (int)blockIdx.x & 3;
#pragma unroll
      for (int q = 0; q < QPT; ++q) {
        const uint32_t sel = bj == 0 ? pre[q][0] : bj == 1 ? pre[q][1] : bj == 2 ? pre[q][2] : pre[q][3];
        const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)sel, bl);
        if (lane == q) mypre = v;
      }
    } else {
      uint64_t w = 0;
      const int tau = lane * G + (int)blockIdx.x;
      if (lane < QPT && tau < nt) {
        const uint64_t want = (uint64_t)(tag0 & TAG_MASK);
        uint32_t spins = 0;
        w = __hip_atomic_load(&tw[tau], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while ((w >> 49) != want) {
          __builtin_amdgcn_s_sleep(1);
          w = __hip_atomic_load(&tw[tau], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (spin_give_up(p, spins)) {
            w = want << 49;
            break;
          }
        }
        mypre = (uint32_t)w & 0xFFFFFFu;
      }
      const uint64_t w0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(w >> 32), 0) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)w, 0);
      b = (uint32_t)(w0 >> 24) & 0xFFFFFFu;
      anyr = (uint32_t)(w0 >> 48) & 1u;
    }
    if (lane == 0) RSTAMP(8);
    const bool known = b == 0 || ncalls == 0 || (!anyr && ncalls == 1 && b <= (uint32_t)nt * RCOV);
    const bool drawn = known && ncalls == 1 && b > 0;
    if (lane < QPT) sh.tpre[lane] = mypre;
    wave_lds_sync();
    if (STG && ncalls) {  // the env waves' resetter lists (written right after B1: normally long done)
      const uint32_t want = (uint32_t)(SMALL ? p.faw : FENVW) * (uint32_t)(k + 1);  // env waves that own envs
      while (__hip_atomic_load(&sh.rdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < want)
        __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
    bprev = b;
    if (lane == 0) RSTAMP(14);
    if (drawn) {
      const uint64_t* spw = nullptr;  // the store waves' windows, if complete (never waited for)
      if (STG && p.spw_on &&
          __hip_atomic_load(&sh.spw_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= (uint32_t)FSTW * (k + 1)) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        spw = reinterpret_cast<const uint64_t*>(stg + QPT * STG_TILE_BYTES);
      }
      const uint32_t jmp = ctrl_fast_finish<OK, QPT, STG>(p, sh, tb, SB, st, b, tq, mypre, stg, cdof, spw, k);
      d_ready += spw ? 1u : 0u;
      d_nojump += jmp ? 0u : 1u;
    } else if (known) {
      publish_next(tb, sh, SB, ncalls ? b : 0u, st.h0, st.u0, lane == 0);
    }
    if (lane == 0) RSTAMP(9);
    if (lane == 0) {
      sh.btot = b;
      sh.anyrej = anyr;
      sh.known = known ? 1u : 0u;
      sh.drawn = drawn ? 1u : 0u;
      RSTAMP(7);
    }
    lds_barrier();  // B2
    // ---- 4. coverage exchanges / stream walks of the unusual cases ----
    fused_resets<OK, QPT, R_CTRL, STG>(p, sh, tb, st, SB, jB, slots, tag0, dummy_u, dummy_i, dummy_c, dummy_c, dummy_u,
                                dummy_p, stg);
    // ---- 5. advance ----
    {
      const PcgJump jt{sh.ju[0], sh.ju[1], sh.ju[2], sh.ju[3]};
      st.s0 = mk128(sh.ns_hi, sh.ns_lo);
      st.h0 = sh.nh;
      st.u0 = sh.nu;
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (chk[c]) CS[c] = apply_jump(jt, CS[c]);
    }
  }
  if (blockIdx.x == 0 && lane == 0) {
    C->s_hi = hi64(st.s0);
    C->s_lo = lo64(st.s0);
    C->has_u32 = st.h0;
    C->uinteger = st.u0;
    C->step = step_base + (uint32_t)K;
    C->fb_last = bprev;
  }
#ifdef GP_STAMPS
  if (lane == 0) {  // launch region slots 6, 7: steps with the SPW windows ready, steps where no lane jumped
    p.dbg[(size_t)256 * 64 * 16 + (size_t)blockIdx.x * 8 + 6] = d_ready;
    p.dbg[(size_t)256 * 64 * 16 + (size_t)blockIdx.x * 8 + 7] = d_nojump;
  }
#else
  (void)d_ready;
  (void)d_nojump;
#endif
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Cache policy of the staged output stream (16-B stores by the store waves). GP_OUT_WT 1: `sc1` vector stores,
// written through the XCD's L2 and dropped from it, so a launch ends with no dirty output lines to write back
// (the kernel-end release pays for every dirty byte: MI355X_MICROARCH.md "boundary"); 0: `nt` (kept in L2).
#ifndef GP_OUT_WT
#define GP_OUT_WT 0  // measured: sc1 made K = 128 launches 9% and K = 20 launches 2% slower than nt
#endif
__device__ __forceinline__ void out_store16(u32x4* d, u32x4 v) {
#if GP_OUT_WT
  asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(d), "v"(v));  // no clobber: never read back
#else
  __builtin_nontemporal_store(v, d);
#endif
}
// Copy one staged output plane of tile tau (n32 = 32-bit words per env) to HBM: 16-B chunks of
// 4 (n32 = 1) or 16 (n32 = 0: byte planes) envs when the destination is 16-B aligned, else 4-B words.
template <int TILE>
__device__ __forceinline__ void stage_plane_whole(const char* src, char* dst, int env_base, int esz, int sl, bool nt) {
  // whole aligned tile (the common case): straight-line 16-B copies, immediate offsets; lane sl takes chunks
  // sl, sl + NL, ... of the plane's TILE / 4 (4-byte elements) or TILE / 16 (bytes) chunks
  constexpr int NL = FSTW * 64, N4 = TILE / 4, N1 = TILE / 16;
  const u32x4* s4 = reinterpret_cast<const u32x4*>(src) + sl;
  u32x4* d4 = reinterpret_cast<u32x4*>(dst + (size_t)env_base * esz) + sl;
  if (esz == 4) {
#pragma unroll
    for (int j = 0; j < (N4 + NL - 1) / NL; ++j) {
      if (N4 % NL != 0 && sl + j * NL >= N4) break;
      if (nt) out_store16(d4 + j * NL, s4[j * NL]);
      else d4[j * NL] = s4[j * NL];
    }
  } else {
#pragma unroll
    for (int j = 0; j < (N1 + NL - 1) / NL; ++j) {
      if (N1 % NL != 0 && sl + j * NL >= N1) break;
      if (nt) out_store16(d4 + j * NL, s4[j * NL]);
      else d4[j * NL] = s4[j * NL];
    }
  }
}
__device__ __forceinline__ void stage_plane(const char* src, char* dst, int env_base, int tile, int B, int esz, int sl,
                                            bool nt) {
  constexpr int NL = FSTW * 64;
  if (env_base + tile <= B && (((uintptr_t)dst + (size_t)env_base * esz) & 15) == 0) {
    if (tile == FEPB) stage_plane_whole<FEPB>(src, dst, env_base, esz, sl, nt);
    else if (tile == FEPB / 2) stage_plane_whole<FEPB / 2>(src, dst, env_base, esz, sl, nt);
    else stage_plane_whole<FEPB / 4>(src, dst, env_base, esz, sl, nt);
    return;
  }
  const bool a16 = (((uintptr_t)dst + (size_t)env_base * esz) & 15) == 0;  // wave-uniform
  const int epc = a16 ? 16 / esz : 4 / esz;                                   // envs per chunk
  for (int c = sl; c < tile / epc; c += NL) {
    const int e = env_base + c * epc;
    if (e + epc <= B) {
      if (a16 && nt)
        out_store16(reinterpret_cast<u32x4*>(dst + (size_t)e * esz), reinterpret_cast<const u32x4*>(src)[c]);
      else if (a16)
        *reinterpret_cast<uint4*>(dst + (size_t)e * esz) = reinterpret_cast<const uint4*>(src)[c];
      else
        *reinterpret_cast<uint32_t*>(dst + (size_t)e * esz) = reinterpret_cast<const uint32_t*>(src)[c];
    } else {
      for (int i = 0; i < epc && e + i < B; ++i)
        for (int j = 0; j < esz; ++j) dst[(size_t)(e + i) * esz + j] = src[(size_t)(c * epc + i) * esz + j];
    }
  }
}

// Env waves beyond p.faw when the tiles are smaller than FEPB (strong-scaling shard sizes: 512 / 1024-env tiles
// so that every CU gets a tile): they help stage the tables, post zero reset counts once and then only take part
// in the block barriers (fused_resets role R_PASS), like the store waves minus the copies.
template <int OK, int QPT>
__device__ __forceinline__ void fused_idle(const GridDev& p, FusedShared& sh, const LTabs& tb, int K) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int G = (int)gridDim.x;
  const uint32_t step_base = p.ctl->step;
  const Stream st{};
  const PcgJump jB{0, 1, 0, 0};
  uint32_t du[QPT][4], dp[QPT] = {};
  int di[QPT][4];
  const uint32_t dc[QPT] = {};
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < QPT; ++q) sh.wcnt[q][wid] = 0;
  if constexpr (GP_PRO2) {
    lds_image_copy_range(const_cast<char*>(tb.dyn), p.limg, 0, p.lds.jt.off, tid, FENVW * 64);
    __syncthreads();
  }
  for (int k = 0; k < K; ++k) {
    const uint32_t tag0 = (step_base + (uint32_t)k + 1u) * 4u;
    uint64_t* slots = p.fslot + (size_t)((step_base + (uint32_t)k) & 1u) * 3 * G;
    lds_barrier();  // B1
    lds_barrier();  // B2
    fused_resets<OK, QPT, R_PASS>(p, sh, tb, st, (u128)0, jB, slots, tag0, du, di, dc, dc, du, dp);
  }
}

// SPW: the store waves' windows for this step (after B1, while the exchange is in flight; see SPW_NJ). 128
// lanes: 3 consecutive draws of each tile window and 2 next-state candidates each.
template <int QPT>
__device__ __forceinline__ void spw_fill(const GridDev& p, FusedShared& sh, const LTabs& tb, uint64_t* spw, int sl,
                                         const u128 inc) {
  const int G = (int)gridDim.x, nt = p.fnt;
  const u128 SB = mk128(sh.spw_sb[0], sh.spw_sb[1]);
  const uint32_t h0 = sh.spw_h0, bp = sh.spw_b;
  const PcgJump* t8 = tb.jt8();
#pragma unroll
  for (int q = 0; q < QPT; ++q) {
    const int tau = q * G + (int)blockIdx.x;
    uint32_t n0 = 0;
    if (tau < nt) {
      // predicted first word of the tile (b spread over the tiles in proportion) plus half its expected count
      const uint32_t cw = (uint32_t)(((uint64_t)bp * (uint32_t)tau) / (uint32_t)nt) + bp / (2u * (uint32_t)nt);
      const uint32_t cn = ((cw > h0 ? cw - h0 : 0u) >> 1) + 1u;  // its u64 draw number
      n0 = cn > (uint32_t)SPW_NJ / 2 ? cn - (uint32_t)SPW_NJ / 2 : 1u;
      if (n0 + (uint32_t)SPW_NJ > 65536u) n0 = 0;  // beyond the radix-256 jumps: no window
    }
    if (n0) {
      const uint32_t n = n0 + 3u * (uint32_t)sl;
      u128 X = apply_jump(t8[256u + (n >> 8)], apply_jump(t8[n & 255u], SB));
      uint64_t* w = spw + q * SPW_NJ + 3 * sl;
      w[0] = pcg_output(X);
      X = pcg_step(X, inc);
      w[1] = pcg_output(X);
      X = pcg_step(X, inc);
      w[2] = pcg_output(X);
    }
    if (sl == 0) sh.spw_n0[q] = n0;
  }
  uint32_t up, hp;
  words_to_draws(bp, h0, up, hp);
  const uint32_t u0 = up > (uint32_t)SPW_NU / 2 ? up - (uint32_t)SPW_NU / 2 : 0u;
  if (u0 + (uint32_t)SPW_NU <= 65536u) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t u = u0 + 2u * (uint32_t)sl + (uint32_t)i;
      const PcgJump J = compose_jump(t8[256u + (u >> 8)], t8[u & 255u]);
      const u128 x = apply_jump(J, SB);
      uint64_t* c = spw + QPT * SPW_NJ + (size_t)(u - u0) * SPW_CAND_U64;
      c[0] = J.a_hi; c[1] = J.a_lo; c[2] = J.c_hi; c[3] = J.c_lo; c[4] = hi64(x); c[5] = lo64(x);
    }
  }
  if (sl == 0) sh.spw_u0 = u0 + (uint32_t)SPW_NU <= 65536u ? u0 : 0xFFFFFFFFu;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if ((sl & 63) == 0) __hip_atomic_fetch_add(&sh.spw_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The store waves of the fused kernel. They take part in every block barrier (fused_resets role
// R_PASS) and, with STG, move step k's staged outputs from LDS to HBM right after step k's resets,
// i.e. while the env waves advance and run step k+1's VALU-bound transitions, so that the outputs'
// HBM write burst does not overlap the next exchange (whose polling loads it would slow down).
template <int OK, int QPT, bool STG, bool SMALL>
__device__ __forceinline__ void fused_store(const GridDev& p, FusedShared& sh, const LTabs& tb, const char* stg, int K,
                                            void* __restrict__ obs, float* __restrict__ rew,
                                            uint8_t* __restrict__ term, uint8_t* __restrict__ trunc) {
  const int sl = (int)threadIdx.x - (FENVW + 1) * 64;
  const int G = (int)gridDim.x, B = p.B;
  const bool nt = (p.xmode & 16) == 0;  // non-temporal output stores (xmode bit 4 = tuning knob: plain)
  const uint32_t step_base = p.ctl->step;
  const Stream st{};
  const PcgJump jB{0, 1, 0, 0};
  uint32_t du[QPT][4], dp[QPT] = {};
  int di[QPT][4];
  int32_t dov[QPT][4];
  const uint32_t dc[QPT] = {};
  (void)dov;
  const u128 inc = mk128(p.ctl->inc_hi, p.ctl->inc_lo);
  if constexpr (GP_PRO2) {
    __syncthreads();  // the prologue barrier; then the PCG jump tables behind the first step's transitions
    lds_image_copy_range(const_cast<char*>(tb.dyn), p.limg, p.lds.jt.off, p.lds.total, sl, FSTW * 64);
  }
  for (int k = 0; k < K; ++k) {
    const uint32_t tag0 = (step_base + (uint32_t)k + 1u) * 4u;
    uint64_t* slots = p.fslot + (size_t)((step_base + (uint32_t)k) & 1u) * 3 * G;
    lds_barrier();  // B1
    if constexpr (STG) {
      if (p.spw_on) spw_fill<QPT>(p, sh, tb, reinterpret_cast<uint64_t*>(const_cast<char*>(stg) + QPT * STG_TILE_BYTES),
                                  sl, inc);
    }
    lds_barrier();  // B2
    fused_resets<OK, QPT, R_PASS>(p, sh, tb, st, (u128)0, jB, slots, tag0, du, di, dc, dc, du, dp);
    if constexpr (STG) {
      size_t off = (size_t)k * B;
#ifdef GP_STAMPS
      if (p.xmode & 8) off = 0;  // diagnostic: every step writes the first step's slice
      if (p.xmode & 4) continue;  // diagnostic: no output stores
#endif
#pragma unroll
      for (int q = 0; q < QPT; ++q) {
        const int tau = q * G + (int)blockIdx.x;
        if (tau >= p.fnt) continue;
        const char* t = stg + q * STG_TILE_BYTES;
        const int tile = SMALL ? p.ftile : FEPB;
        stage_plane(t + FEPB * 4, (char*)(rew + off), tau * tile, tile, B, 4, sl, nt);
        stage_plane(t + FEPB * 8, (char*)(term + off), tau * tile, tile, B, 1, sl, nt);
        stage_plane(t + FEPB * 9, (char*)(trunc + off), tau * tile, tile, B, 1, sl, nt);
      }
      // the obs: the resetters' final obs were written by the control wave before the last barrier
#pragma unroll
      for (int q = 0; q < QPT; ++q) {
        const int tau = q * G + (int)blockIdx.x;
        if (tau >= p.fnt) continue;
        const int tile = SMALL ? p.ftile : FEPB;
        stage_plane(stg + q * STG_TILE_BYTES, (char*)obs + off * 4, tau * tile, tile, B, 4, sl, nt);
      }
    }
  }
}

// The parameters come by value. (Passed as a pointer to the device copy GridDev::self instead, the launch
// read no host-resident kernel arguments, but the step loop re-loaded fields through the scalar cache and ran
// ≈10% slower per step: measured in one call, 5.90 vs 5.33 µs/step.)
template <int OK, int QPT, int NA, bool STG, bool SMALL>
__global__ __launch_bounds__(FTPB) void grid_rollout_numpy(GridDev p_in, int K, const int32_t* __restrict__ act,
                                                           void* __restrict__ obs, float* __restrict__ rew,
                                                           uint8_t* __restrict__ term, uint8_t* __restrict__ trunc) {
  __shared__ FusedShared sh;
  __shared__ __attribute__((aligned(16))) uint64_t s_thr[64];
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  const GridDev& p = p_in;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  LSTAMP(0);
  const LTabs tb{p_in, dyn};
  char* stg = dyn + p.lds.total;  // output staging (STG): after the tables, 16-B aligned
  // The launch prologue: the lookup-table image into LDS in one copy loop (the fused path is only taken
  // when it fits) and the small shared words, then a block barrier. (Letting each role issue its own first
  // global loads before this copy, to overlap their latency, measured slower: 17.2 vs 16.1 µs at K = 1.)
  if constexpr (!GP_PRO2) {
    if (tid < NA * NA) s_thr[tid] = GP_TRIMS ? thr_on_u64(p.thr[tid]) : p.thr[tid];
    lds_image_copy(dyn, p.limg, p.lds.total);
    if (tid < 4) sh.jB[tid] = (&p.fjB->a_hi)[tid];
    if (tid == 0) {
      sh.rdone = 0;
      sh.spw_done = 0;
    }
    if (tid < 8) sh.dof[tid] = (OK == GP_OBS_HANSEN && p.doff && tid < p.obs_dirs) ? p.doff[tid] : 0x7FFFFFFF;
    __syncthreads();
    LSTAMP(1);
  }
  float rsum = 0.f;
  uint32_t eps = 0, lens = 0, nst = 0;
  if (wid == FENVW) {
    __builtin_amdgcn_s_setprio(3);  // the exchange is on every step's critical path
    fused_ctrl<OK, QPT, STG, SMALL>(p, sh, tb, stg, K);
  } else if (SMALL && wid < FENVW && wid >= p.faw) {
    fused_idle<OK, QPT>(p, sh, tb, K);
  } else if (wid > FENVW) {
    // above the env waves: the store waves issue their few copy instructions right after B2 instead of
    // trailing the VALU-bound transitions on their SIMD (+6% measured vs priority 0; 2 was no better)
    __builtin_amdgcn_s_setprio(GP_STORE_PRIO);
    fused_store<OK, QPT, STG, SMALL>(p, sh, tb, stg, K, obs, rew, term, trunc);
  } else {
    fused_env<OK, QPT, NA, STG, SMALL>(p, sh, s_thr, tb, stg, K, act, obs, rew, term, trunc, rsum, eps, lens, nst);
  }
  LSTAMP(2);
  // metrics (the control wave contributes zeros)
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    rsum += __shfl_xor(rsum, d, 64);
    eps += __shfl_xor(eps, d, 64);
    lens += __shfl_xor(lens, d, 64);
    nst += __shfl_xor(nst, d, 64);
  }
  __shared__ float m_r[FWAVES];
  __shared__ uint32_t m_e[FWAVES], m_l[FWAVES], m_n[FWAVES];
  if (lane == 0) { m_r[wid] = rsum; m_e[wid] = eps; m_l[wid] = lens; m_n[wid] = nst; }
  __syncthreads();
  if (tid == 0) {
    float rr = 0; uint32_t e = 0, l = 0, n = 0;
    for (int w = 0; w < FWAVES; ++w) { rr += m_r[w]; e += m_e[w]; l += m_l[w]; n += m_n[w]; }
    // this block's own slot: fire-and-forget adds (a load-modify-store put two memory round trips on
    // the end of every launch)
    MetricSlot& m = p.mslot[blockIdx.x];
    atomicAdd(&m.return_sum, (double)rr);
    atomicAdd(&m.episodes, (unsigned long long)e);
    atomicAdd(&m.length_sum, (unsigned long long)l);
    atomicAdd(&m.env_steps, (unsigned long long)n);
  }
  LSTAMP(3);
}

// ------------------------------------------------------------------ kernels: counter modes ----
// Philox: ctr = (env, step_lo, step_hi, 0x67706f21), key = seed-derived. One draw set per
// env-step: x0,x1 -> 53-bit uniform; x2 -> goal index; x3 -> agent index (multiply-shift).
// The global step index is host-tracked and passed by value.
__device__ __forceinline__ void philox_draws(const GridDev& p, int env, uint64_t step, uint64_t& k53, uint32_t& gi,
                                             uint32_t& ai) {
  Philox4 r = philox4x32_10((uint32_t)env, (uint32_t)step, (uint32_t)(step >> 32), 0x67706f21u, p.key0, p.key1);
  k53 = ((((uint64_t)r.x[0]) << 32) | r.x[1]) >> 11;
  gi = lemire_value(r.x[2], (uint32_t)max(p.n_goal_valid, 1));
  ai = lemire_value(r.x[3], (uint32_t)max(p.n_agent_valid, 1));
}

template <int OK, class TB>
__device__ __forceinline__ void counter_env_step(const GridDev& p, const TB& tb, const uint64_t* thr, uint32_t& ae,
                                                 int& goal, int a, uint64_t k53, uint32_t gi, uint32_t ai, float& r,
                                                 uint8_t& tm, uint8_t& tr, float& rsum, uint32_t& eps,
                                                 uint32_t& lens) {
  Trans t = transition(p, tb, ae, goal, a, k53, thr);
  int agent = t.agent, g = goal, el = t.elapsed;
  rsum += t.rew;
  if (t.term | t.trunc) {
    eps += 1;
    lens += (uint32_t)el;
    el = 0;
    g = p.fixed_goal >= 0 ? p.fixed_goal : (int)tb.gv((int)gi);
    agent = p.fixed_agent >= 0 ? p.fixed_agent : (int)tb.av((int)ai);
  }
  ae = (uint32_t)agent | ((uint32_t)el << 16);
  goal = g;
  r = t.rew;
  tm = t.term;
  tr = t.trunc;
}

template <bool LT>
__device__ __forceinline__ auto make_tabs(const GridDev& p, const char* dyn) {
  if constexpr (LT) return LTabs{p, dyn};
  else return GTabs{p};
}

// LT: the lookup tables staged in LDS (K-step rollouts, when they fit) instead of read through the caches.
template <int OK, bool REPLAY, bool LT = false>
__global__ __launch_bounds__(TPB) void grid_rollout_counter(GridDev p, int K, uint64_t step0,
                                                            const int32_t* __restrict__ act, void* __restrict__ obs,
                                                            float* __restrict__ rew, uint8_t* __restrict__ term,
                                                            uint8_t* __restrict__ trunc) {
  __shared__ uint64_t s_thr[64];
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  if (threadIdx.x < p.nact * p.nact) s_thr[threadIdx.x] = p.thr[threadIdx.x];
  if constexpr (LT) lds_image_copy(dyn, p.limg, p.lds.jt.off);  // all but the PCG jump tables (last)
  __syncthreads();
  const auto tb = make_tabs<LT>(p, dyn);
  const int env0 = blockIdx.x * EPB + threadIdx.x * EPT;
  uint32_t ae4[4];
  load4<uint32_t>(p.ae, env0, p.B, ae4);
  int g4[4];
  if (p.fixed_goal < 0) {
    uint16_t gg[4];
    load4<uint16_t>(p.goal, env0, p.B, gg);
#pragma unroll
    for (int i = 0; i < 4; ++i) g4[i] = gg[i];
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) g4[i] = p.fixed_goal;
  }
  float rsum = 0.f;
  uint32_t eps = 0, lens = 0, nst = 0;
  const size_t ow = (size_t)p.obs_width * ((OK == GP_OBS_HANSEN_VEC || OK == GP_OBS_WINDOW) ? 1 : 4);
  for (int k = 0; k < K; ++k) {
    const size_t off = (size_t)k * p.B;
    int32_t a4[4];
    load4<int32_t>(act + off, env0, p.B, a4);
    float r[4];
    uint8_t tm[4], tr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int env = env0 + i;
      uint64_t k53 = 0;
      uint32_t gi = 0, ai = 0;
      if (env < p.B) {
        if constexpr (REPLAY) {
          k53 = p.rp_u[env];
          gi = p.rp_goal ? (uint32_t)p.rp_goal[env] : 0u;
          ai = p.rp_agent ? (uint32_t)p.rp_agent[env] : 0u;
        } else {
          philox_draws(p, env, step0 + k, k53, gi, ai);
        }
      }
      counter_env_step<OK>(p, tb, s_thr, ae4[i], g4[i], a4[i], k53, gi, ai, r[i], tm[i], tr[i], rsum, eps, lens);
      nst += env < p.B;
    }
    store4<float>(rew + off, env0, p.B, r);
    store4<uint8_t>(term + off, env0, p.B, tm);
    store4<uint8_t>(trunc + off, env0, p.B, tr);
    int ag[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ag[i] = (int)(ae4[i] & 0xFFFF);
    write_obs4<OK>(p, tb, env0, ag, g4, (uint8_t*)obs + (size_t)k * p.B * ow);
  }
  store4<uint32_t>(p.ae, env0, p.B, ae4);
  if (p.fixed_goal < 0) {
    uint16_t gg[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) gg[i] = (uint16_t)g4[i];
    store4<uint16_t>(p.goal, env0, p.B, gg);
  }
  add_metrics(p, rsum, eps, lens, nst);
}

// Philox / replay reset: every env draws goal then agent from its own counter.
template <int OK, bool REPLAY>
__global__ __launch_bounds__(TPB) void grid_reset_counter(GridDev p, uint64_t step, void* __restrict__ obs) {
  const int env = blockIdx.x * TPB + threadIdx.x;
  if (env >= p.B) return;
  uint64_t k53;
  uint32_t gi = 0, ai = 0;
  if constexpr (REPLAY) {
    gi = p.rp_goal ? (uint32_t)p.rp_goal[env] : 0u;
    ai = p.rp_agent ? (uint32_t)p.rp_agent[env] : 0u;
  } else {
    philox_draws(p, env, step, k53, gi, ai);
  }
  const int g = p.fixed_goal >= 0 ? p.fixed_goal : (int)p.goal_valid[gi];
  const int a = p.fixed_agent >= 0 ? p.fixed_agent : (int)p.agent_valid[ai];
  p.ae[env] = (uint32_t)a;
  if (p.fixed_goal < 0) p.goal[env] = (uint16_t)g;
  write_obs<OK>(p, GTabs{p}, env, a, g, obs);
}

// ------------------------------------------------------------------ state access ----
__global__ void grid_get_state(GridDev p, int32_t* agent, int32_t* goal, int32_t* elapsed) {
  const int env = blockIdx.x * TPB + threadIdx.x;
  if (env >= p.B) return;
  const uint32_t ae = p.ae[env];
  if (agent) agent[env] = (int32_t)(ae & 0xFFFF);
  if (elapsed) elapsed[env] = (int32_t)(ae >> 16);
  if (goal) goal[env] = p.fixed_goal >= 0 ? p.fixed_goal : (int32_t)p.goal[env];
}
__global__ void grid_set_state(GridDev p, const int32_t* agent, const int32_t* goal, const int32_t* elapsed) {
  const int env = blockIdx.x * TPB + threadIdx.x;
  if (env >= p.B) return;
  uint32_t ae = p.ae[env];
  if (agent) ae = (ae & 0xFFFF0000u) | (uint32_t)min(max(agent[env], 0), p.ncells - 1);
  if (elapsed) ae = (ae & 0xFFFFu) | ((uint32_t)min(max(elapsed[env], 0), 65535) << 16);
  p.ae[env] = ae;
  if (goal && p.fixed_goal < 0) p.goal[env] = (uint16_t)min(max(goal[env], 0), p.ncells - 1);
}

// ------------------------------------------------------------------ host backend ----
struct GridBackend : EnvBackend {
  GridDev d{};
  int flavor = 0;
  int depth = 1, height = 0, width = 0;
  int grid_persist = 1;        // resident blocks of the persistent numpy-mode kernels
  int nslots = 1;              // metric slots (max grid size of any kernel writing them)
  uint64_t philox_step = 0;    // host-tracked global step for the counter-based mode
  std::vector<int32_t> cells;
  std::vector<uint16_t> goal_valid_h, agent_valid_h;
  DevBuf b_move, b_thr, b_gv, b_av, b_hbase, b_doff, b_hvec, b_t1, b_t2, b_coords, b_window, b_jt, b_lt4, b_lt2,
      b_tja, b_tjw, b_ae, b_goal, b_ctl, b_tcount, b_tlist, b_rflag, b_mslot, b_ftj, b_flt4, b_fjB, b_fslot, b_dbg, b_self, b_jt8,
      b_limg, b_ofix, b_avo;
  int fused_G = 0, fused_qpt = 0;  // fused numpy rollout geometry (0 = not eligible)
  // windowed numpy rollout (wgrid.hip): G blocks of E = 512 * NS envs; 0 = not eligible
  int wg_G = 0, wg_E = 0, wg_NS = 0, wg_H = 0;
  int wg_kmax = WG_KMAX;  // launches of more steps go to the fused kernel when it can take them (gp_debug_set wg_kmax)
  int wg_kmax_default = WG_KMAX;  // the size-based choice before any autotune (the autotune's margin favours it)
  size_t wg_lds = 0;
  int at_launches = 0, at_steps = 0;  // the last gp_autotune's scratch launches (both kernels) and their length
  float at_ms[2] = {0.f, 0.f};        // its mean ms per launch: windowed, fused
  WgParams wg{};
  std::vector<char> wg_img;        // LDS image of its tables (the PCG jump parts rebuilt on every seed)
  DevBuf b_wgp, b_wlimg, b_wjlane, b_wjrej, b_wjblk, b_wslots, b_wjfirst;
  bool fused_stg = false;          // outputs staged in LDS and written by the store waves
  // replay pointers for the next step
  const uint64_t* rp_u = nullptr;
  const int32_t* rp_goal = nullptr;
  const int32_t* rp_agent = nullptr;

  int build(const gp_grid_config* cfg);
  int upload_rng();
  int refresh_lds_image();
  int seed(const RngHost& r, const uint32_t key[2]) override {
    rng = r;
    philox_key[0] = key[0];
    philox_key[1] = key[1];
    d.key0 = key[0];
    d.key1 = key[1];
    philox_step = 0;
    return upload_rng();
  }
  int set_rng_state(const RngHost& r) override {
    rng = r;
    return upload_rng();
  }
  int get_rng_state(RngHost* r) override;
  int check() override;
  int device_error(uint32_t flags);
  int query(const char* key, int64_t* v) const override {
    if (!strcmp(key, "fused_blocks")) *v = fused_G;
    else if (!strcmp(key, "fused_tiles_per_block")) *v = fused_qpt;
    else if (!strcmp(key, "fused_staged")) *v = fused_stg ? 1 : 0;
    else if (!strcmp(key, "fused_spw")) *v = d.spw_on;
    else if (!strcmp(key, "fused_tile_envs")) *v = d.ftile;
    else if (!strcmp(key, "wgrid")) *v = wg_G > 0 ? 1 : 0;
    else if (!strcmp(key, "wgrid_blocks")) *v = wg_G;
    else if (!strcmp(key, "wgrid_block_envs")) *v = wg_E;
    else if (!strcmp(key, "wgrid_halo")) *v = wg_H;
    else if (!strcmp(key, "wgrid_kmax")) *v = wg_kmax;
    else if (!strcmp(key, "wgrid_lds")) *v = (int64_t)wg_lds;  // dynamic LDS bytes of one launch
    // the last autotune: launches it made (both kernels, incl. one warm launch each), their length, and the mean
    // time per launch of each kernel in ns
    else if (!strcmp(key, "autotune_launches")) *v = at_launches;
    else if (!strcmp(key, "autotune_steps")) *v = at_steps;
    else if (!strcmp(key, "autotune_wgrid_ns")) *v = (int64_t)(at_ms[0] * 1e6f);
    else if (!strcmp(key, "autotune_fused_ns")) *v = (int64_t)(at_ms[1] * 1e6f);
    else return EnvBackend::query(key, v);
    return GP_OK;
  }
  int reset(void* obs, hipStream_t s) override;
  int step(const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) override;
  int rollout(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) override;
  int get_state(void* a, void* b, void* c, void* dd, hipStream_t s) override {
    hipLaunchKernelGGL(grid_get_state, dim3((unsigned)((B + TPB - 1) / TPB)), dim3(TPB), 0, s, d, (int32_t*)a,
                       (int32_t*)b, (int32_t*)c);
    GP_HIP_CHECK(hipGetLastError());
    return GP_OK;
  }
  int set_state(const void* a, const void* b, const void* c, const void* dd, hipStream_t s) override {
    hipLaunchKernelGGL(grid_set_state, dim3((unsigned)((B + TPB - 1) / TPB)), dim3(TPB), 0, s, d,
                       (const int32_t*)a, (const int32_t*)b, (const int32_t*)c);
    GP_HIP_CHECK(hipGetLastError());
    has_reset = true;
    return GP_OK;
  }
  int set_replay(const void* u, const void* i0, const void* i1, const void* f0, const void* f1) override {
    if (rng_mode != GP_RNG_REPLAY) {
      gp_set_error("gp_set_replay requires GP_RNG_REPLAY");
      return GP_E_STATE;
    }
    rp_u = (const uint64_t*)u;
    rp_goal = (const int32_t*)i0;
    rp_agent = (const int32_t*)i1;
    return GP_OK;
  }
  int valid_cells(int which, int32_t* out, int cap) const override {
    const std::vector<uint16_t>& v = which == 0 ? goal_valid_h : agent_valid_h;
    for (int i = 0; i < (int)v.size() && i < cap; ++i) out[i] = v[i];
    return (int)v.size();
  }
  int metrics(double out[4]) override;
  int autotune(int K, int reps, int* chosen) override;
#ifdef GP_STAMPS
  int debug_stamps(unsigned long long* out, int cap) override {
    GP_HIP_CHECK(hipDeviceSynchronize());
    const int n = std::min(cap, 256 * 64 * 16 + 256 * 8);
    GP_HIP_CHECK(hipMemcpy(out, d.dbg, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost));
    return n;
  }
#endif
  // the windowed kernel's 16-B output stores need 16-B aligned bases (torch allocations are)
  bool wgrid_ok(const void* act, const void* obs, const void* rew, const void* term, const void* trunc) const {
    auto al = [](const void* x, uintptr_t m) { return ((uintptr_t)x & (m - 1)) == 0; };
    return wg_G && al(act, 4) && al(obs, 16) && al(rew, 16) && al(term, 16) && al(trunc, 16);
  }
  // The windowed kernel for launches of up to wg_kmax steps, the fused kernel (same stream, same state) for longer
  // ones when it can take them.
  bool wgrid_pick(int K, const void* act, const void* obs, const void* rew, const void* term, const void* trunc) const {
    if (!wgrid_ok(act, obs, rew, term, trunc)) return false;
    return K <= wg_kmax || !(fused_ok(act, obs, rew, term, trunc) && B % 4 == 0);
  }
  int launch_wgrid(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) {
    const WgArgs a{b_wgp.as<WgParams>(), K, (const int32_t*)act, (int32_t*)obs, rew, term, trunc};
    timer.begin(s);
    const int e = wgrid_launch(a, wg_NS, d.nact, wg_G, wg_lds, s);
    timer.end(s);
    if (e != hipSuccess) {
      gp_set_error("wgrid launch: %s", hipGetErrorString((hipError_t)e));
      return GP_E_HIP;
    }
    return GP_OK;
  }
  int build_wgrid(const std::vector<uint16_t>& move, const std::vector<uint64_t>& thr, const std::vector<int32_t>& ocell);
  int upload_wgrid();
  template <int OK, int QPT, bool STG>
  void launch_fused_qs(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) {
    const size_t lds = (size_t)d.lds.total +
                       (STG ? (size_t)QPT * STG_TILE_BYTES + (d.spw_on ? (size_t)spw_bytes(QPT) : 0) : 0);
    // SMALL: tiles of 512 / 1024 envs (runtime size, idle env waves); only with <= 2 tiles per block
    if constexpr (QPT <= 2) {
      if (d.ftile != FEPB) {
        if (d.nact == 4)
          hipLaunchKernelGGL((grid_rollout_numpy<OK, QPT, 4, STG, true>), dim3(fused_G), dim3(FTPB), lds, s, d, K,
                             (const int32_t*)act, obs, rew, term, trunc);
        else
          hipLaunchKernelGGL((grid_rollout_numpy<OK, QPT, 8, STG, true>), dim3(fused_G), dim3(FTPB), lds, s, d, K,
                             (const int32_t*)act, obs, rew, term, trunc);
        return;
      }
    }
    if (d.nact == 4)
      hipLaunchKernelGGL((grid_rollout_numpy<OK, QPT, 4, STG, false>), dim3(fused_G), dim3(FTPB), lds, s, d, K,
                         (const int32_t*)act, obs, rew, term, trunc);
    else
      hipLaunchKernelGGL((grid_rollout_numpy<OK, QPT, 8, STG, false>), dim3(fused_G), dim3(FTPB), lds, s, d, K,
                         (const int32_t*)act, obs, rew, term, trunc);
  }
  template <int OK, int QPT>
  void launch_fused_q(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) {
    if constexpr (fused_staged<OK, QPT>()) {
      if (fused_stg) return launch_fused_qs<OK, QPT, true>(K, act, obs, rew, term, trunc, s);
    }
    launch_fused_qs<OK, QPT, false>(K, act, obs, rew, term, trunc, s);
  }
  // the fused kernel's vector I/O assumes 16-B aligned bases (torch allocations are); K-step launches
  // also need B % 4 == 0 so that every step's slice stays aligned
  bool fused_ok(const void* act, const void* obs, const void* rew, const void* term, const void* trunc) const {
    auto al = [](const void* x, uintptr_t m) { return ((uintptr_t)x & (m - 1)) == 0; };
    return fused_G && al(act, 16) && al(obs, 16) && al(rew, 16) && al(term, 4) && al(trunc, 4);
  }
  template <int OK>
  int launch_fused(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) {
    timer.begin(s);
    switch (fused_qpt) {
      case 1: launch_fused_q<OK, 1>(K, act, obs, rew, term, trunc, s); break;
      case 2: launch_fused_q<OK, 2>(K, act, obs, rew, term, trunc, s); break;
      default: launch_fused_q<OK, 4>(K, act, obs, rew, term, trunc, s);
    }
    timer.end(s);
    GP_HIP_CHECK(hipGetLastError());
    return GP_OK;
  }
};

int GridBackend::upload_rng() {
  GP_HIP_CHECK(hipDeviceSynchronize());
  if (d.self) GP_HIP_CHECK(hipMemcpy(const_cast<GridDev*>(d.self), &d, sizeof(GridDev), hipMemcpyHostToDevice));
  GridCtl c;
  GP_HIP_CHECK(hipMemcpy(&c, d.ctl, sizeof(c), hipMemcpyDeviceToHost));
  c.s_hi = hi64(rng.state);
  c.s_lo = lo64(rng.state);
  c.inc_hi = hi64(rng.inc);
  c.inc_lo = lo64(rng.inc);
  c.has_u32 = rng.has_u32;
  c.uinteger = rng.uinteger;
  c.err = 0;  // a new stream position: earlier device errors no longer apply
  // test knob: start the fused kernel's tag counter here (tests cross its 8192-step tag wrap without 8192 steps)
  if (gp_debug_knobs().fused_step >= 0) c.step = (uint32_t)gp_debug_knobs().fused_step;
  GP_HIP_CHECK(hipMemcpy(d.ctl, &c, sizeof(c), hipMemcpyHostToDevice));
  std::vector<PcgJump> jt = build_jump_tables(rng.inc);
  GP_HIP_CHECK(hipMemcpy(b_jt.p, jt.data(), jt.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
  if (b_jt8.p) {
    std::vector<PcgJump> j8(2 * 256);
    for (int dgt = 0; dgt < 256; ++dgt) {
      j8[dgt] = pcg_jump_params((u128)dgt, rng.inc);
      j8[256 + dgt] = pcg_jump_params((u128)(256 * dgt), rng.inc);
    }
    GP_HIP_CHECK(hipMemcpy(b_jt8.p, j8.data(), j8.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
  }
  std::vector<PcgJump> l4(TPB), l2(TPB);
  for (int t = 0; t < TPB; ++t) {
    l4[t] = pcg_jump_params((u128)(4 * t), rng.inc);
    l2[t] = pcg_jump_params((u128)(2 * t), rng.inc);
  }
  GP_HIP_CHECK(hipMemcpy(b_lt4.p, l4.data(), l4.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
  GP_HIP_CHECK(hipMemcpy(b_lt2.p, l2.data(), l2.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
  // per-tile bases: tja[k] = jump(k*EPB + 1), tjw[k] = jump(B + k*EPB/2), built by composition
  std::vector<PcgJump> ta(d.nblk), tw(d.nblk);
  const PcgJump step_tile = pcg_jump_params((u128)EPB, rng.inc), step_half = pcg_jump_params((u128)(EPB / 2), rng.inc);
  auto compose = [](const PcgJump& j2, const PcgJump& j1) {  // j2 o j1
    const u128 a = mk128(j2.a_hi, j2.a_lo) * mk128(j1.a_hi, j1.a_lo);
    const u128 c = mk128(j2.a_hi, j2.a_lo) * mk128(j1.c_hi, j1.c_lo) + mk128(j2.c_hi, j2.c_lo);
    return PcgJump{hi64(a), lo64(a), hi64(c), lo64(c)};
  };
  ta[0] = pcg_jump_params((u128)1, rng.inc);
  tw[0] = pcg_jump_params((u128)B, rng.inc);
  for (int k = 1; k < d.nblk; ++k) {
    ta[k] = compose(step_tile, ta[k - 1]);
    tw[k] = compose(step_half, tw[k - 1]);
  }
  GP_HIP_CHECK(hipMemcpy(b_tja.p, ta.data(), ta.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
  GP_HIP_CHECK(hipMemcpy(b_tjw.p, tw.data(), tw.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
  if (fused_G) {
    std::vector<PcgJump> fl(FTPB), ft(d.fnt);
    for (int t = 0; t < FTPB; ++t) fl[t] = pcg_jump_params((u128)(4 * t), rng.inc);
    const PcgJump step_ftile = pcg_jump_params((u128)d.ftile, rng.inc);
    ft[0] = pcg_jump_params((u128)1, rng.inc);
    for (int k = 1; k < d.fnt; ++k) ft[k] = compose(step_ftile, ft[k - 1]);
    const PcgJump jb[2] = {pcg_jump_params((u128)B, rng.inc),                   // random(B)
                           pcg_jump_params((u128)fused_G * d.ftile, rng.inc)};  // tile stride of a block (q -> q + 1)
    GP_HIP_CHECK(hipMemcpy(b_flt4.p, fl.data(), fl.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
    GP_HIP_CHECK(hipMemcpy(b_ftj.p, ft.data(), ft.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
    GP_HIP_CHECK(hipMemcpy(b_fjB.p, jb, sizeof(jb), hipMemcpyHostToDevice));
  }
  if (wg_G) {
    int e = upload_wgrid();
    if (e) return e;
  }
  return refresh_lds_image();
}

// The LDS table image (GridDev::limg): every staged table copied to its LDS offset, so that a kernel stages
// them all with one copy loop. The PCG jump tables depend on the stream increment: rebuilt on every seed.
int GridBackend::refresh_lds_image() {
  if (!b_limg.p || d.lds.total <= 0) return GP_OK;
  char* img = b_limg.as<char>();
  auto put = [&](const GridLdsTab& t, const void* src) -> int {
    if (t.bytes > 0 && src) GP_HIP_CHECK(hipMemcpy(img + t.off, src, (size_t)t.bytes, hipMemcpyDeviceToDevice));
    return GP_OK;
  };
  int e;
  if ((e = put(d.lds.move, d.move)) || (e = put(d.lds.hbase, d.hbase)) || (e = put(d.lds.hvec, d.hvec)) ||
      (e = put(d.lds.t1, d.t1)) || (e = put(d.lds.t2, d.t2)) || (e = put(d.lds.coords, d.coords)) ||
      (e = put(d.lds.window, d.window)) || (e = put(d.lds.gv, d.goal_valid)) || (e = put(d.lds.av, d.agent_valid)) ||
      (e = put(d.lds.doff, d.doff)) || (e = put(d.lds.jt, d.jt)) || (e = put(d.lds.jt8, d.jt8)) ||
      (e = put(d.lds.ofix, d.ofix)) || (e = put(d.lds.avo, d.avo)))
    return e;
  GP_HIP_CHECK(hipDeviceSynchronize());
  return GP_OK;
}

// The windowed kernel's geometry and static tables (eligibility already checked by build()). B must split into
// G <= #CUs blocks of E = 512 * NS envs (NS in 1, 2, 4, 8), the smallest E that does (so that every CU has a block).
int GridBackend::build_wgrid(const std::vector<uint16_t>& move, const std::vector<uint64_t>& thr,
                             const std::vector<int32_t>& ocell) {
  const GpDebugKnobs& dbg = gp_debug_knobs();
  hipDeviceProp_t prop;
  GP_HIP_CHECK(hipGetDeviceProperties(&prop, device));
  const int cus = std::min(prop.multiProcessorCount, 256);
  int E = 0;
  for (int e = 512; e <= 4096; e *= 2)
    if (B % e == 0 && B / e <= cus && (dbg.wg_block_envs <= 0 || e >= dbg.wg_block_envs)) {
      E = e;
      break;
    }
  if (!E) return GP_OK;  // not eligible: the older fused kernel serves this size
  for (int c : ocell)
    if (c < INT32_MIN / 2 || c > INT32_MAX / 2) return GP_OK;
  const int H = dbg.wg_halo == 512 ? 512 : 256;
  const int nc = d.ncells, na = d.nact;
  // LDS image: j32 | jt8 | move | thr | ocell | avalid, 16-B aligned pieces
  WgLds L{};
  int off = 0;
  auto put = [&](int32_t& o, size_t bytes) {
    o = off;
    off += (int)((bytes + 15) / 16 * 16);
  };
  put(L.j32, sizeof(PcgJump) * 32);
  put(L.jt8, sizeof(PcgJump) * 512);
  put(L.move, (size_t)nc * na * 2);
  put(L.thr, (size_t)na * na * 8);
  put(L.ocell, (size_t)nc * 4);
  put(L.avalid, agent_valid_h.size() * 2);
  L.total = off;
  const size_t lds = (size_t)wg_dyn_bytes(L.total, E, H);
  if (!wgrid_fits(E / 512, na, lds)) return GP_OK;
  wg_img.assign((size_t)L.total, 0);
  memcpy(wg_img.data() + L.move, move.data(), move.size() * 2);
  std::vector<uint64_t> th(thr.size());
  for (size_t i = 0; i < thr.size(); ++i) th[i] = thr_on_u64(thr[i]);
  memcpy(wg_img.data() + L.thr, th.data(), th.size() * 8);
  memcpy(wg_img.data() + L.ocell, ocell.data(), ocell.size() * 4);
  memcpy(wg_img.data() + L.avalid, agent_valid_h.data(), agent_valid_h.size() * 2);
  wg_G = (int)(B / E);
  wg_E = E;
  wg_NS = E / 512;
  wg_H = H;
  wg_lds = lds;
  WgParams& w = wg;
  w.B = (int32_t)B;
  w.G = wg_G;
  w.E = E;
  w.NS = wg_NS;
  w.nact = na;
  w.ncells = nc;
  w.n_agent = d.n_agent_valid;
  w.goal = d.fixed_goal;
  w.thr_agent = d.thr_agent;
  w.time_limit = d.time_limit;
  w.halo = H;
  w.r_step = d.r_step;
  w.r_wall = d.r_wall;
  w.r_goal = d.r_goal;
  w.spin_limit = d.spin_limit;
  w.fault_block = d.fault_block;
  w.rw_words = (E + 2 * H) / 64;
  {  // rows per env wave (waves v and v + 4 share SIMD v): base +- a per-SIMD delta d[v & 3] (knob wg_fill_simd: four
     // signed 4-bit deltas, SIMD 0 in the low nibble; they must sum to 0, else the rows stay even)
    const int base = w.rw_words / 8;
    const int code = dbg.wg_fill_simd != 0 ? dbg.wg_fill_simd : WG_FILL_SIMD;
    int dl[4], sum = 0;
    bool ok = true;
    for (int q = 0; q < 4; ++q) {
      dl[q] = ((code >> (4 * q)) & 15) >= 8 ? ((code >> (4 * q)) & 15) - 16 : ((code >> (4 * q)) & 15);
      sum += dl[q];
      ok = ok && base + dl[q] >= 1;
    }
    if (sum != 0 || !ok) dl[0] = dl[1] = dl[2] = dl[3] = 0;
    int dv[8];  // knob wg_fill_wave: per-wave deltas (eight signed nibbles, wave 0 lowest) on top, summing to 0
    int vsum = 0;
    bool vok = true;
    for (int v = 0; v < 8; ++v) {
      const int n = (int)(((uint32_t)(dbg.wg_fill_wave != 0 ? dbg.wg_fill_wave : WG_FILL_WAVE) >> (4 * v)) & 15u);
      dv[v] = n >= 8 ? n - 16 : n;
      vsum += dv[v];
      vok = vok && base + dl[v & 3] + dv[v] >= 1;
    }
    if (vsum != 0 || !vok)
      for (int v = 0; v < 8; ++v) dv[v] = 0;
    int r = 0;
    for (int v = 0; v < 8; ++v) {
      w.fill_row0[v] = r;
      w.fill_rows[v] = base + dl[v & 3] + dv[v];
      r += w.fill_rows[v];
    }
  }
  w.wg_bias = dbg.wg_bias;
  w.tmode = dbg.wg_tmode;
  w.lds = L;
  int e;
  if ((e = b_wgp.alloc(sizeof(WgParams))) || (e = b_wlimg.alloc((size_t)L.total)) ||
      (e = b_wjlane.alloc(sizeof(PcgJump) * 1024)) || (e = b_wjrej.alloc(sizeof(PcgJump) * 64 * (size_t)wg_G)) ||
      (e = b_wjblk.alloc(sizeof(PcgJump) * 2 * (size_t)wg_G)) || (e = b_wslots.alloc(sizeof(uint64_t) * 4 * (size_t)wg_G)) ||
      (e = b_wjfirst.alloc(sizeof(PcgJump) * 1024)))
    return e;
  w.jfirst = b_wjfirst.as<PcgJump>();
  w.limg = b_wlimg.as<char>();
  w.jlane = b_wjlane.as<PcgJump>();
  w.jrej = b_wjrej.as<PcgJump>();
  w.jblk = b_wjblk.as<PcgJump>();
  w.slots = b_wslots.as<uint64_t>();
  return GP_OK;
}

// The stream-dependent parts of the windowed kernel's tables (every seed: they depend on the PCG increment).
int GridBackend::upload_wgrid() {
  const u128 inc = rng.inc;
  WgParams& w = wg;
  auto compose = [](const PcgJump& j2, const PcgJump& j1) {  // j2 o j1
    const u128 a = mk128(j2.a_hi, j2.a_lo) * mk128(j1.a_hi, j1.a_lo);
    const u128 c = mk128(j2.a_hi, j2.a_lo) * mk128(j1.c_hi, j1.c_lo) + mk128(j2.c_hi, j2.c_lo);
    return PcgJump{hi64(a), lo64(a), hi64(c), lo64(c)};
  };
  PcgJump* j32 = reinterpret_cast<PcgJump*>(wg_img.data() + w.lds.j32);
  PcgJump* jt8 = reinterpret_cast<PcgJump*>(wg_img.data() + w.lds.jt8);
  for (int i = 0; i < 32; ++i) j32[i] = pcg_jump_params((u128)i, inc);
  for (int i = 0; i < 256; ++i) {
    jt8[i] = pcg_jump_params((u128)i, inc);
    jt8[256 + i] = pcg_jump_params((u128)(256 * i), inc);
  }
  std::vector<PcgJump> jl(1024), jr((size_t)64 * wg_G), jb(2 * (size_t)wg_G);
  const PcgJump one = pcg_jump_params((u128)1, inc), j32s = pcg_jump_params((u128)32, inc);
  const PcgJump jBp1 = pcg_jump_params((u128)B + 1, inc);  // B + 1
  jl[1] = jBp1;
  for (int l = 1; l < 512; ++l) jl[2 * l + 1] = compose(j32s, jl[2 * (l - 1) + 1]);  // B + 32 lg + 1
  for (int v = 0; v < 8; ++v) {  // 64 fill_row0[v] + lane
    PcgJump x = pcg_jump_params((u128)(64 * w.fill_row0[v]), inc);
    for (int l = 0; l < 64; ++l) {
      jl[2 * (64 * v + l)] = x;
      x = compose(one, x);
    }
  }
  const PcgJump j62 = pcg_jump_params((u128)62, inc);
  PcgJump row = jBp1;  // B + 62 beta + 1
  for (int b = 0; b < wg_G; ++b) {
    PcgJump x = row;
    for (int l = 0; l < 64; ++l) {
      jr[(size_t)b * 64 + l] = x;
      x = compose(one, x);
    }
    row = compose(j62, row);
    jb[2 * b] = pcg_jump_params((u128)B + (u128)(b ? wg_E * b - wg_H : 0), inc);
    jb[2 * b + 1] = b ? pcg_jump_params((u128)(wg_E * b - wg_H + 1), inc) : PcgJump{0, 1, 0, 0};
  }
  w.jB = pcg_jump_params((u128)B, inc);
  w.jrow = pcg_jump_params((u128)64, inc);
  w.j512 = pcg_jump_params((u128)512, inc);
  std::vector<PcgJump> jf(1024);
  jf[0] = one;                                    // block 0: 1 + lg
  jf[512] = pcg_jump_params((u128)wg_H, inc);     // blocks > 0: H + lg
  for (int l = 1; l < 512; ++l) {
    jf[l] = compose(one, jf[l - 1]);
    jf[512 + l] = compose(one, jf[512 + l - 1]);
  }
  w.jt64 = d.jt;
  w.dbg = d.dbg;
  w.ctl = d.ctl;
  w.mslot = d.mslot;
  w.ae = d.ae;
  GP_HIP_CHECK(hipMemcpy(b_wlimg.p, wg_img.data(), wg_img.size(), hipMemcpyHostToDevice));
  GP_HIP_CHECK(hipMemcpy(b_wjlane.p, jl.data(), jl.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
  GP_HIP_CHECK(hipMemcpy(b_wjrej.p, jr.data(), jr.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
  GP_HIP_CHECK(hipMemcpy(b_wjblk.p, jb.data(), jb.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
  GP_HIP_CHECK(hipMemcpy(b_wjfirst.p, jf.data(), jf.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
  GP_HIP_CHECK(hipMemcpy(b_wgp.p, &w, sizeof(WgParams), hipMemcpyHostToDevice));
  return GP_OK;
}

int GridBackend::get_rng_state(RngHost* r) {
  GP_HIP_CHECK(hipDeviceSynchronize());
  GridCtl c;
  GP_HIP_CHECK(hipMemcpy(&c, d.ctl, sizeof(c), hipMemcpyDeviceToHost));
  r->state = mk128(c.s_hi, c.s_lo);
  r->inc = mk128(c.inc_hi, c.inc_lo);
  r->has_u32 = c.has_u32;
  r->uinteger = c.uinteger;
  if (c.err) return device_error(c.err);
  return GP_OK;
}

int GridBackend::device_error(uint32_t flags) {
  gp_set_error("device error flags 0x%x: %sthe outputs and env state since the last seed are invalid (reseed to clear)",
               flags, gp_derr_text(flags));
  return GP_E_DEVICE;
}

int GridBackend::check() {
  GP_HIP_CHECK(hipDeviceSynchronize());
  uint32_t err = 0;
  GP_HIP_CHECK(hipMemcpy(&err, &d.ctl->err, sizeof(err), hipMemcpyDeviceToHost));
  return err ? device_error(err) : GP_OK;
}

int GridBackend::metrics(double out[4]) {
  GP_HIP_CHECK(hipDeviceSynchronize());
  std::vector<MetricSlot> m(nslots);
  GP_HIP_CHECK(hipMemcpy(m.data(), d.mslot, sizeof(MetricSlot) * nslots, hipMemcpyDeviceToHost));
  out[0] = out[1] = out[2] = out[3] = 0;
  for (const MetricSlot& x : m) {
    out[0] += (double)x.episodes;
    out[1] += x.return_sum;
    out[2] += (double)x.length_sum;
    out[3] += (double)x.env_steps;
  }
  return check();
}

template <class F>
static int dispatch_obs(int ok, F&& f) {
  switch (ok) {
    case GP_OBS_HANSEN: return f(std::integral_constant<int, GP_OBS_HANSEN>());
    case GP_OBS_HANSEN_VEC: return f(std::integral_constant<int, GP_OBS_HANSEN_VEC>());
    case GP_OBS_TABLE: return f(std::integral_constant<int, GP_OBS_TABLE>());
    case GP_OBS_COORDS: return f(std::integral_constant<int, GP_OBS_COORDS>());
    case GP_OBS_WINDOW: return f(std::integral_constant<int, GP_OBS_WINDOW>());
  }
  gp_set_error("bad obs kind %d", ok);
  return GP_E_INVALID;
}

int GridBackend::reset(void* obs, hipStream_t s) {
  GP_HIP_CHECK(hipMemsetAsync(d.mslot, 0, sizeof(MetricSlot) * nslots, s));
  const unsigned g1 = (unsigned)((B + TPB - 1) / TPB);
  const bool rgoal = d.fixed_goal < 0, ragent = d.fixed_agent < 0;
  const unsigned gp = (unsigned)grid_persist;
  int e = dispatch_obs(d.obs_kind, [&](auto okc) -> int {
    constexpr int OK = decltype(okc)::value;
    if (rng_mode == GP_RNG_NUMPY) {
      hipLaunchKernelGGL(grid_reset_init, dim3(g1), dim3(TPB), 0, s, d);
      hipLaunchKernelGGL(grid_resolve_numpy<OK>, dim3(gp), dim3(TPB), 0, s, d, obs, RM_RESET, 0u);
    } else if (rng_mode == GP_RNG_PHILOX) {
      hipLaunchKernelGGL((grid_reset_counter<OK, false>), dim3(g1), dim3(TPB), 0, s, d, philox_step, obs);
      ++philox_step;
    } else {
      GridDev dd = d;
      dd.rp_u = rp_u; dd.rp_goal = rp_goal; dd.rp_agent = rp_agent;
      if ((rgoal && !rp_goal) || (ragent && !rp_agent)) {
        gp_set_error("replay reset needs goal/agent index draws (gp_set_replay)");
        return GP_E_STATE;
      }
      hipLaunchKernelGGL((grid_reset_counter<OK, true>), dim3(g1), dim3(TPB), 0, s, dd, (uint64_t)0, obs);
    }
    return GP_OK;
  });
  if (e) return e;
  GP_HIP_CHECK(hipGetLastError());
  has_reset = true;
  return GP_OK;
}

int GridBackend::step(const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) {
  if (!has_reset) {
    gp_set_error("step() before reset()");
    return GP_E_STATE;
  }
  const bool rgoal = d.fixed_goal < 0, ragent = d.fixed_agent < 0;
  const unsigned gp = (unsigned)grid_persist;
  int e = dispatch_obs(d.obs_kind, [&](auto okc) -> int {
    constexpr int OK = decltype(okc)::value;
    if (rng_mode == GP_RNG_NUMPY) {
      if (wgrid_pick(1, act, obs, rew, term, trunc)) return launch_wgrid(1, act, obs, rew, term, trunc, s);
      if (fused_ok(act, obs, rew, term, trunc)) return launch_fused<OK>(1, act, obs, rew, term, trunc, s);
      timer.begin(s);
      hipLaunchKernelGGL(grid_step_numpy<OK>, dim3(d.nblk), dim3(TPB), 0, s, d, (const int32_t*)act, obs, rew, term,
                         trunc);
      timer.end(s);
      timer2.begin(s);
      hipLaunchKernelGGL(grid_resolve_numpy<OK>, dim3(gp), dim3(TPB), 0, s, d, obs, 0, (uint32_t)B);
      timer2.end(s);
      // (the fused kernels' tags continue from GridCtl::step: the two-kernel path never touches their slots)
    } else if (rng_mode == GP_RNG_PHILOX) {
      timer.begin(s);
      hipLaunchKernelGGL((grid_rollout_counter<OK, false>), dim3(d.nblk), dim3(TPB), 0, s, d, 1, philox_step,
                         (const int32_t*)act, obs, rew, term, trunc);
      timer.end(s);
      ++philox_step;
    } else {
      if (!rp_u || (rgoal && !rp_goal) || (ragent && !rp_agent)) {
        gp_set_error("replay step needs draws (gp_set_replay)");
        return GP_E_STATE;
      }
      GridDev dd = d;
      dd.rp_u = rp_u; dd.rp_goal = rp_goal; dd.rp_agent = rp_agent;
      hipLaunchKernelGGL((grid_rollout_counter<OK, true>), dim3(d.nblk), dim3(TPB), 0, s, dd, 1, (uint64_t)0,
                         (const int32_t*)act, obs, rew, term, trunc);
    }
    return GP_OK;
  });
  if (e) return e;
  GP_HIP_CHECK(hipGetLastError());
  return GP_OK;
}

// Uniform random actions for gp_autotune's scratch launches (a hash of the index; any action mix will do).
__global__ void autotune_actions(int32_t* a, size_t n, int nact) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    a[i] = (int32_t)((x >> 32) % (uint64_t)nact);
  }
}

// Times `reps` K-step launches of the windowed and of the fused kernel on scratch actions / outputs, each from
// the handle's current state, which is restored exactly afterwards (agent cells + elapsed, the stream and the
// kernels' control block, the metric slots; both kernels' granule slots reset as allocated, to a tag neither
// kernel ever expects).
// Launches of K steps then go to the faster one (wg_kmax). Their results are identical; which one is faster at
// short launches differs between MI355X boards (profiles/r05_ab_kernel_by_K.txt).
int GridBackend::autotune(int K, int reps, int* chosen) {
  if (chosen) *chosen = -1;
  if (rng_mode != GP_RNG_NUMPY || !wg_G || !fused_G || B % 4 != 0 || K < 1) return GP_OK;
  if (!has_reset) {
    gp_set_error("autotune() before reset()");
    return GP_E_STATE;
  }
  reps = std::max(1, std::min(reps, 64));
  GP_HIP_CHECK(hipDeviceSynchronize());
  // The scratch launches are at most AT_KMAX steps long (the outputs of one launch are 14 B per env-step: 1.9 GB at
  // K = 128 and 2^20 envs). Longer launches are decided from AT_KMAX-step ones: per step both kernels are then in
  // their long-launch regime (profiles/r05_ab_kernel_by_K.txt).
  constexpr int AT_KMAX = 64;
  const int Kt = std::min(K, AT_KMAX);
  const size_t nb = (size_t)B, kb = (size_t)Kt * nb;
  {
    size_t fr = 0, tot = 0;
    GP_HIP_CHECK(hipMemGetInfo(&fr, &tot));
    const size_t need = 4 * nb + b_mslot.n + 14 * kb;
    if (need > fr / 10 * 9) {
      gp_set_error("autotune: %zu bytes of scratch (%d-step launches of %lld envs) exceed the free device memory (%zu)",
                   need, Kt, (long long)B, fr);
      return GP_E_INVALID;
    }
  }
  DevBuf s_ae, s_ms, a, o, r, t, u;
  GridCtl ctl_h;
  int e;
  if ((e = s_ae.alloc(4 * nb)) || (e = s_ms.alloc(b_mslot.n)) || (e = a.alloc(4 * kb)) || (e = o.alloc(4 * kb)) ||
      (e = r.alloc(4 * kb)) || (e = t.alloc(kb)) || (e = u.alloc(kb)))
    return e;
  GP_HIP_CHECK(hipMemcpy(s_ae.p, d.ae, 4 * nb, hipMemcpyDeviceToDevice));
  GP_HIP_CHECK(hipMemcpy(s_ms.p, d.mslot, b_mslot.n, hipMemcpyDeviceToDevice));
  GP_HIP_CHECK(hipMemcpy(&ctl_h, d.ctl, sizeof(GridCtl), hipMemcpyDeviceToHost));
  hipLaunchKernelGGL(autotune_actions, dim3(1024), dim3(256), 0, 0, a.as<int32_t>(), kb, d.nact);
  GP_HIP_CHECK(hipGetLastError());
  auto restore = [&]() -> int {
    GP_HIP_CHECK(hipDeviceSynchronize());
    GP_HIP_CHECK(hipMemcpy(d.ae, s_ae.p, 4 * nb, hipMemcpyDeviceToDevice));
    GP_HIP_CHECK(hipMemcpy(d.mslot, s_ms.p, b_mslot.n, hipMemcpyDeviceToDevice));
    GP_HIP_CHECK(hipMemcpy(d.ctl, &ctl_h, sizeof(GridCtl), hipMemcpyHostToDevice));
    GP_HIP_CHECK(hipMemset(b_wslots.p, 0, b_wslots.n));   // windowed tags are never 0
    GP_HIP_CHECK(hipMemset(b_fslot.p, 0xFF, b_fslot.n));  // fused tags are never 0x7FFF (as allocated)
    GP_HIP_CHECK(hipDeviceSynchronize());
    return GP_OK;
  };
  hipEvent_t e0, e1;
  GP_HIP_CHECK(hipEventCreate(&e0));
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    gp_set_error("autotune: hipEventCreate failed");
    return GP_E_HIP;
  }
  const bool timer_on = timer.on;  // (the scratch launches are not the caller's to profile)
  timer.on = false;
  float ms[2] = {0.f, 0.f};
  for (int c = 0; c < 2 && !e; ++c) {
    auto one = [&]() -> int {
      if (c == 0) return launch_wgrid(Kt, a.p, o.p, r.as<float>(), t.as<uint8_t>(), u.as<uint8_t>(), 0);
      return dispatch_obs(d.obs_kind, [&](auto okc) -> int {
        constexpr int OK = decltype(okc)::value;
        return launch_fused<OK>(Kt, a.p, o.p, r.as<float>(), t.as<uint8_t>(), u.as<uint8_t>(), 0);
      });
    };
    e = one();  // warm
    if (!e && hipEventRecord(e0, 0) != hipSuccess) e = GP_E_HIP;
    for (int i = 0; i < reps && !e; ++i) e = one();
    if (!e && (hipEventRecord(e1, 0) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
               hipEventElapsedTime(&ms[c], e0, e1) != hipSuccess))
      e = GP_E_HIP;
    if (int e2 = restore()) e = e ? e : e2;  // (also after a failed launch: the state is put back first)
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  timer.on = timer_on;
  if (e) return e;
  // A margin: the kernel the launch length picks by default (wg_kmax_default) is kept unless the other one is at least
  // AT_MARGIN faster (one of five driver-command runs picked the kernel that was slower there with no margin).
  constexpr float AT_MARGIN = 0.02f;
  const bool def_wgrid = K <= wg_kmax_default;
  const bool wgrid_faster = def_wgrid ? !(ms[1] < (1.f - AT_MARGIN) * ms[0]) : ms[0] < (1.f - AT_MARGIN) * ms[1];
  if (wgrid_faster) wg_kmax = std::max(wg_kmax, K);
  else wg_kmax = std::min(wg_kmax, K - 1);
  at_ms[0] = ms[0] / (float)reps;
  at_ms[1] = ms[1] / (float)reps;
  at_launches = 2 * (reps + 1);
  at_steps = Kt;
  if (chosen) *chosen = wgrid_faster ? 1 : 0;
  return check();
}

int GridBackend::rollout(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc,
                         hipStream_t s) {
  if (rng_mode == GP_RNG_NUMPY && wgrid_pick(K, act, obs, rew, term, trunc)) {
    if (!has_reset) {
      gp_set_error("rollout() before reset()");
      return GP_E_STATE;
    }
    return launch_wgrid(K, act, (int32_t*)obs, rew, term, trunc, s);
  }
  if (rng_mode == GP_RNG_NUMPY && fused_ok(act, obs, rew, term, trunc) && B % 4 == 0) {
    if (!has_reset) {
      gp_set_error("rollout() before reset()");
      return GP_E_STATE;
    }
    return dispatch_obs(d.obs_kind, [&](auto okc) -> int {
      constexpr int OK = decltype(okc)::value;
      return launch_fused<OK>(K, act, obs, rew, term, trunc, s);
    });
  }
  if (rng_mode != GP_RNG_PHILOX) return EnvBackend::rollout(K, act, obs, rew, term, trunc, s);
  if (!has_reset) {
    gp_set_error("rollout() before reset()");
    return GP_E_STATE;
  }
  int e = dispatch_obs(d.obs_kind, [&](auto okc) -> int {
    constexpr int OK = decltype(okc)::value;
    timer.begin(s);
    if (d.lds.total > 0)  // tables in LDS (all but the PCG jump tables, which sit at the end of the layout)
      hipLaunchKernelGGL((grid_rollout_counter<OK, false, true>), dim3(d.nblk), dim3(TPB), (size_t)d.lds.jt.off, s, d,
                         K, philox_step, (const int32_t*)act, obs, rew, term, trunc);
    else
      hipLaunchKernelGGL((grid_rollout_counter<OK, false>), dim3(d.nblk), dim3(TPB), 0, s, d, K, philox_step,
                         (const int32_t*)act, obs, rew, term, trunc);
    timer.end(s);
    return GP_OK;
  });
  if (e) return e;
  philox_step += (uint64_t)K;
  GP_HIP_CHECK(hipGetLastError());
  return GP_OK;
}

// ---- host-side table construction ----
static const int DY8[8] = {-1, -1, 0, 1, 1, 1, 0, -1};  // action_utils.py:16-27 N,NE,E,SE,S,SW,W,NW
static const int DX8[8] = {0, 1, 1, 1, 0, -1, -1, -1};

int GridBackend::build(const gp_grid_config* cfg) {
  flavor = cfg->flavor;
  depth = cfg->depth;
  height = cfg->height;
  width = cfg->width;
  const int nc = depth * height * width;
  if (depth < 1 || height < 3 || width < 3 || nc >= 32768) {
    gp_set_error("grid shape %dx%dx%d unsupported (cells must be < 32768)", depth, height, width);
    return GP_E_INVALID;
  }
  if (cfg->n_actions != 4 && cfg->n_actions != 8) {
    gp_set_error("n_actions must be 4 or 8");
    return GP_E_INVALID;
  }
  if (cfg->time_limit < 0 || cfg->time_limit > 65534) {
    gp_set_error("time_limit must be in [0, 65534] (elapsed is stored in 16 bits)");
    return GP_E_INVALID;
  }
  if (B <= 0 || B > (int64_t)1 << 30) {
    gp_set_error("num_envs must be in [1, 2^30]");
    return GP_E_INVALID;
  }
  cells.assign(cfg->cells, cfg->cells + nc);
  const int wallv = flavor == GP_FLAVOR_ROOMS ? -1 : 0;
  auto idx = [&](int z, int y, int x) { return (z * height + y) * width + x; };
  auto walkable = [&](int c) { return flavor == GP_FLAVOR_ROOMS ? cells[c] >= 0 : cells[c] > 0; };
  // floor cells must not touch the border (the reference indexes neighbours without bounds checks)
  for (int z = 0; z < depth; ++z)
    for (int y = 0; y < height; ++y)
      for (int x = 0; x < width; ++x)
        if (walkable(idx(z, y, x)) && (y == 0 || x == 0 || y == height - 1 || x == width - 1)) {
          gp_set_error("walkable cell on the map border at (%d,%d,%d)", z, y, x);
          return GP_E_INVALID;
        }
  const int nact = cfg->n_actions;
  d.nact = nact;
  d.ncells = nc;
  // move table: msrooms.py:401-404,415-428 / rooms.py:211-213
  std::vector<uint16_t> move((size_t)nc * nact);
  for (int z = 0; z < depth; ++z)
    for (int y = 0; y < height; ++y)
      for (int x = 0; x < width; ++x) {
        const int c = idx(z, y, x);
        for (int a = 0; a < nact; ++a) {
          const int o = nact == 4 ? 2 * a : a;
          const int ny = y + DY8[o], nx = x + DX8[o];
          uint16_t m = (uint16_t)(c | 0x8000);
          if (walkable(c) && ny >= 0 && nx >= 0 && ny < height && nx < width) {
            const int nb = idx(z, ny, nx);
            if (cells[nb] != wallv) {
              int dest = nb;
              if (flavor == GP_FLAVOR_MULTISTORY) {
                if (cells[nb] == 3 && z + 1 < depth) dest = idx(z + 1, 11, 1);       // up -> (z+1, SW)
                else if (cells[nb] == 2 && z - 1 >= 0) dest = idx(z - 1, 1, 11);     // down -> (z-1, NE)
              }
              m = (uint16_t)dest;
            }
          }
          move[(size_t)c * nact + a] = m;
        }
      }
  // action-failure thresholds (action_utils.py:38-48, 84-90) as exact integers
  std::vector<uint64_t> thr((size_t)nact * nact);
  const double p = cfg->action_failure_probability;
  const double off = p / (nact - 1);
  for (int a = 0; a < nact; ++a) {
    double s = 0.0;
    for (int j = 0; j < nact; ++j) {
      s += (j == a) ? (1 - p) : off;
      const double x = std::ldexp(s, 53);
      thr[(size_t)a * nact + j] = x >= 18446744073709551615.0 ? ~0ull : (uint64_t)std::floor(x);
    }
  }
  // valid spawn cells
  goal_valid_h.clear();
  agent_valid_h.clear();
  for (int c = 0; c < nc; ++c) {
    const int z = c / (height * width);
    if (flavor == GP_FLAVOR_ROOMS) {
      if (cells[c] >= 0) { goal_valid_h.push_back((uint16_t)c); agent_valid_h.push_back((uint16_t)c); }
    } else if (cells[c] > 0) {
      if (z == 0) agent_valid_h.push_back((uint16_t)c);
      if (z == depth - 1) goal_valid_h.push_back((uint16_t)c);
    }
  }
  d.fixed_goal = cfg->fixed_goal;
  d.fixed_agent = cfg->fixed_agent;
  if (d.fixed_goal < 0 && goal_valid_h.size() == 1) d.fixed_goal = goal_valid_h[0];   // choice of 1 draws nothing
  if (d.fixed_agent < 0 && agent_valid_h.size() == 1) d.fixed_agent = agent_valid_h[0];
  if ((d.fixed_goal < 0 && goal_valid_h.empty()) || (d.fixed_agent < 0 && agent_valid_h.empty())) {
    gp_set_error("no valid spawn cells");
    return GP_E_INVALID;
  }
  if (d.fixed_agent >= nc) {
    gp_set_error("fixed agent outside the grid");
    return GP_E_INVALID;
  }
  d.n_goal_valid = (int)goal_valid_h.size();
  d.n_agent_valid = (int)agent_valid_h.size();
  d.thr_goal = d.n_goal_valid > 1 ? lemire_threshold((uint32_t)d.n_goal_valid) : 0;
  d.thr_agent = d.n_agent_valid > 1 ? lemire_threshold((uint32_t)d.n_agent_valid) : 0;
  if (d.fixed_goal >= 0) {
    const int fg = d.fixed_goal;
    // (an off-grid ROOMS goal, e.g. ENDS["32"], decodes as y = fg / W, x = fg % W)
    d.goal_gz = depth == 1 ? 0 : fg / (height * width);
    d.goal_gy = depth == 1 ? fg / width : (fg / width) % height;
    d.goal_gx = fg % width;
  }
  d.time_limit = cfg->time_limit;
  d.r_step = cfg->step_reward;
  d.r_wall = cfg->wall_reward;
  d.r_goal = cfg->goal_reward;
  d.goal_code = flavor == GP_FLAVOR_ROOMS ? 2 : 3;
  // observation tables
  d.obs_kind = cfg->obs_kind;
  d.obs_dirs = cfg->obs_dirs;
  d.obs_goal = cfg->obs_goal;
  d.obs_n = cfg->obs_n;
  d.ndim = flavor == GP_FLAVOR_ROOMS ? 2 : 3;
  if ((cfg->obs_kind == GP_OBS_HANSEN || cfg->obs_kind == GP_OBS_HANSEN_VEC) && cfg->obs_dirs != 4 &&
      cfg->obs_dirs != 8) {
    gp_set_error("obs_dirs must be 4 or 8");
    return GP_E_INVALID;
  }
  std::vector<int32_t> doff(8, 0);
  for (int i = 0; i < 8; ++i) {
    const int o = cfg->obs_dirs == 4 ? 2 * i : i;
    doff[i] = i < (cfg->obs_dirs == 4 ? 4 : 8) ? DY8[o % 8] * width + DX8[o % 8] : 0x7FFFFFFF;
  }
  auto digit = [&](int v) -> int {
    if (flavor == GP_FLAVOR_ROOMS) return v >= 0 ? 1 : 0;   // observations.py:64-66
    if (v == 0) return 0;                                    // msrooms.py:182-185
    return v <= 3 ? 2 : 1;
  };
  std::vector<uint32_t> hbase(nc, 0);
  std::vector<uint8_t> hvec((size_t)nc * std::max(cfg->obs_dirs, 1), 0);
  std::vector<int16_t> coords((size_t)nc * 3);
  for (int c = 0; c < nc; ++c) {
    const int z = c / (height * width), y = (c / width) % height, x = c % width;
    coords[(size_t)c * 3] = (int16_t)z;
    coords[(size_t)c * 3 + 1] = (int16_t)y;
    coords[(size_t)c * 3 + 2] = (int16_t)x;
    if (cfg->obs_kind == GP_OBS_HANSEN || cfg->obs_kind == GP_OBS_HANSEN_VEC) {
      uint32_t hb = 0, mul = 1;
      for (int i = 0; i < cfg->obs_dirs; ++i) {
        const int o = cfg->obs_dirs == 4 ? 2 * i : i;
        const int ny = y + DY8[o], nx = x + DX8[o];
        int dg = 0;
        if (ny >= 0 && nx >= 0 && ny < height && nx < width) dg = digit(cells[idx(z, ny, nx)]);
        hb += (uint32_t)dg * mul;
        mul *= flavor == GP_FLAVOR_ROOMS ? 2 : 3;
        hvec[(size_t)c * cfg->obs_dirs + i] = (uint8_t)dg;
      }
      hbase[c] = hb;
    }
  }
  // Hansen obs with a fixed goal: a table over the agent cell (obs_value's goal multiplier folded in)
  std::vector<int32_t> ofix;
  if (cfg->obs_kind == GP_OBS_HANSEN && d.fixed_goal >= 0) {
    ofix.assign(nc, 0);
    for (int c = 0; c < nc; ++c) {
      int mult = 1;
      if ((unsigned)d.fixed_goal < (unsigned)nc) {
        const int diff = d.fixed_goal - c;
        for (int i = cfg->obs_dirs - 1; i >= 0; --i)
          if (diff == doff[i]) mult = i + 1;
      }
      ofix[c] = (int32_t)hbase[c] * mult;
    }
  }
  std::vector<uint32_t> avo;
  if (!ofix.empty()) {
    avo.resize(2 * agent_valid_h.size());
    for (size_t j = 0; j < agent_valid_h.size(); ++j) {
      avo[2 * j] = agent_valid_h[j];
      avo[2 * j + 1] = (uint32_t)ofix[agent_valid_h[j]];
    }
  }
  std::vector<uint8_t> window;
  if (cfg->obs_kind == GP_OBS_WINDOW) {
    const int n = cfg->obs_n, h = n / 2;
    if (n < 1 || n > 63) {
      gp_set_error("obs_n must be in [1, 63]");
      return GP_E_INVALID;
    }
    window.assign((size_t)nc * n * n, 0);
    for (int c = 0; c < nc; ++c) {
      const int z = c / (height * width), y = (c / width) % height, x = c % width;
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
          int yy = y + i - h, xx = x + j - h;
          if (yy < 0 || xx < 0 || yy >= height || xx >= width) yy = xx = 0;  // observations.py:92-98
          window[((size_t)c * n + i) * n + j] = (uint8_t)(cells[idx(z, yy, xx)] + 1 > 0 ? 1 : 0);
        }
    }
    if (flavor != GP_FLAVOR_ROOMS) {
      gp_set_error("window obs is only defined for ROOMS");
      return GP_E_INVALID;
    }
  }
  std::vector<int32_t> t1, t2;
  if (cfg->obs_kind == GP_OBS_TABLE) {
    if (!cfg->obs_table) {
      gp_set_error("GP_OBS_TABLE needs obs_table");
      return GP_E_INVALID;
    }
    t1.assign(cfg->obs_table, cfg->obs_table + nc);
    if (cfg->obs_table2) {
      if (d.fixed_goal >= nc) {
        gp_set_error("goal outside the grid cannot index the goal obs table (reference raises IndexError)");
        return GP_E_INVALID;
      }
      t2.assign(cfg->obs_table2, cfg->obs_table2 + nc);
    }
  }
  switch (cfg->obs_kind) {
    case GP_OBS_HANSEN: obs_dtype = GP_DTYPE_I32; obs_width = 1; break;
    case GP_OBS_HANSEN_VEC: obs_dtype = GP_DTYPE_U8; obs_width = cfg->obs_dirs; break;
    case GP_OBS_TABLE: obs_dtype = GP_DTYPE_I32; obs_width = 1; break;
    case GP_OBS_COORDS: obs_dtype = GP_DTYPE_I32; obs_width = d.ndim * (cfg->obs_goal ? 2 : 1); break;
    case GP_OBS_WINDOW: obs_dtype = GP_DTYPE_U8; obs_width = cfg->obs_n * cfg->obs_n; break;
    default: gp_set_error("obs kind %d not valid for GRID", cfg->obs_kind); return GP_E_INVALID;
  }
  d.obs_width = obs_width;
  d.B = (int32_t)B;
  d.nblk = (int32_t)((B + EPB - 1) / EPB);
  int e;
  if ((e = b_move.upload(move)) || (e = b_thr.upload(thr)) || (e = b_gv.upload(goal_valid_h)) ||
      (e = b_av.upload(agent_valid_h)) || (e = b_hbase.upload(hbase)) || (e = b_doff.upload(doff)) ||
      (e = b_ofix.upload(ofix)) || (e = b_avo.upload(avo)) ||
      (e = b_hvec.upload(hvec)) || (e = b_coords.upload(coords)) || (e = b_window.upload(window)) ||
      (e = b_t1.upload(t1)) || (e = b_t2.upload(t2)))
    return e;
  // K2 grid: at most one block per CU (all resident: blocks wait on lower-index blocks' flags)
  {
    hipDeviceProp_t prop;
    GP_HIP_CHECK(hipGetDeviceProperties(&prop, device));
    grid_persist = std::max(1, std::min({d.nblk, prop.multiProcessorCount, 256}));
    if ((d.nblk + grid_persist - 1) / grid_persist > MAX_TPB2) {
      gp_set_error("num_envs too large for the resolver (max %d)", 256 * MAX_TPB2 * EPB);
      return GP_E_INVALID;
    }
  }
  // LDS staging of the lookup tables for the fused kernel (when they fit). The fixed-goal obs table (ofix) and
  // the {agent, obs} pairs (avo) only speed up the staged Hansen path: they are laid out only when the image
  // still fits the budget with them, so that they never cost a config its fused eligibility.
  {
    const int k = cfg->obs_kind;
    auto layout = [&](bool fast) {
      int off = 0;
      auto put = [&](GridLdsTab& t, size_t bytes) {
        t.off = off;
        t.bytes = (int)bytes;
        off += (int)((bytes + 15) / 16 * 16);
      };
      put(d.lds.move, (size_t)nc * nact * sizeof(uint16_t));
      put(d.lds.hbase, k == GP_OBS_HANSEN ? (size_t)nc * sizeof(uint32_t) : 0);
      put(d.lds.hvec, k == GP_OBS_HANSEN_VEC ? hvec.size() : 0);
      put(d.lds.t1, t1.size() * sizeof(int32_t));
      put(d.lds.t2, t2.size() * sizeof(int32_t));
      put(d.lds.coords, (k == GP_OBS_COORDS || k == GP_OBS_WINDOW) ? coords.size() * sizeof(int16_t) : 0);
      put(d.lds.window, window.size());
      put(d.lds.gv, goal_valid_h.size() * sizeof(uint16_t));
      put(d.lds.av, agent_valid_h.size() * sizeof(uint16_t));
      put(d.lds.doff, doff.size() * sizeof(int32_t));
      put(d.lds.ofix, fast ? ofix.size() * sizeof(int32_t) : 0);
      put(d.lds.avo, fast ? avo.size() * sizeof(uint32_t) : 0);
      put(d.lds.jt, sizeof(PcgJump) * JT_LEVELS * JT_RADIX);  // jump tables last (the philox kernel omits them)
      put(d.lds.jt8, sizeof(PcgJump) * 2 * 256);
      return off;
    };
    int off = layout(true);
    if (off > LDS_TABLE_BUDGET && (!ofix.empty() || !avo.empty())) off = layout(false);
    d.lds.total = off <= LDS_TABLE_BUDGET ? off : 0;
  }
  // fused numpy rollout: one 512-thread block per CU, <= 4 tiles of 2048 envs per block
  const GpDebugKnobs& dbg = gp_debug_knobs();  // diagnostic knobs (gp_debug_set); defaults in production
  {
    // fused tile size: 2048 envs (8 env waves) unless that leaves CUs without a tile (strong-scaling shard sizes:
    // 2^17 envs are 64 tiles of 2048 but 256 of 512), halved down to 512 (2 env waves) until every CU has one
    hipDeviceProp_t prop;
    GP_HIP_CHECK(hipGetDeviceProperties(&prop, device));
    const int cus = std::min(prop.multiProcessorCount, FMAXG);
    int tile = FEPB;
    if (dbg.fused_tile == 512 || dbg.fused_tile == 1024 || dbg.fused_tile == 2048) {
      tile = dbg.fused_tile;
    } else {
      while (tile > 512 && (B + tile - 1) / tile < cus) tile /= 2;
    }
    d.ftile = tile;
    d.faw = tile / (64 * EPT);
  }
  d.fnt = (int)((B + d.ftile - 1) / d.ftile);
  // exchange variant: bits 0-1: 1 = every block all-gathers the granules (default), 0 = block-0 aggregator;
  // bit 4: plain (not non-temporal) staged output stores; bits 2-3 (stamps builds only): output diagnostics
  d.xmode = dbg.xmode;
  d.spin_limit = dbg.spin_limit ? dbg.spin_limit : SPIN_LIMIT;
  d.fault_block = dbg.fault_block;
  {
    hipDeviceProp_t prop;
    GP_HIP_CHECK(hipGetDeviceProperties(&prop, device));
    int occ = 0;
    GP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, grid_rollout_numpy<GP_OBS_WINDOW, 4, 8, false, false>,
                                                             FTPB, d.lds.total));
    const int G = std::min({prop.multiProcessorCount, FMAXG, d.fnt});
    const int qpt = (d.fnt + G - 1) / G;
    // (tiles smaller than FEPB only come with <= 2 tiles per block: the kernels for them exist for QPT <= 2)
    if (occ >= 1 && d.fnt <= FMAXT && qpt <= (d.ftile == FEPB ? 4 : 2) && d.lds.total > 0 && !dbg.disable_fused) {
      fused_G = G;
      fused_qpt = qpt <= 1 ? 1 : (qpt <= 2 ? 2 : 4);
      const int k = cfg->obs_kind;
      // staged outputs: <= 2 tiles per block, scalar obs, and only complete tiles (every block owns exactly
      // fused_qpt full tiles: the staged kernel drops the per-env bounds checks)
      if (fused_qpt <= 2 && (k == GP_OBS_HANSEN || k == GP_OBS_TABLE) && !dbg.no_staging &&
          (int64_t)B == (int64_t)fused_qpt * G * d.ftile) {
        int occ2 = 0;
        GP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &occ2, grid_rollout_numpy<GP_OBS_HANSEN, 2, 8, true, false>, FTPB, d.lds.total + 2 * STG_TILE_BYTES));
        fused_stg = occ2 >= 1;
        // SPW windows (one reset call per step: the fast cell draw) when they fit beside the staging area
        if (fused_stg && (d.fixed_goal < 0) != (d.fixed_agent < 0) && !dbg.no_spw) {
          int occ3 = 0;
          GP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
              &occ3, grid_rollout_numpy<GP_OBS_HANSEN, 2, 8, true, false>, FTPB,
              d.lds.total + 2 * STG_TILE_BYTES + spw_bytes(2)));
          d.spw_on = occ3 >= 1;
        }
      }
    }
  }
  // the windowed numpy rollout (wgrid.hip): a fixed goal, random agent spawns and a scalar obs that is a
  // function of the agent cell (Hansen with the goal multiplier folded in, or table[agent] + table2[goal])
  if (rng_mode == GP_RNG_NUMPY && d.fixed_goal >= 0 && d.fixed_agent < 0 && d.n_agent_valid >= 2 &&
      (cfg->obs_kind == GP_OBS_HANSEN || cfg->obs_kind == GP_OBS_TABLE) && !dbg.no_wgrid && !dbg.disable_fused) {
    if (dbg.wg_kmax >= 0) wg_kmax = dbg.wg_kmax;
    std::vector<int32_t> ocell(nc);
    for (int c = 0; c < nc; ++c)
      ocell[c] = cfg->obs_kind == GP_OBS_HANSEN ? ofix[c] : t1[c] + (t2.empty() ? 0 : t2[d.fixed_goal]);
    if (int e2 = build_wgrid(move, thr, ocell)) return e2;
    // The windowed kernel at every launch length for blocks of <= 1,024 envs (<= 2^18 envs, e.g. the strong-scaling
    // shards: 3.02 vs 3.69 us/step at 2^17 envs and 3.32 vs 3.60 at 2^18 in 128-step launches, 67 vs 82 us per
    // 20-step launch at 2^17) and, since its round-6 window-row balance, for 4,096-env blocks (2^20 envs: 109.4-109.6
    // vs 117.0-118.1 us at K = 20, 328.6-328.8 vs 334.8-343.1 at 64, 647.1-647.2 vs 647.3-655.3 at 128,
    // profiles/r06_kernel_by_K.txt). 2,048-env blocks keep WG_KMAX (not re-measured).
    if (dbg.wg_kmax < 0 && wg_G && (wg_NS <= 2 || wg_NS >= 8)) wg_kmax = 1 << 30;
  }
  wg_kmax_default = wg_kmax;
  nslots = std::max({d.nblk, grid_persist, fused_G, wg_G});
  if ((e = b_jt.alloc(sizeof(PcgJump) * JT_LEVELS * JT_RADIX)) || (e = b_lt4.alloc(sizeof(PcgJump) * TPB)) ||
      (e = b_lt2.alloc(sizeof(PcgJump) * TPB)) || (e = b_tja.alloc(sizeof(PcgJump) * (size_t)d.nblk)) ||
      (e = b_tjw.alloc(sizeof(PcgJump) * (size_t)d.nblk)) || (e = b_ae.alloc(sizeof(uint32_t) * (B + 4))) ||
      (e = b_goal.alloc(sizeof(uint16_t) * (B + 8))) || (e = b_ctl.alloc(sizeof(GridCtl))) ||
      (e = b_tcount.alloc(sizeof(uint32_t) * (size_t)d.nblk)) ||
      (e = b_tlist.alloc(sizeof(uint16_t) * (size_t)d.nblk * EPB)) || (e = b_rflag.alloc(sizeof(uint32_t) * 256)) ||
      (e = b_mslot.alloc(sizeof(MetricSlot) * (size_t)nslots)) ||
      (e = b_ftj.alloc(sizeof(PcgJump) * (size_t)std::max(d.fnt, 1))) || (e = b_flt4.alloc(sizeof(PcgJump) * FTPB)) ||
      (e = b_fjB.alloc(2 * sizeof(PcgJump))) || (e = b_fslot.alloc(sizeof(uint64_t) * 8 * (size_t)std::max(d.fnt, 1))))
    return e;
  d.move = b_move.as<uint16_t>();
  d.thr = b_thr.as<uint64_t>();
  d.goal_valid = b_gv.as<uint16_t>();
  d.agent_valid = b_av.as<uint16_t>();
  d.hbase = b_hbase.as<uint32_t>();
  d.doff = b_doff.as<int32_t>();
  d.ofix = ofix.empty() ? nullptr : b_ofix.as<int32_t>();
  d.avo = avo.empty() ? nullptr : b_avo.as<uint32_t>();
  d.hvec = b_hvec.as<uint8_t>();
  d.t1 = t1.empty() ? nullptr : b_t1.as<int32_t>();
  d.t2 = t2.empty() ? nullptr : b_t2.as<int32_t>();
  d.coords = b_coords.as<int16_t>();
  d.window = b_window.as<uint8_t>();
  d.jt = b_jt.as<PcgJump>();
  d.lt4 = b_lt4.as<PcgJump>();
  d.lt2 = b_lt2.as<PcgJump>();
  d.tja = b_tja.as<PcgJump>();
  d.tjw = b_tjw.as<PcgJump>();
  d.mslot = b_mslot.as<MetricSlot>();
  d.ae = b_ae.as<uint32_t>();
  d.goal = b_goal.as<uint16_t>();
  d.ctl = b_ctl.as<GridCtl>();
  d.tcount = b_tcount.as<uint32_t>();
  d.tlist = b_tlist.as<uint16_t>();
  d.rflag = b_rflag.as<uint32_t>();
  d.ftj = b_ftj.as<PcgJump>();
  d.flt4 = b_flt4.as<PcgJump>();
  d.fjB = b_fjB.as<PcgJump>();
  d.fslot = b_fslot.as<uint64_t>();
  // The fused kernel's slots start with tag 0x7FFF: tags are (step + 1) * 4 + round with round <= 2, so this value
  // is never expected (a zeroed slot would match tag 0, i.e. round 0 of every 8192nd step).
  GP_HIP_CHECK(hipMemset(b_fslot.p, 0xFF, b_fslot.n));
#ifdef GP_STAMPS
  if ((e = b_dbg.alloc(sizeof(unsigned long long) * (256 * 64 * 16 + 256 * 8)))) return e;
  d.dbg = b_dbg.as<unsigned long long>();
#endif
  if ((e = b_self.alloc(sizeof(GridDev))) || (e = b_jt8.alloc(sizeof(PcgJump) * 2 * 256)) ||
      (e = b_limg.alloc(d.lds.total > 0 ? (size_t)d.lds.total : 0)))
    return e;
  d.self = b_self.as<GridDev>();
  d.jt8 = b_jt8.as<PcgJump>();
  d.limg = b_limg.as<char>();
  // default seed: numpy's SeedSequence(0) until the caller seeds
  rng = pcg64_from_seed({0u}, {});
  return upload_rng();
}

}  // namespace

std::unique_ptr<EnvBackend> make_grid_backend(const gp_grid_config* cfg, int64_t B, int device, int rng_mode,
                                              int* err) {
  auto g = std::make_unique<GridBackend>();
  g->B = B;
  g->device = device;
  g->rng_mode = rng_mode;
  *err = g->build(cfg);
  if (*err) return nullptr;
  return g;
}
