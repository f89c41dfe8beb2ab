// crooms.hip — the C-ROOMS backend (GP_KIND_CROOMS): CRoomsEnv.step / _apply_action /
// _out_of_bounds / _reset_some / reset and its observation functions (gym_po/envs/rooms/crooms.py:16-338).
//
// Arithmetic: float64, operation for operation as the reference (which computes in numpy float64),
// with contraction into FMAs disabled, so that with the same noise values the device trajectory is
// the reference's trajectory bit-for-bit; float64 state stays in registers across a rollout, so it
// costs no HBM traffic. I/O is float32 by default (BASELINE configs[4]: f32 actions, f32 obs — the
// only rounding is the final cast of the emitted observation), or float64 on request.
//   terminated: ||agent - goal||_2 <= thr is evaluated as  dy*dy + dx*dx <= S  with S the largest
//   double whose correctly rounded sqrt is <= thr (exactly numpy's sqrt(add.reduce(x*x)) <= thr).
//
// RNG: the reference draws numpy ziggurat normals (data-dependent word counts) and choice() from one
// stream, so no parallel kernel can follow it word for word. GP_RNG_PHILOX draws the same laws from a
// counter-based Philox4x32-10 keyed by the seed: normals by Box-Muller on a 53-bit u1 (one Philox block per
// pair; the radius reaches sqrt(-2 ln 2^-53) = 8.57 sigma, no tail cut) in float32 hardware arithmetic
// (GP_CR_NORMAL_F64=1: float64 log / sqrt / sincospi, 2.4x slower rollouts), Lemire cell indices, 53-bit
// uniforms compared against the integer action-failure thresholds. GP_RNG_REPLAY takes the values the
// reference's stream produced (how parity is tested). numpy's own normal algorithm (the 256-layer ziggurat,
// zig_normal below) is restated too and checked bit for bit against numpy over numpy's words
// (gp_standard_normal_words); as the philox sampler its rare rejection path, taken by ~1.5% of the normals
// but by some lane of nearly every wave, made the rollout 2.7x slower than Box-Muller, which is branch-free.
//
// Kernels: a persistent, grid-stride rollout kernel (tables staged in LDS once per block, 512-env
// tiles, K steps per tile, 2 envs per thread).
#include <algorithm>
#include <cassert>
#include <cmath>
#include <cstring>
#include <vector>

#include "gp_internal.h"
#include "gp_libm.h"
#include "ziggurat_tables.h"

#pragma clang fp contract(off)

// gp_debug_set("xg_graph"), read at create (CRoomsBackend::xg_graph_mode): -1 default, 0 never, 1 from the first call.
int gp_xg_graph_knob = -1;

namespace {

constexpr int TPB = 256;
constexpr int EPT = 2;
constexpr int EPB = TPB * EPT;
constexpr int WAVES = TPB / 64;
constexpr uint32_t TAG_NOISE = 0x63726f6fu;  // 'croo'
constexpr uint32_t TAG_DRAW = 0x6d733121u;
// Philox rounds of the philox-mode blocks (noise and reset draws; oracle/philox.py philox4x32(rounds=)): Random123's
// default 10. Round 6 measured 7 (the fewest Salmon et al. 2011 report Crush-resistant) at configs[4]: 1905 vs 1945
// us per 128-step launch (frac 0.393 vs 0.385, one call): too little for the lost margin, so 10 stays.
#ifndef CR_PHILOX_ROUNDS
#define CR_PHILOX_ROUNDS 10
#endif
#ifndef GP_CR_NORMAL_F64
#define GP_CR_NORMAL_F64 0
#endif
// Minimum waves per SIMD of the rollout kernel (caps its VGPRs at 512 / waves; tuning knob).
#ifndef GP_CR_WAVES
#define GP_CR_WAVES 7
#endif
constexpr double MAX_VELOCITY = 5.0;
// Largest batch of the exact (numpy-stream) mode, which runs in one workgroup.

struct alignas(32) CrSlot {
  double return_sum;
  unsigned long long episodes, length_sum, env_steps;
};

// observation kinds handled here (GP_OBS_F32 = continuous coordinates)
struct CrDev {
  int32_t B, ntiles, H, W, ncells;
  int32_t use_velocity, action_kind, action_f64, nact;
  int32_t obs_kind, obs_f64, obs_dirs, obs_goal, obs_n, obs_width, has_t2;
  int32_t goal_fixed, goal_y, goal_x, agent_fixed, agent_y, agent_x;
  int32_t n_valid, time_limit;
  uint32_t key0, key1;
  double cell, half_cell, hi_y, hi_x, s_thr, action_std, action_power;
  double inv_cell;       // 1 / cell when cell is a power of two (then y * inv_cell == y / cell exactly), else 0
  double gcy, gcx;       // fixed goal: its square's centre goal_y + 0.5, goal_x + 0.5 (as the device computes it)
  float r_step, r_wall, r_goal;
  const uint8_t* tabs;   // packed tables, staged into LDS
  int32_t off_wall, off_valid, off_thr, off_t1, off_t2, off_hbase, off_hvec, off_doff, off_window, tab_bytes;
  // state (SoA)
  double* ay;
  double* ax;
  double* vy;
  double* vx;
  uint32_t* goal;        // gy | gx << 16 (int16 each; a fixed goal may lie off the grid)
  int32_t* el;
  CrSlot* mslot;
  int32_t nslot;         // metric slots (the exact-mode step kernel spreads its blocks' atomics over them)
  uint32_t* derr;        // device error word (GP_DERR_*)
  // replay
  const uint64_t* rp_u;
  const int32_t* rp_goal;
  const int32_t* rp_agent;
  const double* rp_noise;
  const double* rp_wall;
};

template <class T>
__device__ __forceinline__ const T* tab(const uint8_t* l, int off) {
  return reinterpret_cast<const T*>(l + off);
}

__device__ __forceinline__ void stage_tables(const CrDev& p, uint8_t* lds) {
  const uint4* src = (const uint4*)p.tabs;
  uint4* dst = (uint4*)lds;
  for (int i = threadIdx.x; i < p.tab_bytes / 16; i += TPB) dst[i] = src[i];
}

// ---- draws ----
// numpy's random_standard_normal (numpy/random/src/distributions/distributions.c, numpy 2.2): the 256-layer
// ziggurat on 64-bit words. `r` is the normal's first word; `next` yields the words it consumes after that
// (a rejected layer draw or the tail, ~1% of normals). Operation for operation as numpy (no FMA
// contraction in this file), so over numpy's word stream it returns numpy's values (checked bit for bit
// against numpy by gp_standard_normal_words).
// log1p of the tail: numpy calls the C library's log1p (npy_log1p -> libm; NOT the SIMD np.log1p ufunc, which
// differs from libm in ~1% of last bits). zlog1p_neg restates glibc 2.35's log1p (sysdeps/ieee754/dbl-64/
// s_log1p.c: fdlibm's reduction and its Lp1..Lp7 polynomial in the parallel R1 + z2 R2 + z4 R3 + z6 R4 order),
// IEEE double ops without contraction, so tail values equal numpy's bit for bit; host copy gp_log1p_libm for
// the CPU test against libm (tests/test_log1p_cpu.py). exp of the wedge test: glibc 2.35's exp restated
// (gp_libm.h, pinned against libm by tests/test_libm_cpu.py), so wedge accepts / rejects are numpy's exactly.
// The host libm's exp build (gp_exp_host_variant: 1 the -mfma build, 0 the plain one), set at create time.
__device__ int g_crooms_exp_fma = 1;
__device__ __forceinline__ double zexp(double y) {
  return g_crooms_exp_fma ? gp_libm::exp<true>(y) : gp_libm::exp<false>(y);
}
GP_HD int32_t zhi(double x) { return (int32_t)(__builtin_bit_cast(uint64_t, x) >> 32); }
GP_HD double zset_hi(double x, int32_t h) {
  return __builtin_bit_cast(double, (__builtin_bit_cast(uint64_t, x) & 0xFFFFFFFFull) | ((uint64_t)(uint32_t)h << 32));
}
// log1p(-u) for u in [0, 1): glibc's __log1p(x) at x = -u (the branches x >= 0.41422, |x| < 2^-54 and
// x <= -1 cannot occur here). No fma anywhere: every operation is a separately rounded IEEE double op.
GP_HD double zlog1p_neg(double u) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01, Lp3 = 2.857142874366239149e-01,
               Lp4 = 2.222219843214978396e-01, Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
               Lp7 = 1.479819860511658591e-01;
  const double x = -u;
  const int32_t hx = zhi(x), ax = hx & 0x7fffffff;
  if (ax < 0x3e200000) return x - x * x * 0.5;  // |x| < 2^-29 (u = 0: x - 0 = -0.0, numpy's log1p(-0.0))
  int32_t k = 1, hu = 0;
  double f = 0.0, c = 0.0;
  if (hx > 0 || hx <= (int32_t)0xbfd2bec3) {  // -0.2929 < x < 0.41422 (glibc keeps fdlibm's 0xbfd2bec3)
    k = 0;
    f = x;
    hu = 1;
  } else {
    double v = 1.0 + x;
    hu = zhi(v);
    k = (hu >> 20) - 1023;
    c = (k > 0) ? 1.0 - (v - x) : x - (v - 1.0);  // correction term
    c /= v;
    hu &= 0x000fffff;
    if (hu < 0x6a09e) {
      v = zset_hi(v, hu | 0x3ff00000);  // normalize v
    } else {
      k += 1;
      v = zset_hi(v, hu | 0x3fe00000);  // normalize v / 2
      hu = (0x00100000 - hu) >> 2;
    }
    f = v - 1.0;
  }
  const double hfsq = 0.5 * f * f;
  const double dk = (double)k;
  if (hu == 0) {  // |f| < 2^-20
    if (f == 0.0) {
      if (k == 0) return 0.0;
      c += dk * ln2_lo;
      return dk * ln2_hi + c;
    }
    const double R = hfsq * (1.0 - 0.66666666666666666 * f);
    if (k == 0) return f - R;
    return dk * ln2_hi - ((R - (dk * ln2_lo + c)) - f);
  }
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double R1 = z * Lp1, z2 = z * z;
  const double R2 = Lp2 + z * Lp3, z4 = z2 * z2;
  const double R3 = Lp4 + z * Lp5, z6 = z4 * z2;
  const double R4 = Lp6 + z * Lp7;
  const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
  if (k == 0) return f - (hfsq - s * (hfsq + R));
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + (dk * ln2_lo + c))) - f);
}

// numpy's ki / wi / fi tables (ziggurat_tables.h), one array: ki at 0, wi at 256, fi at 512.
__device__ const uint64_t d_zig[768] = {GP_ZIG_KI_LIST, GP_ZIG_WI_LIST, GP_ZIG_FI_LIST};
struct ZigTabs {
  const uint64_t* ki;
  const double* wi;
  const double* fi;
};
__device__ __forceinline__ double u53_of(uint64_t w) { return (double)(w >> 11) * (1.0 / 9007199254740992.0); }
// zig_dry(next): the word source ran out (only the diagnostic source below can); a tail loop fed by an exhausted
// source would otherwise spin forever on zero words (0 > 0 never accepts).
template <class NEXT>
__device__ __forceinline__ bool zig_dry(const NEXT&) { return false; }
template <class NEXT>
__device__ __forceinline__ double zig_slow(const ZigTabs& t, uint64_t r, NEXT& next) {
  for (;;) {
    const int idx = (int)(r & 0xff);
    r >>= 8;
    const uint64_t sign = r & 1u, rabs = (r >> 1) & 0x000fffffffffffffull;
    double x = (double)rabs * t.wi[idx];
    if (sign) x = -x;
    if (rabs < t.ki[idx]) return x;
    if (idx == 0) {
      for (;;) {
        const double xx = -GP_ZIG_INV_R * zlog1p_neg(u53_of(next()));
        const double yy = -zlog1p_neg(u53_of(next()));
        if (yy + yy > xx * xx || zig_dry(next)) return ((rabs >> 8) & 1u) ? -(GP_ZIG_R + xx) : GP_ZIG_R + xx;
      }
    }
    if ((t.fi[idx - 1] - t.fi[idx]) * u53_of(next()) + t.fi[idx] < zexp(-0.5 * x * x)) return x;
    r = next();
  }
}
// The fast path (~99% of draws): one word, two table loads; false = the slow path must finish the draw.
__device__ __forceinline__ bool zig_fast(const ZigTabs& t, uint64_t r, double& z) {
  const int idx = (int)(r & 0xff);
  const uint64_t rr = r >> 8, rabs = (rr >> 1) & 0x000fffffffffffffull;
  const double x = (double)rabs * t.wi[idx];
  z = (rr & 1u) ? -x : x;
  return rabs < t.ki[idx];
}
template <class NEXT>
__device__ __forceinline__ double zig_normal(const ZigTabs& t, uint64_t r, NEXT& next) {
  double z;
  if (zig_fast(t, r, z)) return z;
  return zig_slow(t, r, next);
}
// The philox-mode normal pair: Box-Muller on u1 = K 2^-53 in (0, 1] (K = 53 bits of w1, plus 1) and the angle
// u2 from w2: r = sqrt(-2 ln u1), (z0, z1) = r (cos 2 pi u2, sin 2 pi u2); |z| reaches 8.57 (the former
// 24-bit u1 stopped at 5.77). Float32 hardware arithmetic: ln u1 = ln2 (p - 53 + log2 m) with K = m 2^p,
// m in [1, 2) taken to 24 bits (v_log_f32 is log2), v_sqrt_f32, v_sin / v_cos_f32 of a 24-bit angle in
// revolutions; GP_CR_NORMAL_F64: the same in float64 (device libm).
__device__ __forceinline__ void box_muller_pair(uint64_t w1, uint64_t w2, double& z0, double& z1) {
#if GP_CR_NORMAL_F64
  const double u1 = (double)((w1 >> 11) + 1u) * 0x1p-53;
  const double u2 = (double)(w2 >> 11) * 0x1p-53;
  const double r = sqrt(-2.0 * log(u1));
  double sn, cs;
  sincospi(2.0 * u2, &sn, &cs);
  z0 = r * cs;
  z1 = r * sn;
#else
  const uint64_t K = (w1 >> 11) + 1u;
  const int pw = 63 - __builtin_clzll(K);
  const float m = (float)(uint32_t)((K << (63 - pw)) >> 40) * 0x1p-23f;
  const float l2 = (float)(pw - 53) + __builtin_amdgcn_logf(m);                      // log2 u1 <= 0
  const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * l2);                  // sqrt(-2 ln u1)
  const float u2 = (float)(uint32_t)(w2 >> 40) * 0x1p-24f;                            // revolutions
  z0 = (double)(r * __builtin_amdgcn_cosf(u2));
  z1 = (double)(r * __builtin_amdgcn_sinf(u2));
#endif
}


struct Draws {
  uint64_t k53;      // action-failure uniform
  uint32_t gi, ai;   // reset cell indices
};

// Gaussian noise of env-step (env, step): pair 0 = action noise N(0, action_std) (crooms.py:178,
// :194-195), pair 1 = wall noise N(0, 0.5) (:324). Replay: the values numpy returned. Philox: ONE block of
// counter (env, step, TAG_NOISE) per env-step (kept in blk / have by the caller) serves both pairs with
// disjoint bits: pair 0 = box_muller_pair(x1:x0 -> 53-bit u1, x3:x2 -> 24-bit angle); pair 1 takes the bits
// pair 0 leaves: u1 = (x2 + 1) 2^-32 (radius to 6.66 sigma), a 19-bit angle (x0 & 0x7FF, x3 & 0xFF). The
// wall noise is clipped to its cell (|n| <= cell / 2, i.e. |z| <= 1 at the default cell), so its far
// tail never reaches an observation.
__device__ __forceinline__ void box_muller_wall(const Philox4& r, double& z0, double& z1) {
  const float l2 = __builtin_amdgcn_logf(((float)r.x[2] + 1.0f) * 0x1p-32f);            // log2 u1 (u1 in (0, 1])
  const float rad = __builtin_amdgcn_sqrtf(-1.3862943611198906f * l2);
  const float u2 = (float)(((r.x[0] & 0x7FFu) << 8) | (r.x[3] & 0xFFu)) * 0x1p-19f;  // revolutions
  z0 = (double)(rad * __builtin_amdgcn_cosf(u2));
  z1 = (double)(rad * __builtin_amdgcn_sinf(u2));
}
template <bool REPLAY>
__device__ __forceinline__ void draw_normals(const CrDev& p, int env, uint64_t step, int pair, double scale,
                                             double& y, double& x, Philox4& blk, bool& have) {
  if constexpr (REPLAY) {
    const double* src = pair == 0 ? p.rp_noise : p.rp_wall;
    const double2 v = *reinterpret_cast<const double2*>(src + 2 * (size_t)env);
    y = v.x;
    x = v.y;
  } else {
    if (!have) {
      blk = philox4x32<CR_PHILOX_ROUNDS>((uint32_t)env, (uint32_t)step, (uint32_t)(step >> 32), TAG_NOISE, p.key0,
                                         p.key1);
      have = true;
    }
    double z0, z1;
    if (pair == 0)
      box_muller_pair(((uint64_t)blk.x[1] << 32) | blk.x[0], ((uint64_t)blk.x[3] << 32) | blk.x[2], z0, z1);
    else
      box_muller_wall(blk, z0, z1);
    y = scale * z0;
    x = scale * z1;
  }
}

template <bool REPLAY>
__device__ __forceinline__ void draw_ints(const CrDev& p, int env, uint64_t step, Draws& d) {
  if constexpr (REPLAY) {
    d.k53 = p.rp_u ? p.rp_u[env] : 0ull;
    d.gi = p.rp_goal ? (uint32_t)min(max(p.rp_goal[env], 0), p.n_valid - 1) : 0u;
    d.ai = p.rp_agent ? (uint32_t)min(max(p.rp_agent[env], 0), p.n_valid - 1) : 0u;
  } else {
    const Philox4 r =
        philox4x32<CR_PHILOX_ROUNDS>((uint32_t)env, (uint32_t)step, (uint32_t)(step >> 32), TAG_DRAW, p.key0, p.key1);
    d.k53 = ((((uint64_t)r.x[0]) << 32) | r.x[1]) >> 11;
    d.gi = lemire_value(r.x[2], (uint32_t)p.n_valid);
    d.ai = lemire_value(r.x[3], (uint32_t)p.n_valid);
  }
}

// ---- observation builders (crooms.py:16-88 on coord_to_grid cells; observations.py semantics) ----
struct Cells {
  int ac, gc;      // flat cells of agent / goal (gc = -1 when the goal lies off the grid)
};

// coord / cell_size, exactly as numpy divides (a multiply when cell_size is a power of two)
__device__ __forceinline__ double per_cell(const CrDev& p, double v) {
  if (p.inv_cell == 1.0) return v;  // uniform: the default cell size (v * 1.0 == v, two f64 multiplies saved)
  return p.inv_cell != 0.0 ? v * p.inv_cell : v / p.cell;
}

__device__ __forceinline__ int cell_of(const CrDev& p, double y, double x) {
  // coord_to_grid (utils.py:15-20): floor(coord / cell_size)
  const int cy = (int)floor(per_cell(p, y)), cx = (int)floor(per_cell(p, x));
  if (cy < 0 || cx < 0 || cy >= p.H || cx >= p.W) return -1;
  return cy * p.W + cx;
}

// The same for coordinates known to be >= 0 (the clipped position): floor == truncation there, so the integer
// conversion (v_cvt_i32_f64 truncates) is the floor and the two float64 floors go.
__device__ __forceinline__ int cell_of_nonneg(const CrDev& p, double y, double x) {
  const int cy = (int)per_cell(p, y), cx = (int)per_cell(p, x);
  if (cy >= p.H || cx >= p.W) return -1;
  return cy * p.W + cx;
}

// write env's observation; OK = obs kind
template <int OK>
__device__ __forceinline__ void write_obs(const CrDev& p, const uint8_t* lds, int env, double ay, double ax,
                                          uint32_t g, void* __restrict__ obs) {
  const double gyc = (double)(int16_t)(g & 0xFFFF) + 0.5, gxc = (double)(int16_t)(g >> 16) + 0.5;
  if constexpr (OK == GP_OBS_F32) {
    const int w = p.obs_width;
    if (p.obs_f64) {
      double* o = (double*)obs + (size_t)env * w;
      o[0] = ay; o[1] = ax;
      if (w == 4) { o[2] = gyc; o[3] = gxc; }
    } else {
      float* o = (float*)obs + (size_t)env * w;
      if (w == 4) {
        *reinterpret_cast<float4*>(o) = make_float4((float)ay, (float)ax, (float)gyc, (float)gxc);
      } else {
        *reinterpret_cast<float2*>(o) = make_float2((float)ay, (float)ax);
      }
    }
  } else {
    const int ac = max(cell_of(p, ay, ax), 0);
    const int gc = cell_of(p, gyc, gxc);
    const bool gvalid = gc >= 0;
    const int32_t* doff = tab<int32_t>(lds, p.off_doff);
    if constexpr (OK == GP_OBS_HANSEN) {
      int mult = 1;
      if (gvalid) {
        const int diff = gc - ac;
        for (int i = p.obs_dirs - 1; i >= 0; --i)
          if (diff == doff[i]) mult = i + 1;
      }
      ((int32_t*)obs)[env] = (int32_t)tab<uint32_t>(lds, p.off_hbase)[ac] * mult;
    } else if constexpr (OK == GP_OBS_HANSEN_VEC) {
      uint8_t* o = (uint8_t*)obs + (size_t)env * p.obs_width;
      const int diff = gc - ac;
      for (int i = 0; i < p.obs_dirs; ++i) {
        uint8_t v = tab<uint8_t>(lds, p.off_hvec)[ac * p.obs_dirs + i];
        if (p.obs_goal && gvalid && diff == doff[i]) v = 2;
        o[i] = v;
      }
    } else if constexpr (OK == GP_OBS_TABLE) {
      int32_t v = tab<int32_t>(lds, p.off_t1)[ac];
      if (p.has_t2) v += tab<int32_t>(lds, p.off_t2)[max(gc, 0)];
      ((int32_t*)obs)[env] = v;
    } else {  // GP_OBS_WINDOW (observations.py:74-103)
      const int n = p.obs_n, nn = n * n, h = n / 2;
      uint8_t* o = (uint8_t*)obs + (size_t)env * nn;
      const uint8_t* wt = tab<uint8_t>(lds, p.off_window) + (size_t)ac * nn;
      for (int k = 0; k < nn; ++k) o[k] = wt[k];
      if (gvalid) {
        const int dy = gc / p.W - ac / p.W, dx = gc % p.W - ac % p.W;
        if (dy >= -h && dy <= n - 1 - h && dx >= -h && dx <= n - 1 - h) o[(dy + h) * n + (dx + h)] = 2;
      }
    }
  }
}

// Compile-time specialisation of the philox rollout (SPEC = 1: BASELINE configs[4]'s shape -- continuous float32
// (y, x) actions, no velocity, a fixed goal): these configuration fields become constants, so the step loop carries
// none of the other configurations' uniform branches, zero-initialisations or their SGPRs (the generic kernel
// spilled SGPRs to VGPR lanes inside the loop). SPEC = 0 reads them from the arguments.
template <int SPEC> __device__ __forceinline__ int cr_action_kind(const CrDev& p) { return SPEC ? 0 : p.action_kind; }
template <int SPEC> __device__ __forceinline__ bool cr_action_f64(const CrDev& p) { return SPEC ? false : p.action_f64 != 0; }
template <int SPEC> __device__ __forceinline__ bool cr_velocity(const CrDev& p) { return SPEC ? false : p.use_velocity != 0; }
template <int SPEC> __device__ __forceinline__ bool cr_goal_fixed(const CrDev& p) { return SPEC ? true : p.goal_fixed != 0; }

// reset of one env: goal then agent (crooms.py:217-244, 268-274)
template <int SPEC = 0>
__device__ __forceinline__ void reset_env(const CrDev& p, const uint8_t* lds, const Draws& d, double& ay, double& ax,
                                          double& vy, double& vx, uint32_t& g) {
  if (!cr_goal_fixed<SPEC>(p)) {
    const uint32_t yx = tab<uint32_t>(lds, p.off_valid)[d.gi];  // y | x << 16: no integer divide
    g = yx;
  }
  int cy, cx;
  double cs, hs;
  if (p.agent_fixed) {
    cy = p.agent_y; cx = p.agent_x;
    cs = p.cell; hs = p.half_cell;  // grid_to_coord(..., cell_size)
  } else {
    const uint32_t yx = tab<uint32_t>(lds, p.off_valid)[d.ai];
    cy = (int)(yx & 0xFFFFu); cx = (int)(yx >> 16);
    cs = 1.0; hs = 0.5;             // the random branch ignores cell_size (crooms.py:240-244)
  }
  ay = (double)cy * cs + hs;
  ax = (double)cx * cs + hs;
  vy = 0.0;
  vx = 0.0;
}

struct StepOut {
  float rew;
  uint8_t term, trunc, oob;
};

// One env-step of CRoomsEnv.step (crooms.py:276-331). DEFER: a terminated / truncated env is left for the
// caller to reset (its reset draws are not known yet; the exact mode's stream walk). wix (replay): the pair of
// the wall-noise buffer this env reads when it hits a wall (default: its own, env).
template <bool REPLAY, bool DEFER = false, int SPEC = 0>
__device__ __forceinline__ StepOut crooms_env_step(const CrDev& p, const uint8_t* lds, int env, bool live,
                                                   uint64_t step, double a0, double a1, int ad, double& ay,
                                                   double& ax, double& vy, double& vx, uint32_t& g, int32_t& el,
                                                   float& rsum, uint32_t& eps, uint32_t& lens, int wix = -1) {
  StepOut o;
  el += 1;
  Draws d;
  d.k53 = 0;
  d.gi = d.ai = 0;
  // _sample_action (crooms.py:175-198) * action_power (:288)
  double my, mx;
  // the action noise (one draw site for both action kinds, so the sampler is inlined once)
  Philox4 nblk;
  bool nhave = false;
  double ny = 0.0, nx = 0.0;
  if (live && (cr_action_kind<SPEC>(p) == 0 || p.action_std != 0.0))
    draw_normals<REPLAY>(p, env, step, 0, p.action_std, ny, nx, nblk, nhave);
  if (cr_action_kind<SPEC>(p) == 0) {
    my = a0 + ny;
    mx = a1 + nx;
  } else {
    if (live) draw_ints<REPLAY>(p, env, step, d);
    int a = ad;
    if (live && action_out_of_range(a, p.nact)) flag_bad_action(p.derr);  // IndexError in the reference
    if (a < 0) a += p.nact;                 // numpy negative indexing of action_matrix[a]
    a = min(max(a, 0), p.nact - 1);
    const uint64_t* thr = tab<uint64_t>(lds, p.off_thr) + a * p.nact;
    int e = 0;
    for (int j = 0; j < p.nact; ++j) e += (d.k53 > thr[j]) ? 1 : 0;
    e = min(e, p.nact - 1);
    const int o8 = p.nact == 4 ? 2 * e : e;  // ACTIONS_CARDINAL = ACTIONS_ORDINAL[::2]
    const int DY[8] = {-1, -1, 0, 1, 1, 1, 0, -1}, DX[8] = {0, 1, 1, 1, 0, -1, -1, -1};
    my = (double)DY[o8];
    mx = (double)DX[o8];
    if (p.action_std != 0.0) {
      my = my + ny;
      mx = mx + nx;
    }
  }
  if (p.action_power != 1.0) {  // uniform: x * 1.0 == x, so the default power skips two f64 multiplies
    my = my * p.action_power;
    mx = mx * p.action_power;
  }
  // _apply_action (crooms.py:300-331)
  double py, px;
  if (cr_velocity<SPEC>(p)) {
    vy = fmin(fmax(vy + my, -MAX_VELOCITY), MAX_VELOCITY);
    vx = fmin(fmax(vx + mx, -MAX_VELOCITY), MAX_VELOCITY);
    py = ay + vy;
    px = ax + vx;
  } else {
    py = ay + my;
    px = ax + mx;
  }
  py = fmin(fmax(py, 0.0), p.hi_y);
  px = fmin(fmax(px, 0.0), p.hi_x);
  const int pc = cell_of_nonneg(p, py, px);
  const bool oob = pc < 0 || tab<uint8_t>(lds, p.off_wall)[pc] != 0;
  o.oob = oob ? 1 : 0;
  if (!oob) {
    ay = py;
    ax = px;
  } else {
    // stay in the current square: c = grid_to_coord(coord_to_grid(agent)), agent = clip(c + n, c - cs/2, c + cs/2 - 1e-8)
    const double cy = floor(per_cell(p, ay)) * p.cell + p.half_cell;
    const double cx = floor(per_cell(p, ax)) * p.cell + p.half_cell;
    double wy = 0.0, wx = 0.0;
    if (live) draw_normals<REPLAY>(p, REPLAY && wix >= 0 ? wix : env, step, 1, 0.5, wy, wx, nblk, nhave);
    ay = fmin(fmax(cy + wy, cy - p.half_cell), (cy + p.half_cell) - 1e-8);
    ax = fmin(fmax(cx + wx, cx - p.half_cell), (cx + p.half_cell) - 1e-8);
    vy = 0.0;
    vx = 0.0;
  }
  // reward / termination (crooms.py:289-297)
  // the goal square's centre (a fixed goal's from the kernel arguments: uniform, no per-env conversion)
  const double gyc = cr_goal_fixed<SPEC>(p) ? p.gcy : (double)(int16_t)(g & 0xFFFF) + 0.5;
  const double gxc = cr_goal_fixed<SPEC>(p) ? p.gcx : (double)(int16_t)(g >> 16) + 0.5;
  const double dy = ay - gyc, dx = ax - gxc;
  const double s = dy * dy + dx * dx;
  o.term = s <= p.s_thr ? 1 : 0;
  o.rew = o.term ? p.r_goal : (oob ? p.r_wall : p.r_step);
  o.trunc = el > p.time_limit ? 1 : 0;
  if (!live) return o;
  rsum += o.rew;
  if (o.term | o.trunc) {
    eps += 1u;
    lens += (uint32_t)el;
    el = 0;
    if constexpr (!DEFER) {
      if (cr_action_kind<SPEC>(p) == 0) draw_ints<REPLAY>(p, env, step, d);
      reset_env<SPEC>(p, lds, d, ay, ax, vy, vx, g);
    }
  }
  return o;
}

// Per-block metrics into the block's own slot.
__device__ void cr_metrics(const CrDev& p, float rsum, uint32_t eps, uint32_t lens, uint32_t nst) {
  __shared__ float s_r[WAVES];
  __shared__ uint32_t s_e[WAVES], s_l[WAVES], s_n[WAVES];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    rsum += __shfl_xor(rsum, d, 64);
    eps += __shfl_xor(eps, d, 64);
    lens += __shfl_xor(lens, d, 64);
    nst += __shfl_xor(nst, d, 64);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { s_r[wid] = rsum; s_e[wid] = eps; s_l[wid] = lens; s_n[wid] = nst; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0.f;
    unsigned long long e = 0, l = 0, n = 0;
    for (int w = 0; w < WAVES; ++w) { r += s_r[w]; e += s_e[w]; l += s_l[w]; n += s_n[w]; }
    CrSlot& m = p.mslot[blockIdx.x];
    m.return_sum += (double)r;
    m.episodes += e;
    m.length_sum += l;
    m.env_steps += n;
  }
}

// ---- the rollout kernel: K steps for every env; 2 consecutive envs per thread ----
template <int OK, bool REPLAY, int SPEC = 0>
__global__ __launch_bounds__(TPB, GP_CR_WAVES) void crooms_rollout(CrDev p, int K, uint64_t step0, const void* __restrict__ act,
                                                      void* __restrict__ obs, float* __restrict__ rew,
                                                      uint8_t* __restrict__ term, uint8_t* __restrict__ trunc) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  stage_tables(p, lds);
  __syncthreads();
  float rsum = 0.f;
  uint32_t eps = 0, lens = 0, nst = 0;
  for (int tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
    const int env0 = tile * EPB + threadIdx.x * EPT;
    double ay[EPT], ax[EPT], vy[EPT], vx[EPT];
    uint32_t g[EPT];
    int32_t el[EPT];
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int env = env0 + i;
      const bool live = env < p.B;
      ay[i] = live ? p.ay[env] : 0.5;
      ax[i] = live ? p.ax[env] : 0.5;
      vy[i] = (live && cr_velocity<SPEC>(p)) ? p.vy[env] : 0.0;
      vx[i] = (live && cr_velocity<SPEC>(p)) ? p.vx[env] : 0.0;
      g[i] = live ? (cr_goal_fixed<SPEC>(p) ? ((uint32_t)(p.goal_y & 0xFFFF) | ((uint32_t)(p.goal_x & 0xFFFF) << 16))
                                  : p.goal[env])
                  : 0u;
      el[i] = live ? p.el[env] : 0;
    }
    for (int k = 0; k < K; ++k) {
      const size_t off = (size_t)k * p.B;
      const uint64_t stp = step0 + (uint64_t)k;
      double a0[EPT], a1[EPT];
      int ad[EPT];
      const bool full = env0 + EPT - 1 < p.B && (off & 1) == 0;  // pair-aligned rew / flag stores
#pragma unroll
      for (int i = 0; i < EPT; ++i) { a0[i] = a1[i] = 0.0; ad[i] = 0; }
      if (cr_action_kind<SPEC>(p) == 0) {
        if (cr_action_f64<SPEC>(p)) {
          const double* A = (const double*)act + 2 * (off + env0);
#pragma unroll
          for (int i = 0; i < EPT; ++i)
            if (env0 + i < p.B) {
              const double2 q = *reinterpret_cast<const double2*>(A + 2 * i);
              a0[i] = q.x;
              a1[i] = q.y;
            }
        } else {
          const float* A = (const float*)act + 2 * (off + env0);
          if (full) {  // both envs' (y, x) in one 16-B load
            const float4 q = *reinterpret_cast<const float4*>(A);
            a0[0] = q.x; a1[0] = q.y; a0[1] = q.z; a1[1] = q.w;
          } else {
#pragma unroll
            for (int i = 0; i < EPT; ++i)
              if (env0 + i < p.B) {
                const float2 q = *reinterpret_cast<const float2*>(A + 2 * i);
                a0[i] = q.x;
                a1[i] = q.y;
              }
          }
        }
      } else {
        const int32_t* A = (const int32_t*)act + off + env0;
        if (full) {
          const int2 q = *reinterpret_cast<const int2*>(A);
          ad[0] = q.x; ad[1] = q.y;
        } else {
          for (int i = 0; i < EPT; ++i)
            if (env0 + i < p.B) ad[i] = A[i];
        }
      }
      float r[EPT];
      uint8_t tm[EPT], tr[EPT];
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        const int env = env0 + i;
        const bool live = env < p.B;
        StepOut o = crooms_env_step<REPLAY, false, SPEC>(p, lds, env, live, stp, a0[i], a1[i], ad[i], ay[i], ax[i],
                                            vy[i], vx[i], g[i], el[i], rsum, eps, lens);
        r[i] = o.rew;
        tm[i] = o.term;
        tr[i] = o.trunc;
        nst += live ? 1u : 0u;
      }
      if (full) {
        *reinterpret_cast<float2*>(rew + off + env0) = make_float2(r[0], r[1]);
        *reinterpret_cast<uint16_t*>(term + off + env0) = (uint16_t)(tm[0] | (tm[1] << 8));
        *reinterpret_cast<uint16_t*>(trunc + off + env0) = (uint16_t)(tr[0] | (tr[1] << 8));
      } else {
        for (int i = 0; i < EPT; ++i)
          if (env0 + i < p.B) { rew[off + env0 + i] = r[i]; term[off + env0 + i] = tm[i]; trunc[off + env0 + i] = tr[i]; }
      }
      const size_t ob = (size_t)k * p.B * (size_t)p.obs_width * (OK == GP_OBS_F32 ? ((SPEC == 0 && p.obs_f64) ? 8 : 4)
                                                                   : (OK == GP_OBS_HANSEN || OK == GP_OBS_TABLE ? 4 : 1));
      if (OK == GP_OBS_F32 && (SPEC == 1 || !p.obs_f64) && p.obs_width == 2 && full) {
        // vector_mdp (configs[4]): both envs' float32 (y, x) in one 16-B store
        *reinterpret_cast<float4*>((float*)((uint8_t*)obs + ob) + 2 * (size_t)env0) =
            make_float4((float)ay[0], (float)ax[0], (float)ay[1], (float)ax[1]);
      } else {
#pragma unroll
        for (int i = 0; i < EPT; ++i)
          if (env0 + i < p.B) write_obs<OK>(p, lds, env0 + i, ay[i], ax[i], g[i], (uint8_t*)obs + ob);
      }
    }
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int env = env0 + i;
      if (env >= p.B) continue;
      p.ay[env] = ay[i];
      p.ax[env] = ax[i];
      if (cr_velocity<SPEC>(p)) { p.vy[env] = vy[i]; p.vx[env] = vx[i]; }
      if (!cr_goal_fixed<SPEC>(p)) p.goal[env] = g[i];
      p.el[env] = el[i];
    }
  }
  cr_metrics(p, rsum, eps, lens, nst);
}

// reset(): goal then agent for every env (crooms.py:251-266).
template <int OK, bool REPLAY>
__global__ __launch_bounds__(TPB) void crooms_reset(CrDev p, uint64_t step, void* __restrict__ obs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  stage_tables(p, lds);
  __syncthreads();
  for (int env = blockIdx.x * TPB + threadIdx.x; env < p.B; env += gridDim.x * TPB) {
    Draws d;
    draw_ints<REPLAY>(p, env, step, d);
    double ay, ax, vy, vx;
    uint32_t g = (uint32_t)(p.goal_y & 0xFFFF) | ((uint32_t)(p.goal_x & 0xFFFF) << 16);
    reset_env(p, lds, d, ay, ax, vy, vx, g);
    p.ay[env] = ay;
    p.ax[env] = ax;
    if (p.use_velocity) { p.vy[env] = 0.0; p.vx[env] = 0.0; }
    if (!p.goal_fixed) p.goal[env] = g;
    p.el[env] = 0;
    write_obs<OK>(p, lds, env, ay, ax, g, obs);
  }
}

__global__ void crooms_get_state(CrDev p, double* agent, int32_t* goal, double* vel, int32_t* el) {
  const int env = blockIdx.x * TPB + threadIdx.x;
  if (env >= p.B) return;
  if (agent) { agent[2 * env] = p.ay[env]; agent[2 * env + 1] = p.ax[env]; }
  if (goal) {
    const uint32_t g = p.goal_fixed ? ((uint32_t)(p.goal_y & 0xFFFF) | ((uint32_t)(p.goal_x & 0xFFFF) << 16)) : p.goal[env];
    goal[2 * env] = (int16_t)(g & 0xFFFF);
    goal[2 * env + 1] = (int16_t)(g >> 16);
  }
  if (vel) {
    vel[2 * env] = p.use_velocity ? p.vy[env] : 0.0;
    vel[2 * env + 1] = p.use_velocity ? p.vx[env] : 0.0;
  }
  if (el) el[env] = p.el[env];
}
__global__ void crooms_set_state(CrDev p, const double* agent, const int32_t* goal, const double* vel,
                                 const int32_t* el) {
  const int env = blockIdx.x * TPB + threadIdx.x;
  if (env >= p.B) return;
  if (agent) { p.ay[env] = agent[2 * env]; p.ax[env] = agent[2 * env + 1]; }
  if (goal && !p.goal_fixed)
    p.goal[env] = (uint32_t)(goal[2 * env] & 0xFFFF) | ((uint32_t)(goal[2 * env + 1] & 0xFFFF) << 16);
  if (vel && p.use_velocity) { p.vy[env] = vel[2 * env]; p.vx[env] = vel[2 * env + 1]; }
  if (el) p.el[env] = min(max(el[env], 0), 0x7FFFFFFF);
}

// ---- exact (numpy-stream) mode: GP_RNG_NUMPY ----
// The reference's draws, word for word, from its one PCG64 stream (crooms.py:175-198, :300-331,
// :217-244): per step rng.random(B) (discrete actions), rng.normal(scale=action_std, size=(B, 2)),
// rng.normal(scale=0.5, size=(n_oob, 2)) for the envs that hit a wall, then choice() of the reset envs'
// goals and agents. numpy's normal consumes a data-dependent number of words (ziggurat fast path 1 word,
// wedge 2, tail 1 + 2k) and choice() draws buffered 32-bit halves with Lemire rejection, so the word ->
// draw assignment is resolved in windows of XW words: every thread makes one word (a table jump from the
// window base), classifies it on the fast path, one thread walks the few (~1.2%) slow positions in order
// (marking the extra words they consume), and a ballot prefix over the surviving positions gives each
// draw its index. One workgroup runs the whole batch (meant for seed-identical runs at small B); the step
// itself is crooms_env_step<true> (the replay step, fixture-pinned) on the per-env draws, evaluated dry to
// learn the wall hits and the resets that decide the later draw counts.
constexpr int XT = 1024;           // threads of the exact-mode workgroup
constexpr int XW = XT;             // words per window, one per thread
constexpr int XWAVES = XT / 64;

struct CrRng {
  uint64_t s_hi, s_lo, i_hi, i_lo;
  uint32_t has_u32, uinteger, err, pad;
};

struct CrExact {
  CrRng* rng;
  const PcgJump* wj;               // wj[j]: j LCG steps, j = 0..XW
  double* noise;                   // [B, 2] action noise, per env
  double* wall;                    // [B, 2] wall noise, per env
  double* dense;                   // [2B] draws in stream order
  uint64_t* u;                     // [B] action-failure k53
  int32_t* gi;                     // [B] goal / agent indices into valid_states, per env
  int32_t* ai;
  int32_t* rank;                   // [B] scratch: rank of an env among the flagged ones, or -1
  uint32_t lemire_thr;             // (2^32 - n_valid) % n_valid
};

struct XShared {
  uint64_t w[XW];
  double sval[XW];
  uint64_t zt[768];
  uint64_t slow[XWAVES];
  uint32_t wtot[XWAVES], wtot2[XWAVES];
  uint8_t dead[XW], sacc[XW];
  uint16_t sused[XW];
  uint64_t st_hi, st_lo;
  uint32_t has_u32, uinteger, err;
  int wend, endpos, total;
};

__device__ __forceinline__ u128 x_state(const XShared& sh) { return mk128(sh.st_hi, sh.st_lo); }
// The window base moves past the n words consumed: thread n - 1 holds that jump (wj[n]) in registers.
// Call between barriers, after every thread has read the base.
__device__ __forceinline__ void x_advance(XShared& sh, const PcgJump& myj, int n) {
  if (n > 0 && (int)threadIdx.x == n - 1) {
    const u128 s = apply_jump(myj, x_state(sh));
    sh.st_hi = hi64(s);
    sh.st_lo = lo64(s);
  }
}

// Exclusive rank of `f` among the XT threads (ballot per wave, wave totals in LDS); returns the total.
__device__ __forceinline__ int x_rank(XShared& sh, uint32_t f, int& rank) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t b = __ballot(f != 0);
  if (lane == 0) sh.wtot[wv] = (uint32_t)__popcll(b);
  __syncthreads();
  int base = 0, tot = 0;
  for (int i = 0; i < XWAVES; ++i) {
    base += i < wv ? (int)sh.wtot[i] : 0;
    tot += (int)sh.wtot[i];
  }
  rank = base + __popcll(b & ((1ull << lane) - 1ull));
  __syncthreads();
  return tot;
}

// One attempt of numpy's ziggurat starting at window position q whose first word missed the fast path:
// 1 = a normal (value v), 0 = a rejected wedge (the next attempt starts at q + used), -1 = it would read
// past the window (the window ends at q).
__device__ int zig_attempt(const ZigTabs& t, const uint64_t* w, int q, int& used, double& v) {
  uint64_t r = w[q];
  int pos = q + 1;
  const int idx = (int)(r & 0xff);
  r >>= 8;
  const uint64_t sign = r & 1u, rabs = (r >> 1) & 0x000fffffffffffffull;
  double x = (double)rabs * t.wi[idx];
  if (sign) x = -x;
  if (rabs < t.ki[idx]) { used = 1; v = x; return 1; }
  if (idx == 0) {
    for (;;) {
      if (pos + 1 >= XW) return -1;
      const double xx = -GP_ZIG_INV_R * zlog1p_neg(u53_of(w[pos]));
      const double yy = -zlog1p_neg(u53_of(w[pos + 1]));
      pos += 2;
      if (yy + yy > xx * xx) {
        used = pos - q;
        v = ((rabs >> 8) & 1u) ? -(GP_ZIG_R + xx) : GP_ZIG_R + xx;
        return 1;
      }
    }
  }
  if (pos >= XW) return -1;
  used = 2;
  v = x;
  return ((t.fi[idx - 1] - t.fi[idx]) * u53_of(w[pos]) + t.fi[idx] < zexp(-0.5 * x * x)) ? 1 : 0;
}

// n draws of rng.normal(scale=scale) (numpy: loc + scale * standard_normal, loc = 0) into dst[0..n).
__device__ void x_normals(XShared& sh, const CrExact& x, const PcgJump& myj, int64_t n, double scale,
                          double* __restrict__ dst) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  ZigTabs zt;
  zt.ki = sh.zt;
  zt.wi = reinterpret_cast<const double*>(sh.zt + 256);
  zt.fi = reinterpret_cast<const double*>(sh.zt + 512);
  int64_t made = 0;
  while (made < n) {
    const uint64_t w = pcg_output(apply_jump(myj, x_state(sh)));
    sh.w[t] = w;
    sh.dead[t] = 0;
    double z;
    const bool fast = zig_fast(zt, w, z);
    const uint64_t sm = __ballot(!fast);
    if (lane == 0) sh.slow[wv] = sm;
    __syncthreads();
    if (!fast) {  // the attempt this word would start (speculative: it may be an extra word of another)
      int used = 1;
      double v = 0.0;
      const int a = zig_attempt(zt, sh.w, t, used, v);
      sh.sval[t] = v;
      sh.sacc[t] = (uint8_t)(a < 0 ? 2 : a);
      sh.sused[t] = (uint16_t)used;
    }
    __syncthreads();
    if (t == 0) {  // the chain over the slow positions, in order
      int cur = 0, wend = XW;
      for (int i = 0; i < XWAVES && wend == XW; ++i) {
        uint64_t m = sh.slow[i];
        while (m) {
          const int q = i * 64 + __builtin_ctzll(m);
          m &= m - 1;
          if (q < cur) continue;  // an extra word of an earlier attempt
          if (sh.sacc[q] == 2) { wend = q; break; }
          const int used = sh.sused[q];
          for (int j = q + 1; j < q + used; ++j) sh.dead[j] = 1;
          cur = q + used;
        }
      }
      if (wend == 0) sh.err = 1u;  // a tail attempt longer than a window (never in practice): drain
      sh.wend = wend;
      sh.endpos = -1;
    }
    __syncthreads();
    if (sh.err) return;
    const int wend = sh.wend;
    const bool prod = t < wend && !sh.dead[t] && (fast || sh.sacc[t]);
    const double v = fast ? z : sh.sval[t];
    const int used = fast ? 1 : (int)sh.sused[t];
    int rank;
    const int tot = x_rank(sh, prod, rank);
    if (prod && made + rank < n) dst[made + rank] = 0.0 + scale * v;
    if (prod && made + rank == n - 1) sh.endpos = t + used;
    __syncthreads();
    const int consumed = (made + tot >= n) ? sh.endpos : wend;
    made += (made + tot >= n) ? (n - made) : tot;
    x_advance(sh, myj, consumed);
    __syncthreads();
  }
}

// n draws of rng.random() into k53 form (next_double = (w >> 11) * 2^-53; the integer is kept).
__device__ void x_uniforms(XShared& sh, const CrExact& x, const PcgJump& myj, int64_t n, uint64_t* __restrict__ dst) {
  const int t = threadIdx.x;
  for (int64_t made = 0; made < n; made += XW) {
    const uint64_t w = pcg_output(apply_jump(myj, x_state(sh)));
    if (made + t < n) dst[made + t] = w >> 11;
    __syncthreads();
    x_advance(sh, myj, (int)min((int64_t)XW, n - made));
    __syncthreads();
  }
}

// n draws of rng.choice(valid_states) as indices: integers(0, n_valid) -> 32-bit Lemire on next_uint32,
// whose high halves are buffered in the bit generator (has_uint32 / uinteger) across calls.
__device__ void x_choices(XShared& sh, const CrExact& x, const PcgJump& myj, int64_t n, uint32_t nv,
                          int32_t* __restrict__ dst) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  int64_t made = 0;
  while (made < n) {
    const uint32_t h = sh.has_u32;
    const uint64_t w = pcg_output(apply_jump(myj, x_state(sh)));
    const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
    const bool ab = t == 0 && h && !lemire_rejected(sh.uinteger, nv, x.lemire_thr);
    const bool alo = !lemire_rejected(lo, nv, x.lemire_thr), ahi = !lemire_rejected(hi, nv, x.lemire_thr);
    const uint32_t c = (ab ? 1u : 0u) + (alo ? 1u : 0u) + (ahi ? 1u : 0u);  // 0..3
    const uint64_t b0 = __ballot(c & 1u), b1 = __ballot(c & 2u);
    const uint64_t lt = (1ull << lane) - 1ull;
    if (lane == 0) { sh.wtot[wv] = (uint32_t)__popcll(b0); sh.wtot2[wv] = (uint32_t)__popcll(b1); }
    if (t == 0) sh.endpos = -1;
    __syncthreads();
    int base = 0, tot = 0;
    for (int i = 0; i < XWAVES; ++i) {
      const int wc = (int)sh.wtot[i] + 2 * (int)sh.wtot2[i];
      base += i < wv ? wc : 0;
      tot += wc;
    }
    int r = base + __popcll(b0 & lt) + 2 * __popcll(b1 & lt);
    // candidates in stream order: the buffered half (thread 0), then lo, hi of each word; endpos codes the
    // last candidate consumed: 0 = the buffered half, 2t + 1 = lo of word t, 2t + 2 = hi of word t
    if (ab) {
      if (made + r < n) dst[made + r] = (int32_t)lemire_value(sh.uinteger, nv);
      if (made + r == n - 1) sh.endpos = 0;
      ++r;
    }
    if (alo) {
      if (made + r < n) dst[made + r] = (int32_t)lemire_value(lo, nv);
      if (made + r == n - 1) sh.endpos = 2 * t + 1;
      ++r;
    }
    if (ahi) {
      if (made + r < n) dst[made + r] = (int32_t)lemire_value(hi, nv);
      if (made + r == n - 1) sh.endpos = 2 * t + 2;
    }
    __syncthreads();
    const int e = (made + tot >= n) ? sh.endpos : 2 * XW;
    const int words = (e + 1) / 2;                  // lo of word t -> t + 1 words, hi -> t + 1 words
    // numpy's next_uint32 stores the high half of every word it draws (uinteger) and keeps it after
    // handing it out; has_uint32 says whether it is still unused (the last word's lo was the last draw)
    if (words > 0 && t == words - 1) sh.uinteger = hi;
    __syncthreads();
    if (t == 0) sh.has_u32 = (e & 1) ? 1u : 0u;
    x_advance(sh, myj, words);
    made += (made + tot >= n) ? (n - made) : tot;
    __syncthreads();
  }
}

__device__ __forceinline__ void x_load_action(const CrDev& p, const void* act, size_t off, int env, double& a0,
                                              double& a1, int& ad) {
  a0 = a1 = 0.0;
  ad = 0;
  if (p.action_kind == 0) {
    if (p.action_f64) {
      const double* A = (const double*)act + 2 * (off + env);
      a0 = A[0];
      a1 = A[1];
    } else {
      const float* A = (const float*)act + 2 * (off + env);
      a0 = A[0];
      a1 = A[1];
    }
  } else {
    ad = ((const int32_t*)act)[off + env];
  }
}

__device__ __forceinline__ uint32_t x_goal(const CrDev& p, int env) {
  return p.goal_fixed ? ((uint32_t)(p.goal_y & 0xFFFF) | ((uint32_t)(p.goal_x & 0xFFFF) << 16)) : p.goal[env];
}

// Scatter dense[2 rank + j] -> per[2 env + j] (W = 2) or dense[rank] -> per[env] (W = 1) for flagged envs.
template <int W, class T>
__device__ __forceinline__ void x_scatter(const CrDev& p, const CrExact& x, const T* dense, T* per) {
  for (int env = threadIdx.x; env < p.B; env += XT) {
    const int r = x.rank[env];
    if (r >= 0)
      for (int j = 0; j < W; ++j) per[(size_t)W * env + j] = dense[(size_t)W * r + j];
  }
}

// Ranks of the flagged envs (x.rank, -1 when unflagged) over all B envs; returns the count.
template <class F>
__device__ int x_rank_envs(XShared& sh, const CrDev& p, const CrExact& x, F&& flag) {
  int base = 0;
  for (int e0 = 0; e0 < p.B; e0 += XT) {
    const int env = e0 + threadIdx.x;
    const bool f = env < p.B && flag(env);
    int r;
    const int tot = x_rank(sh, f, r);
    if (env < p.B) x.rank[env] = f ? base + r : -1;
    base += tot;
  }
  __syncthreads();
  return base;
}

// K steps (or, with K = 0 and do_reset, reset()) of the whole batch in one workgroup.
template <int OK>
__global__ __launch_bounds__(XT) void crooms_numpy_rollout(CrDev p, CrExact x, int K, int do_reset,
                                                           const void* __restrict__ act, void* __restrict__ obs,
                                                           float* __restrict__ rew, uint8_t* __restrict__ term,
                                                           uint8_t* __restrict__ trunc) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ XShared sh;
  const int t = threadIdx.x;
  const PcgJump myj = x.wj[t + 1];  // every window: word t is t + 1 LCG steps past the window base
  for (int i = t; i < p.tab_bytes / 16; i += XT) ((uint4*)lds)[i] = ((const uint4*)p.tabs)[i];
  for (int i = t; i < 768; i += XT) sh.zt[i] = d_zig[i];
  if (t == 0) {
    sh.st_hi = x.rng->s_hi;
    sh.st_lo = x.rng->s_lo;
    sh.has_u32 = x.rng->has_u32;
    sh.uinteger = x.rng->uinteger;
    sh.err = x.rng->err;
  }
  __syncthreads();
  const size_t osz = (size_t)p.obs_width * (OK == GP_OBS_F32 ? (p.obs_f64 ? 8 : 4)
                                                             : (OK == GP_OBS_HANSEN || OK == GP_OBS_TABLE ? 4 : 1));
  if (do_reset && !sh.err) {  // crooms.py:251-266: goal then agent for every env
    if (!p.goal_fixed) x_choices(sh, x, myj, p.B, (uint32_t)p.n_valid, x.gi);
    if (!p.agent_fixed && !sh.err) x_choices(sh, x, myj, p.B, (uint32_t)p.n_valid, x.ai);
    for (int env = t; env < p.B; env += XT) {
      Draws d;
      d.k53 = 0;
      d.gi = p.goal_fixed ? 0u : (uint32_t)x.gi[env];
      d.ai = p.agent_fixed ? 0u : (uint32_t)x.ai[env];
      double ay, ax, vy, vx;
      uint32_t g = x_goal(p, 0);
      reset_env(p, lds, d, ay, ax, vy, vx, g);
      p.ay[env] = ay;
      p.ax[env] = ax;
      if (p.use_velocity) { p.vy[env] = 0.0; p.vx[env] = 0.0; }
      if (!p.goal_fixed) p.goal[env] = g;
      p.el[env] = 0;
      write_obs<OK>(p, lds, env, ay, ax, g, obs);
    }
  }
  // p.rp_* point at the per-env draw buffers (x.u / gi / ai / noise / wall), set by the host
  float rsum = 0.f;
  uint32_t eps = 0, lens = 0, nst = 0;
  for (int k = 0; k < K && !sh.err; ++k) {
    const size_t off = (size_t)k * p.B;
    // _sample_action's draws (crooms.py:175-198)
    if (p.action_kind != 0) x_uniforms(sh, x, myj, p.B, x.u);
    if (p.action_kind == 0 || p.action_std != 0.0) x_normals(sh, x, myj, 2 * (int64_t)p.B, p.action_std, x.noise);
    __syncthreads();
    // the dry step on copies: which envs hit a wall (draw count of the wall noise, crooms.py:321-325)
    auto dry = [&](int env, StepOut& o) {
      double a0, a1;
      int ad;
      x_load_action(p, act, off, env, a0, a1, ad);
      double ay = p.ay[env], ax = p.ax[env];
      double vy = p.use_velocity ? p.vy[env] : 0.0, vx = p.use_velocity ? p.vx[env] : 0.0;
      uint32_t g = x_goal(p, env);
      int32_t el = p.el[env];
      float rs = 0.f;
      uint32_t ep = 0, ln = 0;
      o = crooms_env_step<true>(p, lds, env, true, 0, a0, a1, ad, ay, ax, vy, vx, g, el, rs, ep, ln);
    };
    const int n_oob = x_rank_envs(sh, p, x, [&](int env) { StepOut o; dry(env, o); return o.oob != 0; });
    if (n_oob) {
      x_normals(sh, x, myj, 2 * (int64_t)n_oob, 0.5, x.dense);
      __syncthreads();
      x_scatter<2>(p, x, x.dense, x.wall);
      __syncthreads();
    }
    // the step itself with the wall noise in place (crooms.py:276-298), resets deferred: which envs reset
    uint8_t* ob = (uint8_t*)obs + (size_t)k * p.B * osz;
    const int n_rs = x_rank_envs(sh, p, x, [&](int env) {
      double a0, a1;
      int ad;
      x_load_action(p, act, off, env, a0, a1, ad);
      double ay = p.ay[env], ax = p.ax[env];
      double vy = p.use_velocity ? p.vy[env] : 0.0, vx = p.use_velocity ? p.vx[env] : 0.0;
      uint32_t g = x_goal(p, env);
      int32_t el = p.el[env];
      const StepOut o =
          crooms_env_step<true, true>(p, lds, env, true, 0, a0, a1, ad, ay, ax, vy, vx, g, el, rsum, eps, lens);
      ++nst;
      rew[off + env] = o.rew;
      term[off + env] = o.term;
      trunc[off + env] = o.trunc;
      const bool rs = (o.term | o.trunc) != 0;
      if (!rs) {
        write_obs<OK>(p, lds, env, ay, ax, g, ob);
        p.ay[env] = ay;
        p.ax[env] = ax;
        if (p.use_velocity) { p.vy[env] = vy; p.vx[env] = vx; }
      }
      p.el[env] = el;
      return rs;
    });
    // the resetting envs' goals then agents (crooms.py:217-244, 293-297), in env order
    if (n_rs) {
      int32_t* di = (int32_t*)x.dense;
      if (!p.goal_fixed) {
        x_choices(sh, x, myj, n_rs, (uint32_t)p.n_valid, di);
        __syncthreads();
        x_scatter<1>(p, x, di, x.gi);
        __syncthreads();
      }
      if (!p.agent_fixed) {
        x_choices(sh, x, myj, n_rs, (uint32_t)p.n_valid, di);
        __syncthreads();
        x_scatter<1>(p, x, di, x.ai);
        __syncthreads();
      }
      for (int env = t; env < p.B; env += XT) {
        if (x.rank[env] < 0) continue;
        Draws d;
        d.k53 = 0;
        d.gi = p.goal_fixed ? 0u : (uint32_t)x.gi[env];
        d.ai = p.agent_fixed ? 0u : (uint32_t)x.ai[env];
        double ay, ax, vy, vx;
        uint32_t g = x_goal(p, env);
        reset_env(p, lds, d, ay, ax, vy, vx, g);
        p.ay[env] = ay;
        p.ax[env] = ax;
        if (p.use_velocity) { p.vy[env] = 0.0; p.vx[env] = 0.0; }
        if (!p.goal_fixed) p.goal[env] = g;
        write_obs<OK>(p, lds, env, ay, ax, g, ob);
      }
    }
    if (sh.err) break;
    __syncthreads();
  }
  // metrics into slot 0
  __shared__ float m_r;
  __shared__ unsigned long long m_e, m_l, m_n;
  if (t == 0) { m_r = 0.f; m_e = m_l = m_n = 0; }
  __syncthreads();
  for (int d = 32; d >= 1; d >>= 1) {
    rsum += __shfl_xor(rsum, d, 64);
    eps += __shfl_xor(eps, d, 64);
    lens += __shfl_xor(lens, d, 64);
    nst += __shfl_xor(nst, d, 64);
  }
  if ((t & 63) == 0) {
    atomicAdd(&m_r, rsum);
    atomicAdd(&m_e, (unsigned long long)eps);
    atomicAdd(&m_l, (unsigned long long)lens);
    atomicAdd(&m_n, (unsigned long long)nst);
  }
  __syncthreads();
  if (t == 0) {
    CrSlot& m = p.mslot[0];
    m.return_sum += (double)m_r;
    m.episodes += m_e;
    m.length_sum += m_l;
    m.env_steps += m_n;
    x.rng->s_hi = sh.st_hi;
    x.rng->s_lo = sh.st_lo;
    x.rng->has_u32 = sh.has_u32;
    x.rng->uinteger = sh.uinteger;
    x.rng->err = sh.err;
  }
}

// ---- exact (numpy-stream) mode, multi-workgroup (B > XG_MIN_ENVS) ----
// The same stream, call for call, resolved over ALL positions of a draw call at once instead of window by window:
// each draw call is a short sequence of grid-wide kernels on the stream (no workgroup walks the stream), with
// the call's stream state in one of two slots (read slot rd, written slot wr = the state after the call).
//   normal(n): position q holds word q (= output of jump(S, q + 1)). A position is "slow" when its word misses
//     the ziggurat fast path (~1.2%); the attempt it would start uses span(q) words (wedge 2, tail 1 + 2k) and
//     may be rejected (a wedge: the chain continues at q + 2). The chain of attempts from position 0 visits
//     every position except the extra words of the on-chain slow attempts, so a position's fate only depends
//     on the slow attempts just before it: each block evaluates the attempts of its positions and of a halo of
//     XG_LOOK positions before them in LDS, walks every slow position back to the start of its cluster (the
//     first slow attempt not spanned by an earlier one; clusters are almost always that one attempt) and
//     forward through it (list ranking by clusters, no serial walk over the call), and counts its produced
//     positions (on-chain and accepted). The next kernel gives every normal its index from those counts (a
//     reduce-then-scan over the call: no block waits on another), and the n-th normal's end is the words used.
//   choice(n): candidates are the buffered half (if any), then lo / hi of each word; a candidate is drawn
//     unless Lemire rejects it (~n / 2^32): counted per block, then indexed the same way; the last draw fixes
//     has_uint32 / uinteger.
//   env phases (dry step -> wall hits, real step -> resets, applying the resets) are per-env kernels that
//     publish a bitmap of their flagged envs and per-block counts; a later phase finds a flagged env's rank
//     (its index into the draws of the call that serves it: the wall noise, the reset choices) from them.
// Counts: every producer block stores its count, and adds (1 << 40 | count) to its group's (64 blocks)
// accumulator; the group's last arriver writes the group sum and clears the accumulator for the next launch.
// A consumer's prefix for block b is the sum of the group sums before b's group and of the counts of the blocks
// before b in it (at most 256 + 63 loads per block, all independent).
constexpr int XGT = 256;          // threads (positions / envs) per block of the grid kernels
constexpr int XGW = XGT / 64;     // waves (bitmap words) per block
constexpr int XG_LOOK = 64;       // the halo of a normal call's block view (one wave)
constexpr int XG_SPAN = 32;       // longest slow attempt (a 15-pair tail; else GP_DERR_STREAM)
constexpr int XG_MIN_ENVS = 1024; // at or below: the one-workgroup kernel (measured crossover)
#ifndef XG_SPLIT_NORMALS
#define XG_SPLIT_NORMALS 0        // 1: normal / choice calls as two launches each (count, then write; round 3's form)
#endif
// Above this many envs a call goes back to two launches (the fused kernel's in-launch prefix is a chain over every
// earlier block). A/B on MI355X, µs/step fused vs two launches: before the round-4 state loads and the
// wall-noise extension 568 vs 569 at 2^20 and 1035 vs 970 at 2^21; after them 571-576 vs 597 at 2^21.
#ifndef XG_FUSE_MAX_ENVS
#define XG_FUSE_MAX_ENVS 2097152
#endif

// GP_STAMPS diagnostic builds (tools/xstamps.py): s_memrealtime stamps (100 MHz, chip-synchronous) by thread 0 of
// blocks < 1024, per kernel kind (0 action normals, 1 dry step, 2 wall normals, 3 step, 4 choices, 5 resets),
// overwritten by every launch of that kind (the last step of a rollout is what is read back).
#ifdef GP_STAMPS
__device__ unsigned long long* g_xgdbg;
#define XSTAMP(ty, i)                                                                                    \
  do {                                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < 1024) {                                                         \
      unsigned long long t_;                                                                             \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                     \
      g_xgdbg[((size_t)(ty) * 1024 + blockIdx.x) * 8 + (i)] = t_;                                        \
    }                                                                                                    \
  } while (0)
#else
#define XSTAMP(ty, i) \
  do {                \
  } while (0)
#endif

struct XgCounts {                 // per-block counts of one producer launch
  uint32_t* bc;                   // [blocks] block counts
  unsigned long long* acc;        // [groups] arrivals << 40 | count sum (zero between launches)
  uint32_t* gs;                   // [groups] group sums (64 blocks per group)
};

struct XgFlags {                  // the flagged envs of one env phase
  uint64_t* bits;                 // [blocks * XGW] bitmap (nullptr: every env, ranked by env index)
  XgCounts c;
};

struct XgCall {                   // one draw call over stream positions
  const PcgJump* jt;              // radix-64 jump tables (JT_LEVELS x 64)
  const PcgJump* wj;              // wj[j]: j LCG steps (j <= XGT)
  CrRng* st;                      // stream-state slots [2]
  int rd, wr;
  XgCounts nsrc;                  // n = nmul * (flagged envs of a phase) when nsrc.gs is set, else n_host
  int nsrc_blocks;
  int nmul;
  int64_t n_host;
  int P;                          // capacity in positions
  uint64_t* bits;                 // normal: slow-position bitmap [P / 64]
  uint64_t* pbits;                // normal: produced-position bitmap [P / 64]
  uint64_t* bstate;               // [P / XGT][2] the call's state jumped to each block's first position
  uint16_t* span;                 // per slow position: words of its attempt
  double* val;                    // per slow position: the attempt's normal
  XgCounts pc;                    // per-block counts of produced normals / drawn choices
  double scale;                   // normal: dst[r] = loc 0 + scale * z (r: the normal's index in the call)
  double* dst;
  int32_t* idst;                  // choice: idst[r]
  uint32_t nv, lthr;              // choice: values, Lemire threshold
  uint32_t* err;                  // device error word (GP_DERR_STREAM)
  // the fused normal call (xg_norm_fused): tagged per-block counts and 64-block group sums of THIS launch
  unsigned long long* tbc;        // [blocks] tag << 32 | produced count
  unsigned long long* tgs;        // [groups] tag << 32 | group sum (written by the group's last arriver)
  unsigned long long* tacc;       // [groups] arrivals << 40 | count sum (zero between launches)
  uint32_t tag;                   // this launch's tag (never 0)
  // the wall-noise extension (round 4): the action-noise call (xinfo set) goes on to draw up to xmax more
  // normals, scaled by xscale, into xdst with each one's end position (from the call's start) in xend and the
  // count made in xinfo[0]; the wall-noise call (xg_wall_one) then only sets the stream state when its n <=
  // xinfo[0], and records its n in xinfo[1] (the next extension asks for 5/4 of it + 1024)
  double* xdst;
  uint32_t* xend;
  uint32_t* xinfo;
  uint32_t xmax;
  double xscale;
  const PcgJump* bj;              // [blocks + 1] jump by bid * XGT positions (nullptr: the radix tables)
  const PcgJump* hj;              // [blocks + 1] jump by bid * XGT - XG_LOOK (bid >= 1): a block's halo
};

// Block-wide sum (every thread gets it). Uses its own LDS; safe to call repeatedly.
__device__ __forceinline__ uint32_t xg_block_sum(uint32_t x) {
  __shared__ uint32_t ws[XGW];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = x;
  __syncthreads();
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < XGW; ++i) s += ws[i];
  __syncthreads();
  return s;
}
// Block-wide exclusive scan of small per-thread counts: this thread's offset, the block total in tot.
__device__ __forceinline__ uint32_t xg_block_scan(uint32_t c, uint32_t& tot) {
  __shared__ uint32_t ws[XGW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t x = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) ws[wv] = x;
  __syncthreads();
  uint32_t base = 0;
  tot = 0;
#pragma unroll
  for (int i = 0; i < XGW; ++i) {
    base += i < wv ? ws[i] : 0u;
    tot += ws[i];
  }
  __syncthreads();
  return base + x - c;
}
// Producer side (thread 0 of block bid of nblocks): the block's count, its group's sum when it arrives last.
__device__ __forceinline__ void xg_publish(const XgCounts& c, int bid, int nblocks, uint32_t cnt) {
  c.bc[bid] = cnt;
  const int g = bid >> 6;
  const unsigned long long old = atomicAdd(&c.acc[g], (1ull << 40) | (unsigned long long)cnt);
  if ((int)(old >> 40) == min(64, nblocks - 64 * g) - 1) {
    c.gs[g] = (uint32_t)(old & ((1ull << 40) - 1ull)) + cnt;
    __hip_atomic_store(&c.acc[g], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// Consumer side (block-cooperative): the counts of blocks [0, bid) of a finished producer launch.
__device__ __forceinline__ uint32_t xg_prefix(const XgCounts& c, int bid) {
  const int g = bid >> 6, t = threadIdx.x;
  uint32_t x = 0;
  for (int j = t; j < g; j += XGT) x += c.gs[j];
  if (t < bid - 64 * g) x += c.bc[64 * g + t];
  return xg_block_sum(x);
}
// Consumer side (block-cooperative): the total of a finished producer launch of nblocks blocks.
__device__ __forceinline__ uint32_t xg_total(const XgCounts& c, int nblocks) {
  uint32_t x = 0;
  for (int j = threadIdx.x; j < (nblocks + 63) / 64; j += XGT) x += c.gs[j];
  return xg_block_sum(x);
}
// This thread's bit in a block's XGW bitmap words and the set bits before it in the block.
__device__ __forceinline__ bool xg_block_bit(const uint64_t* w, uint32_t& before) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t mine = 0;
  before = 0;
#pragma unroll
  for (int j = 0; j < XGW; ++j) {
    const uint64_t x = w[j];
    if (j < wv) before += (uint32_t)__builtin_popcountll(x);
    if (j == wv) mine = x;
  }
  before += (uint32_t)__builtin_popcountll(mine & ((1ull << lane) - 1ull));
  return (mine >> lane) & 1ull;
}
// Stores the block's flag ballots (every wave of the block reaches this) and publishes the block's count.
__device__ __forceinline__ void xg_flag_block(const XgFlags& f, int bid, int nblocks, bool flag) {
  const uint64_t m = __ballot(flag);
  if ((threadIdx.x & 63) == 0) f.bits[bid * XGW + (threadIdx.x >> 6)] = m;
  const uint32_t cnt = xg_block_sum((threadIdx.x & 63) == 0 ? (uint32_t)__builtin_popcountll(m) : 0u);
  if (threadIdx.x == 0) xg_publish(f.c, bid, nblocks, cnt);
}

// n of a call (block-cooperative).
__device__ __forceinline__ int64_t xg_n(const XgCall& a) {
  return a.nsrc.gs ? (int64_t)a.nmul * (int64_t)xg_total(a.nsrc, a.nsrc_blocks) : a.n_host;
}
__device__ __forceinline__ u128 xg_inc(const CrRng& s) { return mk128(s.i_hi, s.i_lo); }
// The stream state of slot k through the vector memory path (a VGPR offset keeps the compiler from a scalar load):
// a scalar load of the slot the previous kernels wrote took 3-17 us on MI355X (GP_STAMPS, tools/xstamps.py).
__device__ __forceinline__ uint32_t xg_vload(const uint32_t* p) {  // the same for one word
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)p[z]);
}
__device__ __forceinline__ CrRng xg_state(const CrRng* st, int k) {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  const uint4* p = reinterpret_cast<const uint4*>(st + k) + z;
  const uint4 a = p[0], b = p[1], c = p[2];
  auto u = [](uint32_t v) -> uint32_t { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
  auto u64 = [&](uint32_t lo, uint32_t hi) -> uint64_t { return ((uint64_t)u(hi) << 32) | (uint64_t)u(lo); };
  CrRng r;
  r.s_hi = u64(a.x, a.y);
  r.s_lo = u64(a.z, a.w);
  r.i_hi = u64(b.x, b.y);
  r.i_lo = u64(b.z, b.w);
  r.has_u32 = u(c.x);
  r.uinteger = u(c.y);
  r.err = u(c.z);
  r.pad = u(c.w);
  return r;
}

// positions a normal call of n draws may need (words per normal: 1.012 on average; capped by the buffers)
__device__ __forceinline__ int xg_norm_need(const XgCall& a, int64_t n) {
  return (int)min((int64_t)a.P, n + n / 16 + 4096);
}
// words a choice call of n draws may need (two candidates per word; Lemire rejections ~n / 2^32)
__device__ __forceinline__ int xg_cho_need(const XgCall& a, int64_t n) {
  return (int)min((int64_t)a.P, n / 2 + n / 1024 + 256);
}
__device__ __forceinline__ void xg_put_state(CrRng* st, int wr, const CrRng& old, u128 s, uint32_t has, uint32_t u) {
  CrRng n = old;
  n.s_hi = hi64(s);
  n.s_lo = lo64(s);
  n.has_u32 = has;
  n.uinteger = u;
  st[wr] = n;
}
// The block's base state jump(S, q0) (thread 0, into LDS bb and, when bstate is set, into bstate[bid]).
__device__ __forceinline__ u128 xg_base_state(const XgCall& a, const CrRng& s0, int q0, uint64_t* bstate) {
  __shared__ uint64_t bb[2];
  if (threadIdx.x == 0) {
    const u128 S = mk128(s0.s_hi, s0.s_lo);
    const u128 b = a.bj ? apply_jump(a.bj[blockIdx.x], S) : pcg_jump_ilp(a.jt, S, (uint32_t)q0);
    bb[0] = hi64(b);
    bb[1] = lo64(b);
    if (bstate) {
      bstate[2 * blockIdx.x] = bb[0];
      bstate[2 * blockIdx.x + 1] = bb[1];
    }
  }
  __syncthreads();
  return mk128(bb[0], bb[1]);
}

// One attempt of numpy's ziggurat starting at position q whose LCG state (before its word) is s:
// 1 = a normal v in `used` words, 0 = a rejected wedge (2 words), -1 = longer than XG_SPAN words.
__device__ int xg_attempt(const ZigTabs& t, u128 s, u128 inc, int& used, double& v) {
  uint64_t r = pcg_output(s);
  int pos = 1;
  auto next = [&]() -> uint64_t {
    s = pcg_step(s, inc);
    ++pos;
    return pcg_output(s);
  };
  const int idx = (int)(r & 0xff);
  r >>= 8;
  const uint64_t sign = r & 1u, rabs = (r >> 1) & 0x000fffffffffffffull;
  double x = (double)rabs * t.wi[idx];
  if (sign) x = -x;
  if (rabs < t.ki[idx]) { used = 1; v = x; return 1; }
  if (idx == 0) {
    for (;;) {
      if (pos + 2 > XG_SPAN) { used = pos; return -1; }
      const double xx = -GP_ZIG_INV_R * zlog1p_neg(u53_of(next()));
      const double yy = -zlog1p_neg(u53_of(next()));
      if (yy + yy > xx * xx) {
        used = pos;
        v = ((rabs >> 8) & 1u) ? -(GP_ZIG_R + xx) : GP_ZIG_R + xx;
        return 1;
      }
    }
  }
  used = 2;
  v = x;
  return ((t.fi[idx - 1] - t.fi[idx]) * u53_of(next()) + t.fi[idx] < zexp(-0.5 * x * x)) ? 1 : 0;
}

__device__ __forceinline__ ZigTabs xg_zig() {
  return ZigTabs{d_zig, reinterpret_cast<const double*>(d_zig + 256), reinterpret_cast<const double*>(d_zig + 512)};
}

// A block's view of positions [q0 - XG_LOOK, q0 + XGT) (the halo: the slow attempts that can reach into the
// block): slow bits, spans, flags (bit 0 on-chain, bit 1 accepted) in LDS. Index i = position - (q0 - XG_LOOK).
template <int NP>  // a view of NP block positions and the XG_LOOK halo before them
struct XgViewT {
  static constexpr int H = XG_LOOK + NP;
  uint64_t bits[H / 64];
  uint16_t span[H];
  uint8_t flag[H];
};
using XgView = XgViewT<XGT>;
constexpr int XGH = XgView::H;
template <class V>
__device__ __forceinline__ bool xv_slow(const V& v, int i) { return (v.bits[i >> 6] >> (i & 63)) & 1ull; }
// The slow positions of view indices [lo, hi) (hi - lo <= 128) as up to three bit words from (lo & ~63).
template <class V>
__device__ __forceinline__ void xv_window(const V& v, int lo, int hi, uint64_t (&m)[3], int& base) {
  base = lo & ~63;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int b0 = base + 64 * k;
    uint64_t w = (b0 < hi && b0 < V::H) ? v.bits[b0 >> 6] : 0ull;
    if (b0 < lo) w &= ~0ull << (lo - b0);
    if (b0 + 64 > hi) w &= (hi - b0) <= 0 ? 0ull : ((hi - b0) >= 64 ? ~0ull : ((1ull << (hi - b0)) - 1ull));
    m[k] = w;
  }
}
// Whether the slow attempt at view index i is on the chain: back to its cluster's start, then forward. -1: the
// cluster may reach before the view (never when the view starts before position 0), for xg_on_chain_abs.
template <class V>
__device__ __forceinline__ int xv_on_chain(const V& v, int i, bool at0) {
  int c = i;
  for (int hop = 0; hop < V::H; ++hop) {
    if (c - XG_SPAN < 0 && !at0) return -1;
    uint64_t m[3];
    int base;
    xv_window(v, max(0, c - XG_SPAN), c, m, base);
    int best = -1;
#pragma unroll
    for (int k = 0; k < 3 && best < 0; ++k) {
      uint64_t w = m[k];
      while (w) {
        const int p = base + 64 * k + __builtin_ctzll(w);
        w &= w - 1;
        if (p + (int)v.span[p] > c) { best = p; break; }
      }
    }
    if (best < 0) break;
    c = best;
  }
  int cur = c;
  for (int p0 = c; p0 <= i; p0 += 128) {
    uint64_t m[3];
    int base;
    xv_window(v, p0, min(i + 1, p0 + 128), m, base);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      uint64_t w = m[k];
      while (w) {
        const int p = base + 64 * k + __builtin_ctzll(w);
        w &= w - 1;
        if (p == i) return p >= cur ? 1 : 0;
        if (p >= cur) cur = p + (int)v.span[p];
      }
    }
  }
  return 1;  // not reached: i is slow
}
// The same walk in stream positions for a cluster that reaches before the block's view (a chain of overlapping
// slow attempts longer than the halo's spare XG_LOOK - XG_SPAN words: rare): positions outside the view are
// evaluated on the spot (their own jump), inside it read from the view.
template <class V>
__device__ __noinline__ int xg_on_chain_abs(const XgCall& a, const V& v, int q0, const CrRng& s0, int qi) {
  const ZigTabs zt = xg_zig();
  const u128 S = mk128(s0.s_hi, s0.s_lo), inc = xg_inc(s0);
  auto slow_at = [&](int p, int& span) -> bool {
    const int i = p - (q0 - XG_LOOK);
    if (i >= 0 && i < V::H) {
      if (!xv_slow(v, i)) return false;
      span = v.span[i];
      return true;
    }
    const u128 X = pcg_jump_ilp(a.jt, S, (uint32_t)p + 1u);
    double z;
    if (zig_fast(zt, pcg_output(X), z)) return false;
    double vv;
    if (xg_attempt(zt, X, inc, span, vv) < 0) atomicOr(a.err, GP_DERR_STREAM);
    return true;
  };
  int c = qi;
  for (;;) {
    int best = -1;
    for (int p = max(0, c - XG_SPAN); p < c && best < 0; ++p) {
      int sp = 1;
      if (slow_at(p, sp) && p + sp > c) best = p;
    }
    if (best < 0) break;
    c = best;
  }
  int cur = c;
  for (int p = c; p < qi; ++p) {
    int sp = 1;
    if (p >= cur && slow_at(p, sp)) cur = p + sp;
  }
  return qi >= cur ? 1 : 0;
}

// N1: words of the block's positions and of its halo, their slow bits and the slow attempts (span, acceptance,
// value), every slow position's place on the chain (for the halo's last XG_LOOK - XG_SPAN positions too), then
// which of the block's positions produce a normal: a slow one when on-chain and accepted, a fast one unless an
// on-chain slow attempt in the XG_SPAN positions before it spans it. Writes the slow and produced bitmaps, span /
// value of the block's slow positions, the block's base state and its count.
__global__ __launch_bounds__(XGT) void xg_norm_classify(XgCall a) {
  const int64_t n = xg_n(a);
  const int need = xg_norm_need(a, n);
  const int q0 = blockIdx.x * XGT;
  if (n == 0 || q0 >= need) return;
  __shared__ XgView v;
  __shared__ uint64_t hb[2];
  const CrRng s0 = xg_state(a.st, a.rd);
  const int t = threadIdx.x, lane = t & 63;
  if (t == 64) {  // the halo's base state (wave 1) beside the block's (thread 0, in xg_base_state)
    const u128 S = mk128(s0.s_hi, s0.s_lo);
    const u128 h = q0 < XG_LOOK ? (u128)0
                   : a.hj  ? apply_jump(a.hj[blockIdx.x], S)
                           : pcg_jump_ilp(a.jt, S, (uint32_t)(q0 - XG_LOOK));
    hb[0] = hi64(h);
    hb[1] = lo64(h);
  }
  const u128 sb = xg_base_state(a, s0, q0, a.bstate);
  const ZigTabs zt = xg_zig();
  const u128 inc = xg_inc(s0);
  // own position (view index XG_LOOK + t) and, for t < XG_LOOK, the halo position (view index t)
  double val = 0.0;
#pragma unroll
  for (int part = 0; part < 2; ++part) {
    if (part == 1 && t >= XG_LOOK) break;  // wave-uniform (XG_LOOK = one wave)
    const int i = part == 0 ? XG_LOOK + t : t;
    const int q = q0 - XG_LOOK + i;
    const bool live = q >= 0 && q < need;
    const u128 X = apply_jump(a.wj[t + 1], part == 0 ? sb : mk128(hb[0], hb[1]));
    double z;
    const bool slow = live && !zig_fast(zt, pcg_output(X), z);
    const uint64_t m = __ballot(slow);
    if (lane == 0) v.bits[i >> 6] = m;
    if (slow) {
      int u = 1;
      double vv = 0.0;
      const int r = xg_attempt(zt, X, inc, u, vv);
      if (r < 0) atomicOr(a.err, GP_DERR_STREAM);
      v.span[i] = (uint16_t)u;
      v.flag[i] = (uint8_t)(r > 0 ? 2u : 0u);
      if (part == 0) val = vv;
    }
  }
  __syncthreads();
  // on-chain bits of the slow positions at view indices [XG_SPAN, XGH): own (t) and the halo's tail (t < 32)
  const int i = XG_LOOK + t, q = q0 + t;
  const bool slow = xv_slow(v, i);
  int on = 0;
  if (slow && (on = xv_on_chain(v, i, q0 == 0)) < 0) on = xg_on_chain_abs(a, v, q0, s0, q);
  const int ih = XG_SPAN + t;
  int onh = 0;
  const bool slowh = t < XG_LOOK - XG_SPAN && xv_slow(v, ih);
  if (slowh && (onh = xv_on_chain(v, ih, q0 == 0)) < 0) onh = xg_on_chain_abs(a, v, q0, s0, q0 - XG_LOOK + ih);
  __syncthreads();  // every walk has read the view's spans; now the flags get their on-chain bit
  if (slow && on) v.flag[i] |= 1u;
  if (slowh && onh) v.flag[ih] |= 1u;
  __syncthreads();
  bool prod;
  if (q >= need) {
    prod = false;
  } else if (slow) {
    prod = (v.flag[i] & 3u) == 3u;
    a.span[q] = v.span[i];
    a.val[q] = val;
  } else {
    prod = true;
    uint64_t m[3];
    int base;
    xv_window(v, i - XG_SPAN, i, m, base);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      uint64_t w = m[k];
      while (w) {
        const int p = base + 64 * k + __builtin_ctzll(w);
        w &= w - 1;
        if ((v.flag[p] & 1u) && p + (int)v.span[p] > i) prod = false;
      }
    }
  }
  const uint64_t pm = __ballot(prod);
  if (lane == 0) {
    a.bits[q >> 6] = v.bits[i >> 6];
    a.pbits[q >> 6] = pm;
  }
  const uint32_t cnt = xg_block_sum(lane == 0 ? (uint32_t)__builtin_popcountll(pm) : 0u);
  if (t == 0) xg_publish(a.pc, blockIdx.x, (need + XGT - 1) / XGT, cnt);
}


// The fused normal call (round 4): N1's classification, then the block's count published with this launch's tag,
// the counts of the blocks before it waited for (64-block group sums from each group's last arriver + the earlier
// blocks of its own group: at most 256 + 63 polls, all of lower-index blocks, which the in-order dispatch has
// started), and N2's indexing and writes from the values still in registers. One launch and no position buffers
// per normal call instead of two launches. A wait that does not end is flagged (GP_DERR_TIMEOUT) and reads 0.
__device__ __forceinline__ uint32_t xg_tpoll(const unsigned long long* p, uint32_t tag, uint32_t* err) {
  for (uint32_t spins = 0;; ++spins) {
    const unsigned long long v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(v >> 32) == tag) return (uint32_t)v;
    if (spins > (1u << 24)) {
      atomicOr(err, GP_DERR_TIMEOUT);
      return 0u;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
// Up to XG_FLAT_MAX blocks a block's prefix sums the tagged block counts themselves (<= XG_FLAT_MAX / XGT loads
// per thread, issued together): the publish is one store, with no returning atomic and no group-sum hop.
#ifndef XG_FLAT_MAX
#define XG_FLAT_MAX 4096
#endif
__device__ __forceinline__ void xg_tpublish(const XgCall& a, int bid, int nblocks, uint32_t cnt) {
  __hip_atomic_store(&a.tbc[bid], ((unsigned long long)a.tag << 32) | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (nblocks <= XG_FLAT_MAX) return;
  const int g = bid >> 6;
  const unsigned long long old = atomicAdd(&a.tacc[g], (1ull << 40) | (unsigned long long)cnt);
  if ((int)(old >> 40) == min(64, nblocks - 64 * g) - 1) {
    const uint32_t gsum = (uint32_t)(old & ((1ull << 40) - 1ull)) + cnt;
    __hip_atomic_store(&a.tacc[g], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.tgs[g], ((unsigned long long)a.tag << 32) | gsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ uint32_t xg_tprefix(const XgCall& a, int bid, int nblocks) {
  const int g = bid >> 6, t = threadIdx.x;
  uint32_t x = 0;
  if (nblocks <= XG_FLAT_MAX) {
    for (int c = 0; c * XGT < bid; c += 4) {  // block-uniform
      unsigned long long v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = t + (c + i) * XGT;
        v[i] = j < bid ? __hip_atomic_load(&a.tbc[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = t + (c + i) * XGT;
        if (j < bid) x += (uint32_t)(v[i] >> 32) == a.tag ? (uint32_t)v[i] : xg_tpoll(&a.tbc[j], a.tag, a.err);
      }
    }
    return xg_block_sum(x);
  }
  for (int j = t; j < g; j += XGT) x += xg_tpoll(&a.tgs[j], a.tag, a.err);
  if (t < bid - 64 * g) x += xg_tpoll(&a.tbc[64 * g + t], a.tag, a.err);
  return xg_block_sum(x);
}

// The fused call's blocks cover XG_PPT positions per thread (XGN per block): the per-block fixed latency (entry
// loads, base states, the publish and the prefix wait, ~20 us) is paid once per XGN positions. At 2^21 envs a call
// of ~4.7M positions was ~21,800 blocks of 256 whose lifetimes, ~4.5 resident per CU, serialised into ~470 us.
// (XG_PPT = 1 below XG_PPT_MIN_BLOCKS blocks of XGT positions: small calls keep their parallelism.)
constexpr int XG_PPT_MIN_BLOCKS = 1024;
// The env kernels (xg_dry, xg_step) likewise take 4 env blocks per workgroup above this many env blocks.
constexpr int XG_SPB_MIN_BLOCKS = 1024;

template <int XG_PPT>
__global__ __launch_bounds__(XGT) void xg_norm_fused(XgCall a) {
  constexpr int XGN = XGT * XG_PPT;
  const int xty = a.nsrc.gs ? 2 : 0;
  XSTAMP(xty, 0);
  const PcgJump myj = a.wj[threadIdx.x + 1];  // (independent of everything: issued first)
  const CrRng s0 = xg_state(a.st, a.rd);  // (issued before n's loads and barrier)
  const int64_t want = a.xinfo ? (int64_t)xg_vload(a.xinfo + 1) : 0;
  const int64_t n = xg_n(a);
  XSTAMP(xty, 1);
  const int bid = blockIdx.x, q0 = bid * XGN;
  // the extension's normals past n (the next call's, xg_wall_one)
  const int64_t X = a.xinfo ? min((int64_t)a.xmax, want + want / 4 + 1024) : 0;
  const int need = min(xg_norm_need(a, n + X), (int)(gridDim.x * XGN));  // (the launch may cap the extension)
  if (n == 0) {  // nothing drawn: the state carries over
    if (bid == 0 && threadIdx.x == 0) a.st[a.wr] = s0;
    return;
  }
  if (q0 >= need) return;
  using View = XgViewT<XGN>;
  __shared__ View v;
  __shared__ uint64_t hb[2];
  __shared__ uint64_t bb[XG_PPT][2];
  __shared__ uint64_t pmw[XGN / 64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  {
    const u128 S = mk128(s0.s_hi, s0.s_lo);
    if (t == 64) {  // the halo's base state (wave 1) beside the sub-blocks' (threads 0 .. XG_PPT - 1)
      const u128 h = q0 < XG_LOOK ? (u128)0
                     : a.hj  ? apply_jump(a.hj[bid * XG_PPT], S)
                             : pcg_jump_ilp(a.jt, S, (uint32_t)(q0 - XG_LOOK));
      hb[0] = hi64(h);
      hb[1] = lo64(h);
    }
    if (t < XG_PPT) {  // sub-block m = t: positions q0 + XGT m .. (bj[k] = k XGT steps)
      const u128 b = a.bj ? apply_jump(a.bj[bid * XG_PPT + t], S) : pcg_jump_ilp(a.jt, S, (uint32_t)(q0 + XGT * t));
      bb[t][0] = hi64(b);
      bb[t][1] = lo64(b);
    }
  }
  __syncthreads();
  XSTAMP(xty, 2);
  const ZigTabs zt = xg_zig();
  const u128 inc = xg_inc(s0);
  double val[XG_PPT], zf[XG_PPT];
  int span[XG_PPT];
  // own positions: view index XG_LOOK + XGT m + t; then (t < XG_LOOK) the halo's, view index t
#pragma unroll
  for (int part = 0; part <= XG_PPT; ++part) {
    if (part == XG_PPT && t >= XG_LOOK) break;  // wave-uniform (XG_LOOK = one wave)
    const bool halo = part == XG_PPT;
    const int i = halo ? t : XG_LOOK + XGT * part + t;
    const int q = q0 - XG_LOOK + i;
    const bool live = q >= 0 && q < need;
    const u128 Xs = apply_jump(myj, halo ? mk128(hb[0], hb[1]) : mk128(bb[part][0], bb[part][1]));
    double z;
    const bool slow = live && !zig_fast(zt, pcg_output(Xs), z);
    if (!halo) {
      zf[part] = z;
      val[part] = 0.0;
      span[part] = 1;
    }
    const uint64_t m = __ballot(slow);
    if (lane == 0) v.bits[i >> 6] = m;
    if (slow) {
      int u = 1;
      double vv = 0.0;
      const int r = xg_attempt(zt, Xs, inc, u, vv);
      if (r < 0) atomicOr(a.err, GP_DERR_STREAM);
      v.span[i] = (uint16_t)u;
      v.flag[i] = (uint8_t)(r > 0 ? 2u : 0u);
      if (!halo) {
        val[part] = vv;
        span[part] = u;
      }
    }
  }
  __syncthreads();
  XSTAMP(xty, 3);
  bool slow[XG_PPT];
  int on[XG_PPT];
#pragma unroll
  for (int m = 0; m < XG_PPT; ++m) {
    const int i = XG_LOOK + XGT * m + t;
    slow[m] = xv_slow(v, i);
    on[m] = 0;
    if (slow[m] && (on[m] = xv_on_chain(v, i, q0 == 0)) < 0) on[m] = xg_on_chain_abs(a, v, q0, s0, q0 + XGT * m + t);
  }
  const int ih = XG_SPAN + t;
  int onh = 0;
  const bool slowh = t < XG_LOOK - XG_SPAN && xv_slow(v, ih);
  if (slowh && (onh = xv_on_chain(v, ih, q0 == 0)) < 0) onh = xg_on_chain_abs(a, v, q0, s0, q0 - XG_LOOK + ih);
  __syncthreads();
#pragma unroll
  for (int m = 0; m < XG_PPT; ++m)
    if (slow[m] && on[m]) v.flag[XG_LOOK + XGT * m + t] |= 1u;
  if (slowh && onh) v.flag[ih] |= 1u;
  __syncthreads();
  XSTAMP(xty, 4);
  bool prod[XG_PPT];
  uint32_t mycnt = 0;
#pragma unroll
  for (int m = 0; m < XG_PPT; ++m) {
    const int i = XG_LOOK + XGT * m + t, q = q0 + XGT * m + t;
    if (q >= need) {
      prod[m] = false;
    } else if (slow[m]) {
      prod[m] = (v.flag[i] & 3u) == 3u;
    } else {
      prod[m] = true;
      uint64_t mw[3];
      int base;
      xv_window(v, i - XG_SPAN, i, mw, base);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        uint64_t w = mw[k];
        while (w) {
          const int p = base + 64 * k + __builtin_ctzll(w);
          w &= w - 1;
          if ((v.flag[p] & 1u) && p + (int)v.span[p] > i) prod[m] = false;
        }
      }
    }
    const uint64_t pm = __ballot(prod[m]);
    if (lane == 0) pmw[(XGT / 64) * m + wv] = pm;
    mycnt += lane == 0 ? (uint32_t)__builtin_popcountll(pm) : 0u;
  }
  const uint32_t cnt = xg_block_sum(mycnt);  // (syncs pmw too)
  const int nb = (need + XGN - 1) / XGN;
  if (t == 0) xg_tpublish(a, bid, nb, cnt);
  XSTAMP(xty, 5);
  const int64_t pre = xg_tprefix(a, bid, nb);
  XSTAMP(xty, 6);
  if (bid == nb - 1 && t == 0) {
    if (pre + cnt < n) atomicOr(a.err, GP_DERR_STREAM);
    if (X > 0) a.xinfo[0] = (uint32_t)min(X, max((int64_t)0, pre + (int64_t)cnt - n));
  }
  if (pre >= n + X) return;
  uint32_t before = 0;  // produced positions of the block's earlier bitmap words
#pragma unroll
  for (int m = 0; m < XG_PPT; ++m) {
    const int wi = (XGT / 64) * m + wv;  // this position's bitmap word
    const uint64_t pm = pmw[wi];
    uint32_t b = before + __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
    for (int j = 0; j < wi; ++j) b += j >= (XGT / 64) * m ? (uint32_t)__builtin_popcountll(pmw[j]) : 0u;
    if (prod[m]) {
      const int q = q0 + XGT * m + t;
      const int64_t r = pre + b;
      if (r >= n) {
        if (r < n + X) {  // the extension: the next call's normals, at its scale, with their end positions
          a.xdst[r - n] = 0.0 + a.xscale * (slow[m] ? val[m] : zf[m]);
          a.xend[r - n] = (uint32_t)q + (slow[m] ? (uint32_t)span[m] : 1u);
        }
      } else {
        a.dst[r] = 0.0 + a.scale * (slow[m] ? val[m] : zf[m]);  // numpy: loc + scale * standard_normal
        if (r == n - 1) {
          const uint32_t endpos = (uint32_t)q + (slow[m] ? (uint32_t)span[m] : 1u);
          xg_put_state(a.st, a.wr, s0, pcg_jump_ilp(a.jt, mk128(s0.s_hi, s0.s_lo), endpos), s0.has_u32, s0.uinteger);
        }
      }
    }
    // the words of sub-block m, all waves: the next sub-block's positions come after them
#pragma unroll
    for (int j = 0; j < XGT / 64; ++j) before += (uint32_t)__builtin_popcountll(pmw[(XGT / 64) * m + j]);
  }
  XSTAMP(xty, 7);
}

// The wall-noise call after an extended action-noise call, in one workgroup (crooms.py:321-325: normal(0.5,
// (n_oob, 2)), n = 2 * the dry step's wall hits). When the extension made them (n <= xinfo[0]) only the stream
// state moves, to the end of the extension's n-th normal; otherwise (the first step, or a jump in the wall-hit
// count past the extension's 5/4 margin) the call is drawn here from the action-noise call's end, one 1024-word
// window per round (x_normals). One small launch per step instead of a grid-wide normal call.
__global__ __launch_bounds__(XT) void xg_wall_one(XgCall a, CrExact x) {
  __shared__ XShared sh;
  __shared__ uint32_t red[XT / 64];
  const int t = threadIdx.x;
  XSTAMP(2, 0);
  const CrRng s0 = xg_state(a.st, a.rd);  // the action-noise call's end
  const uint32_t made = xg_vload(a.xinfo);  // the extension's normals
  uint32_t c = 0;
  for (int j = t; j < (a.nsrc_blocks + 63) / 64; j += XT) c += a.nsrc.gs[j];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
  if ((t & 63) == 0) red[t >> 6] = c;
  __syncthreads();
  uint32_t tot = 0;
#pragma unroll
  for (int i = 0; i < XT / 64; ++i) tot += red[i];
  const int64_t n = (int64_t)a.nmul * tot;
  XSTAMP(2, 1);
  if (t == 0) a.xinfo[1] = (uint32_t)n;
  if (n == 0) {
    if (t == 0) a.st[a.wr] = s0;
    return;
  }
  if (n <= (int64_t)made) {
    if (t == 0) {
      const CrRng sa = xg_state(a.st, a.wr);  // the action-noise call's start (the slot this call writes)
      xg_put_state(a.st, a.wr, sa, pcg_jump_ilp(a.jt, mk128(sa.s_hi, sa.s_lo), xg_vload(a.xend + (n - 1))),
                   sa.has_u32, sa.uinteger);
    }
    XSTAMP(2, 7);
    return;
  }
  const PcgJump myj = a.wj[t + 1];
  for (int i = t; i < 768; i += XT) sh.zt[i] = d_zig[i];
  if (t == 0) {
    sh.st_hi = s0.s_hi;
    sh.st_lo = s0.s_lo;
    sh.has_u32 = s0.has_u32;
    sh.uinteger = s0.uinteger;
    sh.err = 0;
  }
  __syncthreads();
  x_normals(sh, x, myj, n, a.scale, a.dst);
  __syncthreads();
  if (t == 0) {
    if (sh.err) atomicOr(a.err, GP_DERR_STREAM);
    CrRng o = s0;
    o.s_hi = sh.st_hi;
    o.s_lo = sh.st_lo;
    a.st[a.wr] = o;
  }
  XSTAMP(2, 6);
}

// N2: every produced normal's index r (prefix of the block counts + its rank in the block) -> dst[r]; the n-th
// one ends the call. No block waits on another.
__global__ __launch_bounds__(XGT) void xg_norm_write(XgCall a) {
  const int64_t n = xg_n(a);
  const int need = xg_norm_need(a, n);
  const int bid = blockIdx.x, q0 = bid * XGT;
  const CrRng s0 = xg_state(a.st, a.rd);
  if (n == 0) {  // nothing drawn: the state carries over
    if (bid == 0 && threadIdx.x == 0) a.st[a.wr] = s0;
    return;
  }
  if (q0 >= need) return;
  const int64_t pre = xg_prefix(a.pc, bid);
  const int nb = (need + XGT - 1) / XGT;
  if (bid == nb - 1 && threadIdx.x == 0 && pre + a.pc.bc[bid] < n) atomicOr(a.err, GP_DERR_STREAM);
  if (pre >= n) return;  // block-uniform
  uint32_t before;
  const bool prod = xg_block_bit(a.pbits + (size_t)bid * XGW, before);
  const int64_t r = pre + before;
  if (!prod || r >= n) return;
  const int q = q0 + threadIdx.x;
  const bool fq = !((a.bits[q >> 6] >> (threadIdx.x & 63)) & 1ull);
  double val;
  if (fq) {
    const u128 sb = mk128(a.bstate[2 * bid], a.bstate[2 * bid + 1]);
    zig_fast(xg_zig(), pcg_output(apply_jump(a.wj[threadIdx.x + 1], sb)), val);
  } else {
    val = a.val[q];
  }
  a.dst[r] = 0.0 + a.scale * val;  // numpy: loc + scale * standard_normal
  if (r == n - 1) {
    const uint32_t endpos = (uint32_t)q + (fq ? 1u : (uint32_t)a.span[q]);
    xg_put_state(a.st, a.wr, s0, pcg_jump_ilp(a.jt, mk128(s0.s_hi, s0.s_lo), endpos), s0.has_u32, s0.uinteger);
  }
}

// choice(n), per word q: the Lemire acceptances of (lo, hi) (+ the buffered half at q = 0) as 3 flag bits.
__device__ __forceinline__ uint32_t xg_cho_flags(const XgCall& a, const CrRng& s0, int q, int need, uint64_t w) {
  uint32_t f = 0;
  if (q < need) {
    if (q == 0 && s0.has_u32 && !lemire_rejected(s0.uinteger, a.nv, a.lthr)) f |= 1u;
    if (!lemire_rejected((uint32_t)w, a.nv, a.lthr)) f |= 2u;
    if (!lemire_rejected((uint32_t)(w >> 32), a.nv, a.lthr)) f |= 4u;
  }
  return f;
}
// C1: per block, the drawn candidates (and the block's base state).
__global__ __launch_bounds__(XGT) void xg_cho_count(XgCall a) {
  const int64_t n = xg_n(a);
  const int need = xg_cho_need(a, n);
  const int q0 = blockIdx.x * XGT;
  if (n == 0 || q0 >= need) return;
  const CrRng s0 = xg_state(a.st, a.rd);
  const u128 sb = xg_base_state(a, s0, q0, a.bstate);
  const uint64_t w = pcg_output(apply_jump(a.wj[threadIdx.x + 1], sb));
  const uint32_t cnt = xg_block_sum((uint32_t)__builtin_popcount(xg_cho_flags(a, s0, q0 + threadIdx.x, need, w)));
  if (threadIdx.x == 0) xg_publish(a.pc, blockIdx.x, (need + XGT - 1) / XGT, cnt);
}
// The fused choice call (round 4): C1's count, published with this launch's tag, the prefix over the earlier blocks
// waited for in-launch (xg_tprefix), then C2's writes: one launch per choice call instead of two.
__global__ __launch_bounds__(XGT) void xg_cho_fused(XgCall a) {
  XSTAMP(4, 0);
#ifdef GP_STAMPS
  {
    const int rd_ = a.rd;
    asm volatile("" ::"s"(rd_));
    XSTAMP(4, 4);
  }
#endif
  const CrRng s0 = xg_state(a.st, a.rd);  // (issued before n's loads and barrier)
#ifdef GP_STAMPS
  asm volatile("" ::"s"(s0.s_lo));
  XSTAMP(4, 3);
#endif
  const int64_t n = xg_n(a);
  XSTAMP(4, 1);
  const int need = xg_cho_need(a, n);
  const int bid = blockIdx.x, q0 = bid * XGT;
  if (n == 0) {
    if (bid == 0 && threadIdx.x == 0) a.st[a.wr] = s0;
    return;
  }
  if (q0 >= need) return;
  const int q = q0 + threadIdx.x;
  const u128 sb = xg_base_state(a, s0, q0, nullptr);
  XSTAMP(4, 2);
  const uint64_t w = pcg_output(apply_jump(a.wj[threadIdx.x + 1], sb));
  const uint32_t f = xg_cho_flags(a, s0, q, need, w);
  uint32_t tot;
  const uint32_t off = xg_block_scan((uint32_t)__builtin_popcount(f), tot);
  const int nb = (need + XGT - 1) / XGT;
  if (threadIdx.x == 0) xg_tpublish(a, bid, nb, tot);
  XSTAMP(4, 5);
  const int64_t pre = xg_tprefix(a, bid, nb);
  XSTAMP(4, 6);
  if (bid == nb - 1 && threadIdx.x == 0 && pre + tot < n) atomicOr(a.err, GP_DERR_STREAM);
  if (pre >= n) return;
  int64_t r = pre + off;
  // candidates in stream order: buffered half (code 0), lo of word q (2q + 1), hi (2q + 2)
  const uint32_t cand[3] = {s0.uinteger, (uint32_t)w, (uint32_t)(w >> 32)};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if (!((f >> c) & 1u)) continue;
    if (r < n) a.idst[r] = (int32_t)lemire_value(cand[c], a.nv);
    if (r == n - 1) {
      const uint32_t e = c == 0 ? 0u : 2u * (uint32_t)q + (uint32_t)c;  // the last candidate consumed
      const uint32_t words = (e + 1u) / 2u;
      // numpy's next_uint32 buffers the high half of every word it draws and keeps it after handing it out
      xg_put_state(a.st, a.wr, s0, pcg_jump_ilp(a.jt, mk128(s0.s_hi, s0.s_lo), words), (e & 1u),
                   e ? (uint32_t)(w >> 32) : s0.uinteger);
    }
    ++r;
  }
  XSTAMP(4, 7);
}
// C2: the draws to idst[r]; the n-th one fixes the next state, has_uint32 and uinteger.
__global__ __launch_bounds__(XGT) void xg_cho_write(XgCall a) {
  const int64_t n = xg_n(a);
  const int need = xg_cho_need(a, n);
  const int bid = blockIdx.x, q0 = bid * XGT;
  const CrRng s0 = xg_state(a.st, a.rd);
  if (n == 0) {
    if (bid == 0 && threadIdx.x == 0) a.st[a.wr] = s0;
    return;
  }
  if (q0 >= need) return;
  const int64_t pre = xg_prefix(a.pc, bid);
  const int nb = (need + XGT - 1) / XGT;
  if (bid == nb - 1 && threadIdx.x == 0 && pre + a.pc.bc[bid] < n) atomicOr(a.err, GP_DERR_STREAM);
  if (pre >= n) return;  // block-uniform
  const int q = q0 + threadIdx.x;
  const uint64_t w = pcg_output(apply_jump(a.wj[threadIdx.x + 1], mk128(a.bstate[2 * bid], a.bstate[2 * bid + 1])));
  const uint32_t f = xg_cho_flags(a, s0, q, need, w);
  uint32_t tot;
  int64_t r = pre + xg_block_scan((uint32_t)__builtin_popcount(f), tot);
  // candidates in stream order: buffered half (code 0), lo of word q (2q + 1), hi (2q + 2)
  const uint32_t cand[3] = {s0.uinteger, (uint32_t)w, (uint32_t)(w >> 32)};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if (!((f >> c) & 1u)) continue;
    if (r < n) a.idst[r] = (int32_t)lemire_value(cand[c], a.nv);
    if (r == n - 1) {
      const uint32_t e = c == 0 ? 0u : 2u * (uint32_t)q + (uint32_t)c;  // the last candidate consumed
      const uint32_t words = (e + 1u) / 2u;
      // numpy's next_uint32 buffers the high half of every word it draws and keeps it after handing it out
      xg_put_state(a.st, a.wr, s0, pcg_jump_ilp(a.jt, mk128(s0.s_hi, s0.s_lo), words), (e & 1u),
                   e ? (uint32_t)(w >> 32) : s0.uinteger);
    }
    ++r;
  }
}

// random(n): n uniforms k53 = w >> 11 (numpy next_double), word e for draw e.
__global__ __launch_bounds__(XGT) void xg_uniforms(XgCall a, uint64_t* __restrict__ dst) {
  const int64_t n = a.n_host;
  const int q0 = blockIdx.x * XGT;
  const CrRng s0 = xg_state(a.st, a.rd);
  const u128 S = mk128(s0.s_hi, s0.s_lo);
  if (blockIdx.x == 0 && threadIdx.x == 0) xg_put_state(a.st, a.wr, s0, pcg_jump_ilp(a.jt, S, (uint32_t)n), s0.has_u32,
                                                         s0.uinteger);
  if (q0 >= n) return;
  const u128 sb = xg_base_state(a, s0, q0, nullptr);
  const int q = q0 + threadIdx.x;
  if (q < n) dst[q] = pcg_output(apply_jump(a.wj[threadIdx.x + 1], sb)) >> 11;
}

// Dry step on copies: which envs hit a wall (the wall-noise draw count, crooms.py:321-325) -> fd.
// Round 4: the previous step's resets (fr: its resetting envs, gi / ai their draws, obs_prev its observation row)
// are applied here first, as xg_apply_resets would (one launch per step fewer); fr.bits == nullptr: none pending.
// SPB env blocks (of XGT envs: the unit of the flag bitmaps and counts) per workgroup, in turn: large batches
// pay the per-workgroup latency (table staging, the prefix loads) once per SPB blocks; nsub = env blocks in all.
template <int OK, int SPB>
__global__ __launch_bounds__(XGT) void xg_dry(CrDev p, XgFlags fd, const void* __restrict__ act, size_t off,
                                              XgFlags fr, const int32_t* __restrict__ gi,
                                              const int32_t* __restrict__ ai, void* __restrict__ obs_prev, int nsub) {
  XSTAMP(1, 0);
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int sb0 = blockIdx.x * SPB;
  // the env blocks' reset bitmap words, lane-indexed (vector loads: the previous step's kernel wrote them)
  uint64_t rw[SPB];
  uint64_t anyb = 0;
#pragma unroll
  for (int b = 0; b < SPB; ++b) {
    rw[b] = 0;
    if (fr.bits && lane < XGW && sb0 + b < nsub) rw[b] = fr.bits[(size_t)(sb0 + b) * XGW + lane];
    anyb |= rw[b];
  }
  for (int i = threadIdx.x; i < p.tab_bytes / 16; i += XGT) ((uint4*)lds)[i] = ((const uint4*)p.tabs)[i];
  uint32_t pre = 0;
  const bool any = __syncthreads_or(anyb != 0ull);
  if (any) pre = xg_prefix(fr.c, sb0);  // block-uniform (its block sum syncs the table copy too)
  __syncthreads();
#pragma unroll
  for (int b = 0; b < SPB; ++b) {
    const int bid = sb0 + b;
    if (bid >= nsub) break;  // block-uniform
    uint64_t mine = 0;
    uint32_t before = 0;
#pragma unroll
    for (int j = 0; j < XGW; ++j) {
      const uint64_t x = __shfl(rw[b], j, 64);
      if (j < wv) before += (uint32_t)__builtin_popcountll(x);
      if (j == wv) mine = x;
    }
    before += (uint32_t)__builtin_popcountll(mine & ((1ull << lane) - 1ull));
    const bool rf = (mine >> lane) & 1ull;
    const int env = bid * XGT + threadIdx.x;
    bool f = false;
    if (env < p.B) {
      double a0, a1;
      int ad;
      x_load_action(p, act, off, env, a0, a1, ad);
      double ay, ax, vy, vx;
      uint32_t g;
      if (rf) {  // crooms.py:217-244 with the previous step's draws (as xg_apply_resets)
        const int r = (int)(pre + before);
        Draws d;
        d.k53 = 0;
        d.gi = p.goal_fixed ? 0u : (uint32_t)gi[r];
        d.ai = p.agent_fixed ? 0u : (uint32_t)ai[r];
        g = x_goal(p, env);
        reset_env(p, lds, d, ay, ax, vy, vx, g);
        vy = vx = 0.0;
        p.ay[env] = ay;
        p.ax[env] = ax;
        if (p.use_velocity) { p.vy[env] = 0.0; p.vx[env] = 0.0; }
        if (!p.goal_fixed) p.goal[env] = g;
        write_obs<OK>(p, lds, env, ay, ax, g, obs_prev);
      } else {
        ay = p.ay[env];
        ax = p.ax[env];
        vy = p.use_velocity ? p.vy[env] : 0.0;
        vx = p.use_velocity ? p.vx[env] : 0.0;
        g = x_goal(p, env);
      }
      int32_t el = p.el[env];
      float rs = 0.f;
      uint32_t ep = 0, ln = 0;
      const StepOut o = crooms_env_step<true>(p, lds, env, true, 0, a0, a1, ad, ay, ax, vy, vx, g, el, rs, ep, ln);
      f = o.oob != 0;
    }
    xg_flag_block(fd, bid, nsub, f);
    // the next env block's resets follow this one's (its count, published by the previous step's kernel)
    if (any && b + 1 < SPB && bid + 1 < nsub) pre += fr.c.bc[bid];
  }
  XSTAMP(1, 7);
}

// The step with the wall noise in place (crooms.py:276-298; an env that hits a wall reads pair r of the wall
// noise, r = its rank among fd's envs), resets deferred -> fs. SPB env blocks per workgroup, as xg_dry.
template <int OK, int SPB>
__global__ __launch_bounds__(XGT) void xg_step(CrDev p, XgFlags fd, XgFlags fs, const void* __restrict__ act,
                                               size_t off, void* __restrict__ obs, float* __restrict__ rew,
                                               uint8_t* __restrict__ term, uint8_t* __restrict__ trunc, int nsub) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  XSTAMP(3, 0);
  for (int i = threadIdx.x; i < p.tab_bytes / 16; i += XGT) ((uint4*)lds)[i] = ((const uint4*)p.tabs)[i];
  const int sb0 = blockIdx.x * SPB;
  uint32_t wpre = xg_prefix(fd.c, sb0);  // (its block sum syncs the table copy too)
  XSTAMP(3, 1);
  float rsum = 0.f;
  uint32_t eps = 0, lens = 0, nst = 0;
#pragma unroll
  for (int b = 0; b < SPB; ++b) {
    const int bid = sb0 + b;
    if (bid >= nsub) break;  // block-uniform
    uint32_t wbefore;
    xg_block_bit(fd.bits + (size_t)bid * XGW, wbefore);
    const int env = bid * XGT + threadIdx.x;
    bool f = false;
    if (env < p.B) {
      double a0, a1;
      int ad;
      x_load_action(p, act, off, env, a0, a1, ad);
      double ay = p.ay[env], ax = p.ax[env];
      double vy = p.use_velocity ? p.vy[env] : 0.0, vx = p.use_velocity ? p.vx[env] : 0.0;
      uint32_t g = x_goal(p, env);
      int32_t el = p.el[env];
      const StepOut o = crooms_env_step<true, true>(p, lds, env, true, 0, a0, a1, ad, ay, ax, vy, vx, g, el, rsum,
                                                    eps, lens, (int)(wpre + wbefore));
      nst += 1;
      rew[off + env] = o.rew;
      term[off + env] = o.term;
      trunc[off + env] = o.trunc;
      f = (o.term | o.trunc) != 0;
      if (!f) {
        write_obs<OK>(p, lds, env, ay, ax, g, obs);
        p.ay[env] = ay;
        p.ax[env] = ax;
        if (p.use_velocity) { p.vy[env] = vy; p.vx[env] = vx; }
      }
      p.el[env] = el;
    }
    xg_flag_block(fs, bid, nsub, f);
    if (b + 1 < SPB && bid + 1 < nsub) wpre += fd.c.bc[bid];  // the next env block's wall hits follow this one's
  }
  XSTAMP(3, 2);
  // episode statistics: block reduction, one set of atomics per workgroup
  __shared__ float m_r[XGW];
  __shared__ uint32_t m_e[XGW], m_l[XGW], m_n[XGW];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    rsum += __shfl_xor(rsum, d, 64);
    eps += __shfl_xor(eps, d, 64);
    lens += __shfl_xor(lens, d, 64);
    nst += __shfl_xor(nst, d, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) { m_r[wv] = rsum; m_e[wv] = eps; m_l[wv] = lens; m_n[wv] = nst; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0.f;
    uint32_t ee = 0, l = 0, nn = 0;
    for (int i = 0; i < XGW; ++i) { r += m_r[i]; ee += m_e[i]; l += m_l[i]; nn += m_n[i]; }
    CrSlot& m = p.mslot[blockIdx.x % p.nslot];  // (one slot for every block serialised up to 6 us of atomics)
    atomicAdd(&m.return_sum, (double)r);
    atomicAdd(&m.episodes, (unsigned long long)ee);
    atomicAdd(&m.length_sum, (unsigned long long)l);
    atomicAdd(&m.env_steps, (unsigned long long)nn);
  }
  XSTAMP(3, 7);
}

// The resets (crooms.py:217-244 goal then agent; :251-266 for reset()): fs's envs, the env of rank r taking
// gi[r] / ai[r]; or every env (fs.bits == nullptr: reset(), by env index; elapsed and velocity cleared too).
template <int OK>
__global__ __launch_bounds__(XGT) void xg_apply_resets(CrDev p, XgFlags fs, const int32_t* __restrict__ gi,
                                                       const int32_t* __restrict__ ai, void* __restrict__ obs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  XSTAMP(5, 0);
  const int bid = blockIdx.x, env = bid * XGT + threadIdx.x;
  int r = env;
  bool f = env < p.B;
  if (fs.bits) {
    const uint64_t* w = fs.bits + (size_t)bid * XGW;
    uint64_t any = 0;
#pragma unroll
    for (int j = 0; j < XGW; ++j) any |= w[j];
    if (!any) return;  // block-uniform: nothing resets here
    const uint32_t pre = xg_prefix(fs.c, bid);
    uint32_t before;
    f = xg_block_bit(w, before);
    r = (int)(pre + before);
  }
  for (int i = threadIdx.x; i < p.tab_bytes / 16; i += XGT) ((uint4*)lds)[i] = ((const uint4*)p.tabs)[i];
  __syncthreads();
  XSTAMP(5, 1);
  if (!f) return;
  Draws d;
  d.k53 = 0;
  d.gi = p.goal_fixed ? 0u : (uint32_t)gi[r];
  d.ai = p.agent_fixed ? 0u : (uint32_t)ai[r];
  double ay, ax, vy, vx;
  uint32_t g = x_goal(p, env);
  reset_env(p, lds, d, ay, ax, vy, vx, g);
  p.ay[env] = ay;
  p.ax[env] = ax;
  if (p.use_velocity) { p.vy[env] = 0.0; p.vx[env] = 0.0; }
  if (!p.goal_fixed) p.goal[env] = g;
  if (!fs.bits) p.el[env] = 0;
  write_obs<OK>(p, lds, env, ay, ax, g, obs);
}

__global__ void xg_copy_state(CrRng* st, int from, int to) {
  if (threadIdx.x == 0 && blockIdx.x == 0) st[to] = st[from];
}

// ------------------------------------------------------------------ host backend ----
template <class F>
static int dispatch_obs(int ok, F&& f) {
  switch (ok) {
    case GP_OBS_F32: return f(std::integral_constant<int, GP_OBS_F32>());
    case GP_OBS_HANSEN: return f(std::integral_constant<int, GP_OBS_HANSEN>());
    case GP_OBS_HANSEN_VEC: return f(std::integral_constant<int, GP_OBS_HANSEN_VEC>());
    case GP_OBS_TABLE: return f(std::integral_constant<int, GP_OBS_TABLE>());
    case GP_OBS_WINDOW: return f(std::integral_constant<int, GP_OBS_WINDOW>());
  }
  gp_set_error("crooms: bad obs kind %d", ok);
  return GP_E_INVALID;
}

struct CRoomsBackend : EnvBackend {
  CrDev d{};
  int grid = 1;
  uint64_t philox_step = 0;
  std::vector<int32_t> valid_h;
  DevBuf b_tabs, b_ay, b_ax, b_vy, b_vx, b_goal, b_el, b_slot;
  DevErr derr;
  // exact (numpy-stream) mode
  DevBuf x_rng, x_wj, x_noise, x_wall, x_dense, x_u, x_gi, x_ai, x_rank;
  CrExact xd{};
  int x_alloc();
  int x_upload_rng(const RngHost& r);
  // multi-workgroup exact mode (B > XG_MIN_ENVS): position buffers, block counts, the env phases' flags
  DevBuf xg_jt, xg_bits, xg_pbits, xg_bstate, xg_span, xg_val, xg_cnt, xg_ebits;
  DevBuf xg_tbc, xg_tgs, xg_tacc;  // the fused normal call's tagged counts (tacc zero between launches)
  uint32_t xg_tag = 0;
  // Round 6: xg_rollout's K-step launch sequence (5-6 dependent launches per step, all sized on the host from B and
  // K alone) captured once and replayed as a hipGraph: a dependent launch costs ~1 us less replayed than launched
  // (tools/mb_graph.hip, profiles/r06_mb_graph.txt). A captured fused call's tag is fixed (bit 31 set; eager tags
  // stay below it), and the graph ends by clearing the tagged slots, so no replay finds one of its tags already
  // published. One graph is kept, keyed by K, the caller's buffers and the geometry knobs; by default it is
  // captured on the second identical call (a one-off call stays eager), up to XG_GRAPH_MAX_ENVS envs: replayed vs
  // launched, µs/step (profiles/r06_crooms_numpy_graph_ab.txt) 32.0 vs 36.5 at 4,096 envs, 49.7 vs 50.0 at 65,536,
  // but 76.6 vs 74.2 at 2^18 (not explained) and 290-292 vs 289-303 at 2^21: eager launches above 65,536 envs.
  static constexpr int64_t XG_GRAPH_MAX_ENVS = 65536;
  struct XgGraphKey {
    int K = -1;
    const void *act = nullptr, *obs = nullptr, *rew = nullptr, *term = nullptr, *trunc = nullptr;
    int spb = 0, ppt = 0;
    bool operator==(const XgGraphKey& o) const {
      return K == o.K && act == o.act && obs == o.obs && rew == o.rew && term == o.term && trunc == o.trunc &&
             spb == o.spb && ppt == o.ppt;
    }
  };
  int xg_graph_mode = -1;  // gp_debug_set("xg_graph") at create: -1 from the 2nd identical call, 0 never, 1 always
  bool xg_graph_broken = false;  // a capture failed: eager launches from then on
  XgGraphKey xg_gkey, xg_glast;  // the graph's key; the last eager call's
  hipGraph_t xg_graph = nullptr;
  hipGraphExec_t xg_gexec = nullptr;
  hipStream_t xg_cap = nullptr;  // the capture stream (the caller's may be the null stream, which cannot capture)
  bool xg_capturing = false;
  uint32_t xg_gtag = 0;
  uint32_t xg_next_tag() {
    if (xg_capturing) return 0x80000000u | ++xg_gtag;
    if (++xg_tag >= 0x80000000u) xg_tag = 1;  // (a wrapped tag could only meet slots 2^31 launches old)
    return xg_tag;
  }
  void xg_graph_drop() {
    if (xg_gexec) (void)hipGraphExecDestroy(xg_gexec);
    if (xg_graph) (void)hipGraphDestroy(xg_graph);
    xg_gexec = nullptr;
    xg_graph = nullptr;
    xg_gkey = XgGraphKey{};
  }
  ~CRoomsBackend() override {
    xg_graph_drop();
    if (xg_cap) (void)hipStreamDestroy(xg_cap);
  }
  int xg_graph_capture(const XgGraphKey& key, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc);
#ifdef GP_STAMPS
  DevBuf xg_dbg;  // [6 kinds][1024 blocks][8] stamps (tools/xstamps.py)
  int debug_stamps(unsigned long long* out, int cap) override {
    GP_HIP_CHECK(hipDeviceSynchronize());
    if (!xg_dbg.p) return 0;
    const int n = std::min(cap, 6 * 1024 * 8);
    GP_HIP_CHECK(hipMemcpy(out, xg_dbg.p, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost));
    return n;
  }
#endif
  int xg_P = 0;                  // positions of a draw call (>= what normal(2B) needs)
  int xg_nbe = 0;                // env blocks
  int xg_slot = 0;               // the stream-state slot holding the current state (0 between API calls)
  int xg_min = XG_MIN_ENVS;       // at or below: the one-workgroup kernel (gp_debug_set xg_min_envs at create)
  bool xg_on() const { return rng_mode == GP_RNG_NUMPY && B > xg_min; }
  bool xg_split = false;         // gp_debug_set("disable_fused", 1) at create: the two-launch draw calls (tests)
  bool xg_fused() const { return !XG_SPLIT_NORMALS && !xg_split && B <= XG_FUSE_MAX_ENVS; }  // one launch per call
  DevBuf xg_xend, xg_xinfo;      // the wall-noise extension of the action-noise call (XgCall::xinfo)
  DevBuf xg_bj, xg_hj;           // per-block base / halo jumps (XgCall::bj, hj) for the stream's increment
  // count sets in xg_cnt: 0 = the draw calls' positions, 1 = dry-step wall hits, 2 = resetting envs
  // One count set: acc (8-B atomics) | gs | bc, the set's size rounded up to 256 B so that every set's acc
  // array stays 8-byte aligned (a misaligned 64-bit atomic faults the queue; with an odd group count the
  // unrounded 12 * ng + 4 * cap bytes put set 1 on a 4-byte boundary).
  size_t xg_cnt_groups() const {
    const size_t nbp = (size_t)xg_P / XGT, cap = std::max(nbp, (size_t)xg_nbe);
    return cap / 64 + 1;
  }
  size_t xg_cnt_set_bytes() const {
    const size_t nbp = (size_t)xg_P / XGT, cap = std::max(nbp, (size_t)xg_nbe), ng = xg_cnt_groups();
    return (8 * ng + 4 * ng + 4 * cap + 255) & ~(size_t)255;
  }
  XgCounts xg_counts(int k) {
    const size_t ng = xg_cnt_groups();
    uint8_t* base = xg_cnt.as<uint8_t>() + (size_t)k * xg_cnt_set_bytes();
    XgCounts c{};
    c.acc = reinterpret_cast<unsigned long long*>(base);
    c.gs = reinterpret_cast<uint32_t*>(base + 8 * ng);
    c.bc = reinterpret_cast<uint32_t*>(base + 12 * ng);
    assert(((uintptr_t)c.acc & 7u) == 0);
    return c;
  }
  size_t xg_cnt_bytes() const { return 3 * xg_cnt_set_bytes(); }
  XgFlags xg_flags(int k) {  // k = 1 wall hits, 2 resets
    XgFlags f{};
    f.bits = xg_ebits.as<uint64_t>() + (size_t)(k - 1) * xg_nbe * XGW;
    f.c = xg_counts(k);
    return f;
  }
  XgCall xg_call(int64_t n_host, int nsrc, int nmul) {  // nsrc: n = nmul * (flagged envs of count set nsrc)
    XgCall a{};
    a.jt = xg_jt.as<PcgJump>();
    a.bj = xg_bj.as<PcgJump>();
    a.hj = xg_hj.as<PcgJump>();
    a.wj = x_wj.as<PcgJump>();
    a.st = x_rng.as<CrRng>();
    a.rd = xg_slot;
    a.wr = xg_slot ^ 1;
    if (nsrc) {
      a.nsrc = xg_counts(nsrc);
      a.nsrc_blocks = xg_nbe;
    }
    a.nmul = nmul;
    a.n_host = n_host;
    a.P = xg_P;
    a.bits = xg_bits.as<uint64_t>();
    a.pbits = xg_pbits.as<uint64_t>();
    a.bstate = xg_bstate.as<uint64_t>();
    a.span = xg_span.as<uint16_t>();
    a.val = xg_val.as<double>();
    a.pc = xg_counts(0);
    a.nv = (uint32_t)d.n_valid;
    a.lthr = xd.lemire_thr;
    a.err = derr.ptr();
    return a;
  }
  // ext: 1 = the action-noise call extended by the wall noise (xd.wall), 2 = the wall-noise call after it
  int xg_normals(int64_t n_host, int nsrc, int nmul, double scale, double* dst, hipStream_t s, int ext = 0) {
    XgCall a = xg_call(n_host, nsrc, nmul);
    a.scale = scale;
    a.dst = dst;
    if (ext && xg_fused()) {
      a.xinfo = xg_xinfo.as<uint32_t>();
      a.xend = xg_xend.as<uint32_t>();
      a.xdst = xd.wall;
      a.xmax = (uint32_t)(2 * B);
      a.xscale = 0.5;
    }
    // positions the launch covers (the extension's launch up to B / 2 normals past n: a 25% wall-hit rate)
    int64_t npos = xg_P;
    if (ext == 1 && a.xinfo) {
      const int64_t nx = n_host + B / 2;
      npos = std::min<int64_t>(npos, nx + nx / 16 + 4096);
    }
    const int pmin = gp_debug_knobs().xg_ppt_min >= 0 ? gp_debug_knobs().xg_ppt_min : XG_PPT_MIN_BLOCKS;
    const int ppt = xg_fused() && (npos + XGT - 1) / XGT > pmin ? 4 : 1;  // positions per thread
    const unsigned nbp = (unsigned)((npos + XGT * ppt - 1) / (XGT * ppt));
    if (ext == 2 && a.xinfo) {
      hipLaunchKernelGGL(xg_wall_one, dim3(1), dim3(XT), 0, s, a, xd);
    } else if (!xg_fused()) {
      hipLaunchKernelGGL(xg_norm_classify, dim3(nbp), dim3(XGT), 0, s, a);
      hipLaunchKernelGGL(xg_norm_write, dim3(nbp), dim3(XGT), 0, s, a);
    } else {
      a.tbc = xg_tbc.as<unsigned long long>();
      a.tgs = xg_tgs.as<unsigned long long>();
      a.tacc = xg_tacc.as<unsigned long long>();
      a.tag = xg_next_tag();
      if (ppt == 4) hipLaunchKernelGGL(xg_norm_fused<4>, dim3(nbp), dim3(XGT), 0, s, a);
      else hipLaunchKernelGGL(xg_norm_fused<1>, dim3(nbp), dim3(XGT), 0, s, a);
    }
    xg_slot ^= 1;
    GP_HIP_CHECK(hipGetLastError());
    return GP_OK;
  }
  int xg_choices(int64_t n_host, int nsrc, int32_t* dst, hipStream_t s) {
    XgCall a = xg_call(n_host, nsrc, 1);
    a.idst = dst;
    const unsigned nbc = (unsigned)((B / 2 + B / 1024 + 256 + XGT - 1) / XGT);
    if (!xg_fused()) {
      hipLaunchKernelGGL(xg_cho_count, dim3(nbc), dim3(XGT), 0, s, a);
      hipLaunchKernelGGL(xg_cho_write, dim3(nbc), dim3(XGT), 0, s, a);
    } else {
      a.tbc = xg_tbc.as<unsigned long long>();
      a.tgs = xg_tgs.as<unsigned long long>();
      a.tacc = xg_tacc.as<unsigned long long>();
      a.tag = xg_next_tag();
      hipLaunchKernelGGL(xg_cho_fused, dim3(nbc), dim3(XGT), 0, s, a);
    }
    xg_slot ^= 1;
    GP_HIP_CHECK(hipGetLastError());
    return GP_OK;
  }
  int xg_finish(hipStream_t s) {  // the current state back into slot 0 (what get_rng_state / the next call read)
    if (xg_slot) {
      hipLaunchKernelGGL(xg_copy_state, dim3(1), dim3(64), 0, s, x_rng.as<CrRng>(), 1, 0);
      xg_slot = 0;
    }
    GP_HIP_CHECK(hipGetLastError());
    return GP_OK;
  }
  int xg_reset(void* obs, hipStream_t s);
  int xg_rollout(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s);
  int xg_launches(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s);
  const uint64_t* rp_u = nullptr;
  const int32_t* rp_goal = nullptr;
  const int32_t* rp_agent = nullptr;
  const double* rp_noise = nullptr;
  const double* rp_wall = nullptr;

  int build(const gp_crooms_config* cfg);
  size_t rollout_action_bytes_per_env() const override {
    return d.action_kind == 0 ? (d.action_f64 ? 16 : 8) : 4;
  }
  int seed(const RngHost& r, const uint32_t key[2]) override {
    rng = r;
    d.key0 = key[0];
    d.key1 = key[1];
    philox_step = 0;
    if (int e = derr.clear()) return e;
    return rng_mode == GP_RNG_NUMPY ? x_upload_rng(r) : GP_OK;
  }
  int set_rng_state(const RngHost& r) override {
    if (rng_mode != GP_RNG_NUMPY) {
      gp_set_error("crooms: the PCG64 stream is used on the device only in numpy mode");
      return GP_E_UNSUPPORTED;
    }
    rng = r;
    return x_upload_rng(r);
  }
  int get_rng_state(RngHost* r) override {
    if (rng_mode != GP_RNG_NUMPY) {
      gp_set_error("crooms: the PCG64 stream is used on the device only in numpy mode");
      return GP_E_UNSUPPORTED;
    }
    GP_HIP_CHECK(hipDeviceSynchronize());
    CrRng h;
    GP_HIP_CHECK(hipMemcpy(&h, x_rng.p, sizeof(CrRng), hipMemcpyDeviceToHost));
    if (h.err) {
      gp_set_error("crooms numpy mode: a ziggurat tail attempt outran its word window; the stream is invalid");
      return GP_E_DEVICE;
    }
    r->state = mk128(h.s_hi, h.s_lo);
    r->inc = mk128(h.i_hi, h.i_lo);
    r->has_u32 = h.has_u32;
    r->uinteger = h.uinteger;
    rng = *r;
    return GP_OK;
  }
  int check() override {
    if (int e = derr.check("crooms")) return e;
    if (rng_mode != GP_RNG_NUMPY) return GP_OK;
    RngHost r;
    return get_rng_state(&r);
  }
  int x_launch(int K, int do_reset, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc,
               hipStream_t s) {
    CrDev dd = dev_for_launch();
    dd.rp_u = xd.u;          // the exact kernel's per-env draws, consumed by the replay step
    dd.rp_goal = xd.gi;
    dd.rp_agent = xd.ai;
    dd.rp_noise = xd.noise;
    dd.rp_wall = xd.wall;
    const CrExact xx = xd;
    int e = dispatch_obs(d.obs_kind, [&](auto okc) -> int {
      constexpr int OK = decltype(okc)::value;
      hipLaunchKernelGGL((crooms_numpy_rollout<OK>), dim3(1), dim3(XT), d.tab_bytes, s, dd, xx, K, do_reset, act,
                         obs, rew, term, trunc);
      return GP_OK;
    });
    if (e) return e;
    GP_HIP_CHECK(hipGetLastError());
    return GP_OK;
  }
  // the configuration crooms_rollout<GP_OBS_F32, false, 1> is compiled for (cr_action_kind & co.)
  bool generic = false;  // gp_debug_set("generic_kernels") at creation
  bool spec1() const {
    return !generic && d.obs_kind == GP_OBS_F32 && !d.obs_f64 && d.action_kind == 0 && !d.action_f64 && !d.use_velocity &&
           d.goal_fixed;
  }
  CrDev dev_for_launch() const {
    CrDev dd = d;
    dd.rp_u = rp_u;
    dd.rp_goal = rp_goal;
    dd.rp_agent = rp_agent;
    dd.rp_noise = rp_noise;
    dd.rp_wall = rp_wall;
    return dd;
  }
  int reset(void* obs, hipStream_t s) override {
    GP_HIP_CHECK(hipMemsetAsync(d.mslot, 0, sizeof(CrSlot) * grid, s));
    if (rng_mode == GP_RNG_REPLAY && ((!d.goal_fixed && !rp_goal) || (!d.agent_fixed && !rp_agent))) {
      gp_set_error("crooms replay reset needs goal/agent index draws (gp_set_replay i0/i1)");
      return GP_E_STATE;
    }
    if (rng_mode == GP_RNG_NUMPY) {
      int e = xg_on() ? xg_reset(obs, s) : x_launch(0, 1, nullptr, obs, nullptr, nullptr, nullptr, s);
      if (e) return e;
      has_reset = true;
      return GP_OK;
    }
    const CrDev dd = dev_for_launch();
    const bool rep = rng_mode == GP_RNG_REPLAY;
    const uint64_t st = philox_step;
    int e = dispatch_obs(d.obs_kind, [&](auto okc) -> int {
      constexpr int OK = decltype(okc)::value;
      if (rep) hipLaunchKernelGGL((crooms_reset<OK, true>), dim3(grid), dim3(TPB), d.tab_bytes, s, dd, st, obs);
      else hipLaunchKernelGGL((crooms_reset<OK, false>), dim3(grid), dim3(TPB), d.tab_bytes, s, dd, st, obs);
      return GP_OK;
    });
    if (e) return e;
    GP_HIP_CHECK(hipGetLastError());
    if (!rep) ++philox_step;
    has_reset = true;
    return GP_OK;
  }
  int rollout(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) override {
    if (!has_reset) {
      gp_set_error("step() before reset()");
      return GP_E_STATE;
    }
    const bool rep = rng_mode == GP_RNG_REPLAY;
    if (rep) {
      if ((d.action_kind == 0 || d.action_std != 0.0) && !rp_noise) {
        gp_set_error("crooms replay step needs action noise (gp_set_replay f0)");
        return GP_E_STATE;
      }
      if (d.action_kind != 0 && !rp_u) {
        gp_set_error("crooms replay step needs action-failure uniforms (gp_set_replay u)");
        return GP_E_STATE;
      }
      if (!rp_wall || (!d.goal_fixed && !rp_goal) || (!d.agent_fixed && !rp_agent)) {
        gp_set_error("crooms replay step needs wall noise (f1) and reset indices (i0/i1)");
        return GP_E_STATE;
      }
      if (K > 1) return EnvBackend::rollout(K, act, obs, rew, term, trunc, s);
    }
    auto al = [](const void* x, uintptr_t m) { return ((uintptr_t)x & (m - 1)) == 0; };
    if (!al(act, d.action_kind == 0 ? (d.action_f64 ? 16 : 8) : 4) || !al(obs, 16) || !al(rew, 4)) {
      gp_set_error("crooms: misaligned action / obs / reward buffer");
      return GP_E_INVALID;
    }
    if (rng_mode == GP_RNG_NUMPY) {
      timer.begin(s);
      int e = xg_on() ? xg_rollout(K, act, obs, rew, term, trunc, s) : x_launch(K, 0, act, obs, rew, term, trunc, s);
      timer.end(s);
      return e;
    }
    const CrDev dd = dev_for_launch();
    const uint64_t st = philox_step;
    int e = dispatch_obs(d.obs_kind, [&](auto okc) -> int {
      constexpr int OK = decltype(okc)::value;
      timer.begin(s);
      if (rep)
        hipLaunchKernelGGL((crooms_rollout<OK, true>), dim3(grid), dim3(TPB), d.tab_bytes, s, dd, K, st, act, obs,
                           rew, term, trunc);
      else if (OK == GP_OBS_F32 && spec1())  // configs[4]'s shape, compiled for it
        hipLaunchKernelGGL((crooms_rollout<GP_OBS_F32, false, 1>), dim3(grid), dim3(TPB), d.tab_bytes, s, dd, K, st,
                           act, obs, rew, term, trunc);
      else
        hipLaunchKernelGGL((crooms_rollout<OK, false>), dim3(grid), dim3(TPB), d.tab_bytes, s, dd, K, st, act, obs,
                           rew, term, trunc);
      timer.end(s);
      return GP_OK;
    });
    if (e) return e;
    GP_HIP_CHECK(hipGetLastError());
    if (!rep) philox_step += (uint64_t)K;
    return GP_OK;
  }
  int step(const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) override {
    return rollout(1, act, obs, rew, term, trunc, s);
  }
  int get_state(void* a, void* b, void* c, void* e, hipStream_t s) override {
    hipLaunchKernelGGL(crooms_get_state, dim3((unsigned)((B + TPB - 1) / TPB)), dim3(TPB), 0, s, d, (double*)a,
                       (int32_t*)b, (double*)c, (int32_t*)e);
    GP_HIP_CHECK(hipGetLastError());
    return GP_OK;
  }
  int set_state(const void* a, const void* b, const void* c, const void* e, hipStream_t s) override {
    hipLaunchKernelGGL(crooms_set_state, dim3((unsigned)((B + TPB - 1) / TPB)), dim3(TPB), 0, s, d,
                       (const double*)a, (const int32_t*)b, (const double*)c, (const int32_t*)e);
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
    rp_noise = (const double*)f0;
    rp_wall = (const double*)f1;
    return GP_OK;
  }
  int valid_cells(int which, int32_t* out, int cap) const override {
    for (int i = 0; i < (int)valid_h.size() && i < cap; ++i) out[i] = valid_h[i];
    return (int)valid_h.size();
  }
  int metrics(double out[4]) override {
    GP_HIP_CHECK(hipDeviceSynchronize());
    std::vector<CrSlot> m(grid);
    GP_HIP_CHECK(hipMemcpy(m.data(), d.mslot, sizeof(CrSlot) * grid, hipMemcpyDeviceToHost));
    out[0] = out[1] = out[2] = out[3] = 0;
    for (const CrSlot& x : m) {
      out[0] += (double)x.episodes;
      out[1] += x.return_sum;
      out[2] += (double)x.length_sum;
      out[3] += (double)x.env_steps;
    }
    return check();  // device errors (invalid actions; numpy mode: an invalid stream) invalidate the run
  }
};

// Largest double S with sqrt(S) <= thr (IEEE sqrt is correctly rounded and monotone).
static double sq_threshold(double thr) {
  if (!(thr >= 0.0)) return -1.0;
  double lo = 0.0, hi = std::max(thr * thr * 4.0, 1.0);
  while (std::sqrt(hi) <= thr) hi *= 2.0;
  uint64_t a, b;
  memcpy(&a, &lo, 8);
  memcpy(&b, &hi, 8);  // invariant: sqrt(bits a) <= thr < sqrt(bits b)
  while (b - a > 1) {
    const uint64_t m = a + (b - a) / 2;
    double x;
    memcpy(&x, &m, 8);
    if (std::sqrt(x) <= thr) a = m; else b = m;
  }
  double r;
  memcpy(&r, &a, 8);
  return r;
}

int CRoomsBackend::build(const gp_crooms_config* cfg) {
  generic = gp_debug_knobs().generic_kernels != 0;
  static const int DY8[8] = {-1, -1, 0, 1, 1, 1, 0, -1}, DX8[8] = {0, 1, 1, 1, 0, -1, -1, -1};
  const int H = cfg->height, W = cfg->width, nc = H * W;
  if (H < 3 || W < 3 || nc >= 32768 || !cfg->cells) {
    gp_set_error("crooms: grid %dx%d unsupported", H, W);
    return GP_E_INVALID;
  }
  if (!(cfg->cell_size >= 1.0)) {
    gp_set_error("crooms: cell_size %g < 1 indexes past the grid (the reference raises IndexError)", cfg->cell_size);
    return GP_E_INVALID;
  }
  if (cfg->action_kind != 0 && cfg->action_kind != 4 && cfg->action_kind != 8) {
    gp_set_error("crooms: action_kind must be 0 (yx), 4 or 8");
    return GP_E_INVALID;
  }
  if (cfg->time_limit < 0) {
    gp_set_error("crooms: negative time_limit");
    return GP_E_INVALID;
  }
  std::vector<int32_t> cells(cfg->cells, cfg->cells + nc);
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x)
      if (cells[y * W + x] >= 0 && (y == 0 || x == 0 || y == H - 1 || x == W - 1)) {
        gp_set_error("crooms: walkable cell on the map border");
        return GP_E_INVALID;
      }
  d.H = H;
  d.W = W;
  d.ncells = nc;
  d.use_velocity = cfg->use_velocity != 0;
  d.action_kind = cfg->action_kind;
  d.action_f64 = cfg->action_f64 != 0;
  d.nact = cfg->action_kind == 0 ? 0 : cfg->action_kind;
  d.cell = cfg->cell_size;
  d.half_cell = cfg->cell_size / 2;
  {
    int ex = 0;
    const double m = std::frexp(cfg->cell_size, &ex);
    d.inv_cell = (m == 0.5 && cfg->cell_size > 0) ? 1.0 / cfg->cell_size : 0.0;  // exact reciprocal of 2^k
  }
  d.hi_y = (double)(H - 1) - 1e-6;  // gridshape - 1 - 1e-6 (crooms.py:311-313)
  d.hi_x = (double)(W - 1) - 1e-6;
  d.s_thr = sq_threshold(cfg->goal_threshold);
  d.action_std = cfg->action_std;
  d.action_power = cfg->action_power;
  d.time_limit = cfg->time_limit;
  d.r_step = cfg->step_reward;
  d.r_wall = cfg->wall_reward;
  d.r_goal = cfg->goal_reward;
  d.goal_fixed = cfg->goal_fixed != 0;
  d.goal_y = cfg->goal_y;
  d.goal_x = cfg->goal_x;
  d.gcy = (double)(int16_t)(cfg->goal_y & 0xFFFF) + 0.5;  // what the packed int16 goal word decodes to
  d.gcx = (double)(int16_t)(cfg->goal_x & 0xFFFF) + 0.5;
  d.agent_fixed = cfg->agent_fixed != 0;
  d.agent_y = cfg->agent_y;
  d.agent_x = cfg->agent_x;
  if (d.goal_fixed && (d.goal_y < -32768 || d.goal_y > 32767 || d.goal_x < -32768 || d.goal_x > 32767)) {
    gp_set_error("crooms: fixed goal out of range");
    return GP_E_INVALID;
  }
  if (d.agent_fixed && (d.agent_y < 0 || d.agent_x < 0 || d.agent_y >= H || d.agent_x >= W)) {
    gp_set_error("crooms: fixed agent outside the grid");
    return GP_E_INVALID;
  }
  valid_h.clear();
  for (int c = 0; c < nc; ++c)
    if (cells[c] >= 0) valid_h.push_back(c);  // np.flatnonzero(grid >= 0) (crooms.py:165)
  if (valid_h.empty()) {
    gp_set_error("crooms: no valid cells");
    return GP_E_INVALID;
  }
  d.n_valid = (int)valid_h.size();
  // tables
  std::vector<uint8_t> wall(nc);
  for (int c = 0; c < nc; ++c) wall[c] = cells[c] == -1 ? 1 : 0;  // _out_of_bounds: grid == -1 (:333-338)
  // valid cells as (y | x << 16) (the goal's own packing), so a reset needs no integer divide
  std::vector<uint32_t> valid(valid_h.size());
  for (size_t i = 0; i < valid_h.size(); ++i)
    valid[i] = (uint32_t)(valid_h[i] / W) | ((uint32_t)(valid_h[i] % W) << 16);
  std::vector<uint64_t> thr;
  if (d.nact) {
    thr.assign((size_t)d.nact * d.nact, 0);
    const double pf = cfg->action_failure_probability, off = pf / (d.nact - 1);
    for (int a = 0; a < d.nact; ++a) {
      double s = 0.0;
      for (int j = 0; j < d.nact; ++j) {
        s += (j == a) ? (1 - pf) : off;
        const double x = std::ldexp(s, 53);
        thr[(size_t)a * d.nact + j] = x >= 18446744073709551615.0 ? ~0ull : (uint64_t)std::floor(x);
      }
    }
  }
  d.obs_kind = cfg->obs_kind;
  d.obs_f64 = cfg->obs_f64 != 0;
  d.obs_dirs = cfg->obs_dirs;
  d.obs_goal = cfg->obs_goal != 0;
  d.obs_n = cfg->obs_n;
  std::vector<int32_t> doff(8, 0x7FFFFFFF), t1, t2;
  std::vector<uint32_t> hbase;
  std::vector<uint8_t> hvec, window;
  switch (cfg->obs_kind) {
    case GP_OBS_F32:
      obs_dtype = d.obs_f64 ? GP_DTYPE_F64 : GP_DTYPE_F32;
      obs_width = d.obs_goal ? 4 : 2;
      break;
    case GP_OBS_HANSEN:
    case GP_OBS_HANSEN_VEC: {
      if (cfg->obs_dirs != 4 && cfg->obs_dirs != 8) {
        gp_set_error("crooms: obs_dirs must be 4 or 8");
        return GP_E_INVALID;
      }
      hbase.assign(nc, 0);
      hvec.assign((size_t)nc * cfg->obs_dirs, 0);
      for (int i = 0; i < cfg->obs_dirs; ++i) {
        const int o = cfg->obs_dirs == 4 ? 2 * i : i;
        doff[i] = DY8[o] * W + DX8[o];
      }
      for (int c = 0; c < nc; ++c) {
        const int y = c / W, x = c % W;
        uint32_t hb = 0;
        for (int i = 0; i < cfg->obs_dirs; ++i) {
          const int o = cfg->obs_dirs == 4 ? 2 * i : i;
          const int ny = y + DY8[o], nx = x + DX8[o];
          const int dg = (ny >= 0 && nx >= 0 && ny < H && nx < W && cells[ny * W + nx] >= 0) ? 1 : 0;
          hb += (uint32_t)dg << i;  // observations.py:44-71 (binary)
          hvec[(size_t)c * cfg->obs_dirs + i] = (uint8_t)dg;
        }
        hbase[c] = hb;
      }
      obs_dtype = cfg->obs_kind == GP_OBS_HANSEN ? GP_DTYPE_I32 : GP_DTYPE_U8;
      obs_width = cfg->obs_kind == GP_OBS_HANSEN ? 1 : cfg->obs_dirs;
      break;
    }
    case GP_OBS_TABLE:
      if (!cfg->obs_table) {
        gp_set_error("crooms: GP_OBS_TABLE needs obs_table");
        return GP_E_INVALID;
      }
      t1.assign(cfg->obs_table, cfg->obs_table + nc);
      if (cfg->obs_table2) {
        if (d.goal_fixed && (d.goal_y < 0 || d.goal_x < 0 || d.goal_y >= H || d.goal_x >= W)) {
          gp_set_error("crooms: goal outside the grid cannot index the goal obs table (reference raises)");
          return GP_E_INVALID;
        }
        t2.assign(cfg->obs_table2, cfg->obs_table2 + nc);
      }
      obs_dtype = GP_DTYPE_I32;
      obs_width = 1;
      break;
    case GP_OBS_WINDOW: {
      const int n = cfg->obs_n, h = n / 2;
      if (n < 1 || n > 63) {
        gp_set_error("crooms: obs_n must be in [1, 63]");
        return GP_E_INVALID;
      }
      window.assign((size_t)nc * n * n, 0);
      for (int c = 0; c < nc; ++c) {
        const int y = c / W, x = c % W;
        for (int i = 0; i < n; ++i)
          for (int j = 0; j < n; ++j) {
            int yy = y + i - h, xx = x + j - h;
            if (yy < 0 || xx < 0 || yy >= H || xx >= W) yy = xx = 0;  // observations.py:92-98
            window[((size_t)c * n + i) * n + j] = (uint8_t)(cells[yy * W + xx] + 1 > 0 ? 1 : 0);
          }
      }
      obs_dtype = GP_DTYPE_U8;
      obs_width = n * n;
      break;
    }
    default:
      gp_set_error("crooms: obs kind %d not supported", cfg->obs_kind);
      return GP_E_INVALID;
  }
  d.obs_width = obs_width;
  d.has_t2 = !t2.empty();
  // pack the tables (16-B aligned sections)
  std::vector<uint8_t> blob;
  auto put = [&](const void* src, size_t bytes) -> int32_t {
    const size_t off = (blob.size() + 15) & ~(size_t)15;
    blob.resize(off + bytes);
    if (bytes) memcpy(blob.data() + off, src, bytes);
    return (int32_t)off;
  };
  d.off_thr = put(thr.data(), thr.size() * 8);
  d.off_wall = put(wall.data(), wall.size());
  d.off_valid = put(valid.data(), valid.size() * 4);
  d.off_t1 = put(t1.data(), t1.size() * 4);
  d.off_t2 = put(t2.data(), t2.size() * 4);
  d.off_hbase = put(hbase.data(), hbase.size() * 4);
  d.off_hvec = put(hvec.data(), hvec.size());
  d.off_doff = put(doff.data(), doff.size() * 4);
  d.off_window = put(window.data(), window.size());
  blob.resize((blob.size() + 15) & ~(size_t)15);
  d.tab_bytes = (int32_t)blob.size();
  if (d.tab_bytes > 96 * 1024) {
    gp_set_error("crooms: tables (%d B) exceed the LDS budget", d.tab_bytes);
    return GP_E_INVALID;
  }
  int e;
  if ((e = b_tabs.upload(blob))) return e;
  d.tabs = b_tabs.as<uint8_t>();
  d.B = (int32_t)B;
  d.ntiles = (int32_t)((B + EPB - 1) / EPB);
  if ((e = b_ay.alloc((size_t)B * 8)) || (e = b_ax.alloc((size_t)B * 8)) || (e = b_el.alloc((size_t)B * 4)) ||
      (e = b_goal.alloc((size_t)B * 4)))
    return e;
  if (d.use_velocity && ((e = b_vy.alloc((size_t)B * 8)) || (e = b_vx.alloc((size_t)B * 8)))) return e;
  d.ay = b_ay.as<double>();
  d.ax = b_ax.as<double>();
  d.vy = b_vy.as<double>();
  d.vx = b_vx.as<double>();
  d.el = b_el.as<int32_t>();
  d.goal = b_goal.as<uint32_t>();
  hipDeviceProp_t prop;
  GP_HIP_CHECK(hipGetDeviceProperties(&prop, device));
  int occ = 0;
  GP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, crooms_rollout<GP_OBS_F32, false>, TPB, d.tab_bytes));
  grid = persistent_grid(d.ntiles, prop.multiProcessorCount, occ);
  persist_grid = grid;
  persist_occ = occ;
  if ((e = b_slot.alloc(sizeof(CrSlot) * grid))) return e;
  d.mslot = b_slot.as<CrSlot>();
  d.nslot = grid;
  if ((e = derr.alloc())) return e;
  d.derr = derr.ptr();
  xg_split = gp_debug_knobs().disable_fused != 0;
  xg_graph_mode = gp_xg_graph_knob;
  if (rng_mode == GP_RNG_NUMPY && (e = x_alloc())) return e;
  return GP_OK;
}

int CRoomsBackend::x_alloc() {
  int e;
  const size_t b = (size_t)B;
  if ((e = x_rng.alloc(2 * sizeof(CrRng))) || (e = x_wj.alloc(sizeof(PcgJump) * (XW + 1))) ||
      (e = x_noise.alloc(16 * b)) || (e = x_wall.alloc(16 * b)) || (e = x_dense.alloc(16 * b)) ||
      (e = x_u.alloc(8 * b)) || (e = x_gi.alloc(4 * b)) || (e = x_ai.alloc(4 * b)) || (e = x_rank.alloc(4 * b)))
    return e;
  xd.rng = x_rng.as<CrRng>();
  xd.wj = x_wj.as<PcgJump>();
  xd.noise = x_noise.as<double>();
  xd.wall = x_wall.as<double>();
  xd.dense = x_dense.as<double>();
  xd.u = x_u.as<uint64_t>();
  xd.gi = x_gi.as<int32_t>();
  xd.ai = x_ai.as<int32_t>();
  xd.rank = x_rank.as<int32_t>();
  xd.lemire_thr = lemire_threshold((uint32_t)d.n_valid);
  if (gp_debug_knobs().xg_min_envs >= 0) xg_min = gp_debug_knobs().xg_min_envs;
  if (B > xg_min) {
    // positions of a draw call: normal(2B) needs 2B + 2B / 16 + 4096 at most (xg_norm_need), rounded to blocks;
    // with the wall-noise extension (fused calls) up to 2B more normals
    const int64_t nmax = (xg_fused() ? 4 : 2) * b;
    const int64_t P = ((nmax + nmax / 16 + 4096 + 64 * XGT - 1) / (64 * XGT)) * (64 * XGT);
    if (P > (int64_t)1 << 30) {
      gp_set_error("crooms numpy mode: num_envs too large");
      return GP_E_INVALID;
    }
    xg_P = (int)P;
    xg_nbe = (int)((b + XGT - 1) / XGT);
    const size_t nbp = (size_t)P / XGT + 1;
    if ((e = xg_jt.alloc(sizeof(PcgJump) * JT_LEVELS * JT_RADIX)) || (e = xg_bits.alloc((size_t)P / 8)) ||
        (e = xg_pbits.alloc((size_t)P / 8)) || (e = xg_bstate.alloc(16 * nbp)) || (e = xg_span.alloc(2 * (size_t)P)) ||
        (e = xg_val.alloc(8 * (size_t)P)) || (e = xg_cnt.alloc(xg_cnt_bytes())) ||
        (e = xg_ebits.alloc(2 * 8 * (size_t)xg_nbe * XGW)) || (e = xg_tbc.alloc(8 * (nbp + 64))) ||
        (e = xg_tgs.alloc(8 * (nbp / 64 + 2))) || (e = xg_tacc.alloc(8 * (nbp / 64 + 2))))
      return e;
    GP_HIP_CHECK(hipMemset(xg_cnt.p, 0, xg_cnt_bytes()));  // the group accumulators start (and stay) cleared
    if ((e = xg_bj.alloc(sizeof(PcgJump) * (nbp + 1))) || (e = xg_hj.alloc(sizeof(PcgJump) * (nbp + 1)))) return e;
    if (xg_fused()) {
      if ((e = xg_xend.alloc(4 * 2 * b)) || (e = xg_xinfo.alloc(16))) return e;
      GP_HIP_CHECK(hipMemset(xg_xinfo.p, 0, 16));
    }
#ifdef GP_STAMPS
    if ((e = xg_dbg.alloc(8 * 6 * 1024 * 8))) return e;
    GP_HIP_CHECK(hipMemset(xg_dbg.p, 0, 8 * 6 * 1024 * 8));
    GP_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_xgdbg), &xg_dbg.p, sizeof(void*)));
#endif
  }
  return x_upload_rng(rng);
}

int CRoomsBackend::xg_reset(void* obs, hipStream_t s) {  // crooms.py:251-266: goal then agent for every env
  xg_slot = 0;
  int e;
  if (!d.goal_fixed && (e = xg_choices(B, 0, xd.gi, s))) return e;
  if (!d.agent_fixed && (e = xg_choices(B, 0, xd.ai, s))) return e;
  XgFlags ev{};  // every env, by env index
  const CrDev dd = dev_for_launch();
  const unsigned nbe = (unsigned)((B + XGT - 1) / XGT);
  e = dispatch_obs(d.obs_kind, [&](auto okc) -> int {
    constexpr int OK = decltype(okc)::value;
    hipLaunchKernelGGL(xg_apply_resets<OK>, dim3(nbe), dim3(XGT), d.tab_bytes, s, dd, ev, (const int32_t*)xd.gi,
                       (const int32_t*)xd.ai, obs);
    return GP_OK;
  });
  if (e) return e;
  return xg_finish(s);
}

int CRoomsBackend::xg_rollout(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc,
                              hipStream_t s) {
  if (xg_graph_mode == 0 || (xg_graph_mode < 0 && B > XG_GRAPH_MAX_ENVS) || xg_graph_broken || !xg_fused())
    return xg_launches(K, act, obs, rew, term, trunc, s);
  XgGraphKey key;
  key.K = K;
  key.act = act;
  key.obs = obs;
  key.rew = rew;
  key.term = term;
  key.trunc = trunc;
  key.spb = gp_debug_knobs().xg_spb_min;
  key.ppt = gp_debug_knobs().xg_ppt_min;
  if (!(xg_gexec && key == xg_gkey)) {
    const bool again = key == xg_glast;
    xg_glast = key;
    if (xg_graph_mode < 0 && !again) return xg_launches(K, act, obs, rew, term, trunc, s);
    if (xg_graph_capture(key, act, obs, rew, term, trunc)) return xg_launches(K, act, obs, rew, term, trunc, s);
  }
  GP_HIP_CHECK(hipGraphLaunch(xg_gexec, s));
  return GP_OK;
}

// Captures xg_launches(K, ...) plus the clearing of the tagged count slots into xg_gexec; nonzero (and eager
// launches from then on) if the runtime refuses any of it.
int CRoomsBackend::xg_graph_capture(const XgGraphKey& key, const void* act, void* obs, float* rew, uint8_t* term,
                                    uint8_t* trunc) {
  xg_graph_drop();
  if (!xg_cap && hipStreamCreateWithFlags(&xg_cap, hipStreamNonBlocking) != hipSuccess) {
    xg_cap = nullptr;
    xg_graph_broken = true;
    return 1;
  }
  if (hipStreamBeginCapture(xg_cap, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    (void)hipGetLastError();
    xg_graph_broken = true;
    return 1;
  }
  xg_capturing = true;
  xg_gtag = 0;
  int e = xg_launches(key.K, act, obs, rew, term, trunc, xg_cap);
  xg_capturing = false;
  if (!e && (hipMemsetAsync(xg_tbc.p, 0, xg_tbc.n, xg_cap) != hipSuccess ||
             hipMemsetAsync(xg_tgs.p, 0, xg_tgs.n, xg_cap) != hipSuccess))
    e = 1;
  hipGraph_t g = nullptr;
  if (hipStreamEndCapture(xg_cap, &g) != hipSuccess || !g) e = 1;
  if (!e && hipGraphInstantiate(&xg_gexec, g, nullptr, nullptr, 0) != hipSuccess) {
    xg_gexec = nullptr;
    e = 1;
  }
  xg_slot = 0;
  if (e) {
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    xg_graph_broken = true;
    return 1;
  }
  xg_graph = g;
  xg_gkey = key;
  return 0;
}

int CRoomsBackend::xg_launches(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc,
                               hipStream_t s) {
  xg_slot = 0;
  CrDev dd = dev_for_launch();
  dd.rp_u = xd.u;  // the per-env draws of the call sequence, consumed by the replay step
  dd.rp_goal = xd.gi;
  dd.rp_agent = xd.ai;
  dd.rp_noise = xd.noise;
  dd.rp_wall = xd.wall;
  const unsigned nbe = (unsigned)((B + XGT - 1) / XGT);
  const size_t osz = (size_t)d.obs_width * (d.obs_kind == GP_OBS_F32 ? (d.obs_f64 ? 8 : 4)
                                            : (d.obs_kind == GP_OBS_HANSEN || d.obs_kind == GP_OBS_TABLE ? 4 : 1));
  const XgFlags fd = xg_flags(1), fs = xg_flags(2);  // wall hits of the dry step, resets of the step
  const int spb_min = gp_debug_knobs().xg_spb_min >= 0 ? gp_debug_knobs().xg_spb_min : XG_SPB_MIN_BLOCKS;
  int e;
  for (int k = 0; k < K; ++k) {
    const size_t off = (size_t)k * B;
    uint8_t* ob = (uint8_t*)obs + off * osz;
    // _sample_action's draws (crooms.py:175-198)
    if (d.action_kind != 0) {
      XgCall a = xg_call(B, 0, 1);
      hipLaunchKernelGGL(xg_uniforms, dim3(nbe), dim3(XGT), 0, s, a, xd.u);
      xg_slot ^= 1;
    }
    const bool noise = d.action_kind == 0 || d.action_std != 0.0;
    if (noise && (e = xg_normals(2 * B, 0, 1, d.action_std, xd.noise, s, 1))) return e;
    // the dry step: which envs hit a wall; their noise normal(0.5, (n_oob, 2)) (crooms.py:321-325)
    e = dispatch_obs(d.obs_kind, [&](auto okc) -> int {
      constexpr int OK = decltype(okc)::value;
      const XgFlags fr = k ? fs : XgFlags{};
      void* op = k ? (void*)(ob - B * osz) : nullptr;
      if ((int)nbe > spb_min)
        hipLaunchKernelGGL((xg_dry<OK, 4>), dim3((nbe + 3) / 4), dim3(XGT), d.tab_bytes, s, dd, fd, act, off, fr,
                           (const int32_t*)xd.gi, (const int32_t*)xd.ai, op, (int)nbe);
      else
        hipLaunchKernelGGL((xg_dry<OK, 1>), dim3(nbe), dim3(XGT), d.tab_bytes, s, dd, fd, act, off, fr,
                           (const int32_t*)xd.gi, (const int32_t*)xd.ai, op, (int)nbe);
      return GP_OK;
    });
    if (e || (e = xg_normals(0, 1, 2, 0.5, xd.wall, s, noise ? 2 : 0))) return e;
    // the step itself with the wall noise in place, resets deferred; then the resetting envs' goals / agents
    e = dispatch_obs(d.obs_kind, [&](auto okc) -> int {
      constexpr int OK = decltype(okc)::value;
      if ((int)nbe > spb_min)
        hipLaunchKernelGGL((xg_step<OK, 4>), dim3((nbe + 3) / 4), dim3(XGT), d.tab_bytes, s, dd, fd, fs, act, off,
                           (void*)ob, rew, term, trunc, (int)nbe);
      else
        hipLaunchKernelGGL((xg_step<OK, 1>), dim3(nbe), dim3(XGT), d.tab_bytes, s, dd, fd, fs, act, off, (void*)ob,
                           rew, term, trunc, (int)nbe);
      return GP_OK;
    });
    if (e) return e;
    if (!d.goal_fixed && (e = xg_choices(0, 2, xd.gi, s))) return e;
    if (!d.agent_fixed && (e = xg_choices(0, 2, xd.ai, s))) return e;
    if (k + 1 < K) continue;  // the next step's dry kernel applies these resets
    e = dispatch_obs(d.obs_kind, [&](auto okc) -> int {
      constexpr int OK = decltype(okc)::value;
      hipLaunchKernelGGL(xg_apply_resets<OK>, dim3(nbe), dim3(XGT), d.tab_bytes, s, dd, fs, (const int32_t*)xd.gi,
                         (const int32_t*)xd.ai, (void*)ob);
      return GP_OK;
    });
    if (e) return e;
  }
  return xg_finish(s);
}

// The device stream state and the window jump table wj[j] = j LCG steps (j = 0..XW) for its increment.
int CRoomsBackend::x_upload_rng(const RngHost& r) {
  std::vector<PcgJump> wj(XW + 1);
  u128 a = 1, c = 0;
  for (int j = 0; j <= XW; ++j) {
    wj[j] = PcgJump{hi64(a), lo64(a), hi64(c), lo64(c)};
    a = pcg_mult() * a;
    c = pcg_mult() * c + r.inc;
  }
  GP_HIP_CHECK(hipDeviceSynchronize());
  GP_HIP_CHECK(hipMemcpy(x_wj.p, wj.data(), sizeof(PcgJump) * wj.size(), hipMemcpyHostToDevice));
  if (xg_jt.p) {
    const std::vector<PcgJump> jt = build_jump_tables(r.inc);
    GP_HIP_CHECK(hipMemcpy(xg_jt.p, jt.data(), sizeof(PcgJump) * jt.size(), hipMemcpyHostToDevice));
    // per-block jumps: bj[b] = b * XGT steps, hj[b] = b * XGT - XG_LOOK steps (= XGT - XG_LOOK after bj[b - 1])
    const size_t nb = xg_bj.n / sizeof(PcgJump);
    std::vector<PcgJump> bj(nb), hj(nb);
    const PcgJump J = pcg_jump_params((u128)XGT, r.inc), Jh = pcg_jump_params((u128)(XGT - XG_LOOK), r.inc);
    auto after = [](const PcgJump& second, const PcgJump& first) {  // second o first
      const u128 A2 = mk128(second.a_hi, second.a_lo), C2 = mk128(second.c_hi, second.c_lo);
      const u128 A = A2 * mk128(first.a_hi, first.a_lo), C = A2 * mk128(first.c_hi, first.c_lo) + C2;
      return PcgJump{hi64(A), lo64(A), hi64(C), lo64(C)};
    };
    bj[0] = hj[0] = PcgJump{0, 1, 0, 0};
    for (size_t k = 1; k < nb; ++k) {
      bj[k] = after(J, bj[k - 1]);
      hj[k] = after(Jh, bj[k - 1]);
    }
    GP_HIP_CHECK(hipMemcpy(xg_bj.p, bj.data(), sizeof(PcgJump) * nb, hipMemcpyHostToDevice));
    GP_HIP_CHECK(hipMemcpy(xg_hj.p, hj.data(), sizeof(PcgJump) * nb, hipMemcpyHostToDevice));
  }
  xg_slot = 0;
  CrRng h{hi64(r.state), lo64(r.state), hi64(r.inc), lo64(r.inc), r.has_u32, r.uinteger, 0u, 0u};
  GP_HIP_CHECK(hipMemcpy(x_rng.p, &h, sizeof(CrRng), hipMemcpyHostToDevice));
  return GP_OK;
}

}  // namespace

// ---- diagnostics of the normal sampler (C ABI below) ----
namespace {

// The caller's words in order; past the end it returns 0 and sets `dry` (a wedge / tail draw of the current
// normal ran past the words: that normal is NaN, and zig_dry ends its tail loop).
struct ZigWordSource {
  const uint64_t* w;
  int64_t nw, pos;
  bool dry;
  __device__ uint64_t operator()() {
    if (pos < nw) return w[pos++];
    dry = true;
    return 0ull;
  }
};
__device__ __forceinline__ bool zig_dry(const ZigWordSource& s) { return s.dry; }

// numpy's standard_normal over a caller word stream, one lane, in order (numpy consumes the words
// sequentially and a normal may take several).
__global__ void zig_words_kernel(const uint64_t* __restrict__ w, int64_t nw, double* __restrict__ out, int64_t n,
                                 int64_t* __restrict__ used) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const ZigTabs t{d_zig, reinterpret_cast<const double*>(d_zig + 256), reinterpret_cast<const double*>(d_zig + 512)};
  ZigWordSource next{w, nw, 0, false};
  for (int64_t i = 0; i < n; ++i) {
    if (next.pos >= nw) {
      out[i] = __builtin_nan("");
      continue;
    }
    const uint64_t r = w[next.pos++];
    next.dry = false;
    const double z = zig_normal(t, r, next);
    out[i] = next.dry ? __builtin_nan("") : z;
  }
  *used = next.pos;
}

// n normals of the philox-mode sampler (counter (i, 0, 0, TAG_NOISE) for the pair 2i, 2i+1, as
// draw_normals): exceedance counts |z| > thr[j] and the sum / sum of squares, without storing them.
constexpr int ZT_MAX = 8;
__global__ __launch_bounds__(256) void zig_tail_kernel(uint32_t k0, uint32_t k1, uint64_t npairs, const double* __restrict__ thr,
                                                       int nthr, unsigned long long* __restrict__ counts,
                                                       double* __restrict__ mom) {
  __shared__ uint64_t zt[768];
  __shared__ double sthr[ZT_MAX];
  for (int i = threadIdx.x; i < 768; i += blockDim.x) zt[i] = d_zig[i];
  if (threadIdx.x < ZT_MAX) sthr[threadIdx.x] = threadIdx.x < nthr ? thr[threadIdx.x] : 1e300;
  __syncthreads();
  ZigTabs t;  // (member-wise: a braced initializer of LDS addresses is folded into an invalid static one)
  t.ki = zt;
  t.wi = reinterpret_cast<const double*>(zt + 256);
  t.fi = reinterpret_cast<const double*>(zt + 512);
  unsigned long long c[ZT_MAX] = {};
  double s1 = 0.0, s2 = 0.0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < npairs; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t e = (uint32_t)i, s0 = (uint32_t)(i >> 32);
    const Philox4 r = philox4x32<CR_PHILOX_ROUNDS>(e, s0, 0u, TAG_NOISE, k0, k1);
    double z0, z1;
    box_muller_pair(((uint64_t)r.x[1] << 32) | r.x[0], ((uint64_t)r.x[3] << 32) | r.x[2], z0, z1);
    s1 += z0 + z1;
    s2 += z0 * z0 + z1 * z1;
#pragma unroll
    for (int j = 0; j < ZT_MAX; ++j) c[j] += (fabs(z0) > sthr[j] ? 1u : 0u) + (fabs(z1) > sthr[j] ? 1u : 0u);
  }
#pragma unroll
  for (int j = 0; j < ZT_MAX; ++j) {
    unsigned long long v = c[j];
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&counts[j], v);
  }
  for (int d = 32; d >= 1; d >>= 1) {
    s1 += __shfl_xor(s1, d, 64);
    s2 += __shfl_xor(s2, d, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&mom[0], s1);
    atomicAdd(&mom[1], s2);
  }
}
}  // namespace

// Host copy of the device's zlog1p_neg (same source, same IEEE operation order): the CPU suite checks it against
// the C library's log1p, which numpy's tail draws call.
extern "C" int gp_zig_log1p_neg(const double* u, double* out, int64_t n) {
  if (n < 0 || (n && (!u || !out))) {
    gp_set_error("gp_zig_log1p_neg: bad arguments");
    return GP_E_INVALID;
  }
  for (int64_t i = 0; i < n; ++i) out[i] = zlog1p_neg(u[i]);
  return GP_OK;
}

extern "C" int gp_standard_normal_words(const uint64_t* words, int64_t nwords, double* out, int64_t n, int64_t* used,
                                        void* stream) {
  if (!words || !out || !used || nwords < 0 || n < 0) {
    gp_set_error("gp_standard_normal_words: bad argument");
    return GP_E_INVALID;
  }
  hipStream_t s = (hipStream_t)stream;
  DevBuf u;
  int e;
  if ((e = u.alloc(sizeof(int64_t)))) return e;
  hipLaunchKernelGGL(zig_words_kernel, dim3(1), dim3(64), 0, s, words, nwords, out, n, u.as<int64_t>());
  GP_HIP_CHECK(hipGetLastError());
  GP_HIP_CHECK(hipMemcpyAsync(used, u.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  GP_HIP_CHECK(hipStreamSynchronize(s));
  return GP_OK;
}

extern "C" int gp_normal_tail_counts(uint64_t key, int64_t n, const double* thr, int nthr, uint64_t* counts,
                                     double moments[2], void* stream) {
  if (n < 2 || !thr || !counts || !moments || nthr < 1 || nthr > ZT_MAX) {
    gp_set_error("gp_normal_tail_counts: bad argument (1 <= nthr <= %d, n >= 2)", ZT_MAX);
    return GP_E_INVALID;
  }
  hipStream_t s = (hipStream_t)stream;
  DevBuf dthr, dc, dm;
  int e;
  if ((e = dthr.alloc(sizeof(double) * ZT_MAX)) || (e = dc.alloc(sizeof(uint64_t) * ZT_MAX)) ||
      (e = dm.alloc(sizeof(double) * 2)))
    return e;
  GP_HIP_CHECK(hipMemcpy(dthr.p, thr, sizeof(double) * nthr, hipMemcpyHostToDevice));
  int dev = 0, cus = 256;
  GP_HIP_CHECK(hipGetDevice(&dev));
  GP_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  hipLaunchKernelGGL(zig_tail_kernel, dim3(cus * 8), dim3(256), 0, s, (uint32_t)key, (uint32_t)(key >> 32),
                     (uint64_t)n / 2, dthr.as<double>(), nthr, dc.as<unsigned long long>(), dm.as<double>());
  GP_HIP_CHECK(hipGetLastError());
  GP_HIP_CHECK(hipStreamSynchronize(s));
  std::vector<uint64_t> c(ZT_MAX);
  GP_HIP_CHECK(hipMemcpy(c.data(), dc.p, sizeof(uint64_t) * ZT_MAX, hipMemcpyDeviceToHost));
  GP_HIP_CHECK(hipMemcpy(moments, dm.p, sizeof(double) * 2, hipMemcpyDeviceToHost));
  for (int j = 0; j < nthr; ++j) counts[j] = c[j];
  return GP_OK;
}

std::unique_ptr<EnvBackend> make_crooms_backend(const gp_crooms_config* cfg, int64_t B, int device, int rng_mode,
                                                int* err) {
  if (B < 1 || B > (int64_t)1 << 30) {
    gp_set_error("crooms: num_envs %lld out of range", (long long)B);
    *err = GP_E_INVALID;
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    gp_set_error("crooms: hipSetDevice(%d) failed", device);
    *err = GP_E_HIP;
    return nullptr;
  }
  auto be = std::make_unique<CRoomsBackend>();
  be->B = B;
  be->device = device;
  be->rng_mode = rng_mode;
  int e = be->build(cfg);
  if (e) {
    *err = e;
    return nullptr;
  }
  if (rng_mode == GP_RNG_NUMPY) {  // the ziggurat wedge's exp(-x^2/2) from the host's libm build
    const int fma = gp_exp_host_variant() == 0 ? 0 : 1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_crooms_exp_fma), &fma, sizeof(fma)) != hipSuccess) {
      gp_set_error("crooms: hipMemcpyToSymbol(exp variant) failed");
      *err = GP_E_HIP;
      return nullptr;
    }
  }
  return be;
}
