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
// counter-based Philox4x32-10 keyed by the seed (Box-Muller normals, Lemire cell indices, 53-bit
// uniforms compared against the integer action-failure thresholds); GP_RNG_REPLAY takes the values
// the reference's stream produced (how parity is tested).
//
// Kernels: a persistent, grid-stride rollout kernel (tables staged in LDS once per block, 512-env
// tiles, K steps per tile, 2 envs per thread).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "gp_internal.h"

#pragma clang fp contract(off)

namespace {

constexpr int TPB = 256;
constexpr int EPT = 2;
constexpr int EPB = TPB * EPT;
constexpr int WAVES = TPB / 64;
constexpr uint32_t TAG_NOISE = 0x63726f6fu;  // 'croo'
constexpr uint32_t TAG_DRAW = 0x6d733121u;
constexpr double MAX_VELOCITY = 5.0;        // crooms.py:170

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
// Box-Muller on two 32-bit words: z0 = r cos(2 pi u2), z1 = r sin(2 pi u2), r = sqrt(-2 ln u1), u1 in (0,1].
// Hardware transcendentals (float32 accuracy, which is all the law needs): v_log_f32 = log2,
// v_sin/cos_f32 take revolutions, i.e. sin(2 pi u2) directly.
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, double& z0, double& z1) {
  const float u1 = ((float)(a >> 8) + 1.0f) * 5.9604644775390625e-08f;  // (k+1) 2^-24, in (0, 1]
  const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));  // sqrt(-2 ln u1)
  const float u2 = (float)(b >> 8) * 5.9604644775390625e-08f;           // k 2^-24, in [0, 1)
  z0 = (double)(r * __builtin_amdgcn_cosf(u2));
  z1 = (double)(r * __builtin_amdgcn_sinf(u2));
}

struct Draws {
  uint64_t k53;      // action-failure uniform
  uint32_t gi, ai;   // reset cell indices
};

// Gaussian noise of env-step (env, step): pair 0 = action noise N(0, action_std) (crooms.py:178,
// :194-195), pair 1 = wall noise N(0, 0.5) (:324). Replay: the values numpy returned.
template <bool REPLAY>
__device__ __forceinline__ void draw_normals(const CrDev& p, int env, uint64_t step, int pair, double scale,
                                             double& y, double& x, Philox4* blk = nullptr, bool* have = nullptr) {
  if constexpr (REPLAY) {
    const double* src = pair == 0 ? p.rp_noise : p.rp_wall;
    const double2 v = *reinterpret_cast<const double2*>(src + 2 * (size_t)env);
    y = v.x;
    x = v.y;
  } else {
    // one Philox block per env-step serves both pairs (the caller keeps it in blk / have)
    Philox4 r;
    if (have && *have) {
      r = *blk;
    } else {
      r = philox4x32_10((uint32_t)env, (uint32_t)step, (uint32_t)(step >> 32), TAG_NOISE, p.key0, p.key1);
      if (have) { *blk = r; *have = true; }
    }
    double z0, z1;
    box_muller(r.x[2 * pair], r.x[2 * pair + 1], z0, z1);
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
    const Philox4 r = philox4x32_10((uint32_t)env, (uint32_t)step, (uint32_t)(step >> 32), TAG_DRAW, p.key0, p.key1);
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
  return p.inv_cell != 0.0 ? v * p.inv_cell : v / p.cell;
}

__device__ __forceinline__ int cell_of(const CrDev& p, double y, double x) {
  // coord_to_grid (utils.py:15-20): floor(coord / cell_size)
  const int cy = (int)floor(per_cell(p, y)), cx = (int)floor(per_cell(p, x));
  if (cy < 0 || cx < 0 || cy >= p.H || cx >= p.W) return -1;
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

// reset of one env: goal then agent (crooms.py:217-244, 268-274)
__device__ __forceinline__ void reset_env(const CrDev& p, const uint8_t* lds, const Draws& d, double& ay, double& ax,
                                          double& vy, double& vx, uint32_t& g) {
  if (!p.goal_fixed) {
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
  uint8_t term, trunc;
};

// One env-step of CRoomsEnv.step (crooms.py:276-331).
template <bool REPLAY>
__device__ __forceinline__ StepOut crooms_env_step(const CrDev& p, const uint8_t* lds, int env, bool live,
                                                   uint64_t step, double a0, double a1, int ad, double& ay,
                                                   double& ax, double& vy, double& vx, uint32_t& g, int32_t& el,
                                                   float& rsum, uint32_t& eps, uint32_t& lens) {
  StepOut o;
  el += 1;
  Draws d;
  d.k53 = 0;
  d.gi = d.ai = 0;
  // _sample_action (crooms.py:175-198) * action_power (:288)
  double my, mx;
  Philox4 nblk;
  bool nhave = false;
  if (p.action_kind == 0) {
    double ny = 0.0, nx = 0.0;
    if (live) draw_normals<REPLAY>(p, env, step, 0, p.action_std, ny, nx, &nblk, &nhave);
    my = a0 + ny;
    mx = a1 + nx;
  } else {
    if (live) draw_ints<REPLAY>(p, env, step, d);
    int a = ad;
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
      double ny = 0.0, nx = 0.0;
      if (live) draw_normals<REPLAY>(p, env, step, 0, p.action_std, ny, nx, &nblk, &nhave);
      my = my + ny;
      mx = mx + nx;
    }
  }
  my = my * p.action_power;
  mx = mx * p.action_power;
  // _apply_action (crooms.py:300-331)
  double py, px;
  if (p.use_velocity) {
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
  const int pc = cell_of(p, py, px);
  const bool oob = pc < 0 || tab<uint8_t>(lds, p.off_wall)[pc] != 0;
  if (!oob) {
    ay = py;
    ax = px;
  } else {
    // stay in the current square: c = grid_to_coord(coord_to_grid(agent)), agent = clip(c + n, c - cs/2, c + cs/2 - 1e-8)
    const double cy = floor(per_cell(p, ay)) * p.cell + p.half_cell;
    const double cx = floor(per_cell(p, ax)) * p.cell + p.half_cell;
    double wy = 0.0, wx = 0.0;
    if (live) draw_normals<REPLAY>(p, env, step, 1, 0.5, wy, wx, &nblk, &nhave);
    ay = fmin(fmax(cy + wy, cy - p.half_cell), (cy + p.half_cell) - 1e-8);
    ax = fmin(fmax(cx + wx, cx - p.half_cell), (cx + p.half_cell) - 1e-8);
    vy = 0.0;
    vx = 0.0;
  }
  // reward / termination (crooms.py:289-297)
  const double gyc = (double)(int16_t)(g & 0xFFFF) + 0.5, gxc = (double)(int16_t)(g >> 16) + 0.5;
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
    if (p.action_kind == 0) draw_ints<REPLAY>(p, env, step, d);
    reset_env(p, lds, d, ay, ax, vy, vx, g);
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
template <int OK, bool REPLAY>
__global__ __launch_bounds__(TPB) void crooms_rollout(CrDev p, int K, uint64_t step0, const void* __restrict__ act,
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
      vy[i] = (live && p.use_velocity) ? p.vy[env] : 0.0;
      vx[i] = (live && p.use_velocity) ? p.vx[env] : 0.0;
      g[i] = live ? (p.goal_fixed ? ((uint32_t)(p.goal_y & 0xFFFF) | ((uint32_t)(p.goal_x & 0xFFFF) << 16))
                                  : p.goal[env])
                  : 0u;
      el[i] = live ? p.el[env] : 0;
    }
    for (int k = 0; k < K; ++k) {
      const size_t off = (size_t)k * p.B;
      double a0[EPT], a1[EPT];
      int ad[EPT];
      const bool full = env0 + EPT - 1 < p.B && (off & 1) == 0;  // pair-aligned rew / flag stores
#pragma unroll
      for (int i = 0; i < EPT; ++i) { a0[i] = a1[i] = 0.0; ad[i] = 0; }
      if (p.action_kind == 0) {
        if (p.action_f64) {
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
        StepOut o = crooms_env_step<REPLAY>(p, lds, env, live, step0 + (uint64_t)k, a0[i], a1[i], ad[i], ay[i], ax[i],
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
      const size_t ob = (size_t)k * p.B * (size_t)p.obs_width * (OK == GP_OBS_F32 ? (p.obs_f64 ? 8 : 4)
                                                                   : (OK == GP_OBS_HANSEN || OK == GP_OBS_TABLE ? 4 : 1));
      if (OK == GP_OBS_F32 && !p.obs_f64 && p.obs_width == 2 && full) {
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
      if (p.use_velocity) { p.vy[env] = vy[i]; p.vx[env] = vx[i]; }
      if (!p.goal_fixed) p.goal[env] = g[i];
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
    return GP_OK;
  }
  int set_rng_state(const RngHost&) override {
    gp_set_error("crooms: the PCG64 stream is not used on the device (philox / replay modes)");
    return GP_E_UNSUPPORTED;
  }
  int get_rng_state(RngHost*) override {
    gp_set_error("crooms: the PCG64 stream is not used on the device (philox / replay modes)");
    return GP_E_UNSUPPORTED;
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
    const CrDev dd = dev_for_launch();
    const uint64_t st = philox_step;
    int e = dispatch_obs(d.obs_kind, [&](auto okc) -> int {
      constexpr int OK = decltype(okc)::value;
      timer.begin(s);
      if (rep)
        hipLaunchKernelGGL((crooms_rollout<OK, true>), dim3(grid), dim3(TPB), d.tab_bytes, s, dd, K, st, act, obs,
                           rew, term, trunc);
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
    return GP_OK;
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
  occ = std::max(1, std::min(occ, 8));
  grid = std::max(1, std::min(d.ntiles, prop.multiProcessorCount * occ));
  if ((e = b_slot.alloc(sizeof(CrSlot) * grid))) return e;
  d.mslot = b_slot.as<CrSlot>();
  return GP_OK;
}

}  // namespace

std::unique_ptr<EnvBackend> make_crooms_backend(const gp_crooms_config* cfg, int64_t B, int device, int rng_mode,
                                                int* err) {
  if (rng_mode == GP_RNG_NUMPY) {
    gp_set_error("crooms: rng_mode numpy is not available on the device (numpy's ziggurat normals consume a "
                 "data-dependent number of words from one stream); use philox (same laws) or replay");
    *err = GP_E_UNSUPPORTED;
    return nullptr;
  }
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
  return be;
}
