// anttag.hip — grid Ant-Tag (GP_KIND_ANTTAG): a build-defined grid restatement of the task rules of
// gym_po/envs/ant_tag.py:88-157 (the reference env is a MuJoCo ant; only its tag task is restated).
//
// Spec (DESIGN.md §"ant_tag grid", oracle/anttag.py restates it in numpy):
//   arena   size x size cells (default 10: the 10 m interior of assets/ant_tag_small.xml:72-83, 1 m cells;
//           the target cage +-4.5 m covers every cell centre)
//   actions 0 N, 1 E, 2 S, 3 W, 4 stay; a move off the arena leaves the ant in place
//   target  after the ant moves (ant_tag.py:140-142): with (dy, dx) = ant - target and
//           choose = uniform{0,1,2,3} (:107-118): 0 away (-dy, -dx); 1 (-dx, dy); 2 (dx, -dy); 3 stay.
//           The direction v is rounded to one grid step: the dominant axis of v, or the diagonal when
//           |vy| == |vx| (none when v = 0). A step leaving the cage is not taken (:120-121).
//   tag     d^2 <= tag_radius2 (1.5 m -> 2): reward tag_reward, terminated (:147-150)
//   obs     int32 [ant y, ant x, target y, target x], the target replaced by (-1, -1) unless
//           d^2 < visible_radius2 (3 m -> 9) (:77-86, :153)
//   reset   ant uniform over the cells; target uniform over the cells with d^2 > min_start_dist2
//           (5 m -> 25): the law of the rejection loop of reset_model (:88-103)
//   trunc   elapsed >= time_limit (gymnasium TimeLimit, max_episode_steps=500, envs/__init__.py:15-19)
// State per env: ONE packed uint32 (ant cell | target cell << 8 | elapsed << 16) in registers across a
// rollout. RNG: philox (counter = env, step) or replay (caller-decided choose / reset indices).
#include <algorithm>
#include <cstring>
#include <vector>

#include "gp_internal.h"

namespace {

constexpr int TPB = 256;
constexpr int EPT = 4;
constexpr int EPB = TPB * EPT;
constexpr int WAVES = TPB / 64;
constexpr int MAX_SIZE = 16;  // cells fit 8 bits of the packed state
constexpr int NACT = 5;
constexpr uint32_t TAG = 0x616e7431u;  // 'ant1'

struct alignas(32) AtSlot {
  double return_sum;
  unsigned long long episodes, length_sum, env_steps;
};

struct AtDev {
  int32_t B, ntiles, N, ncells;
  uint32_t divm;           // ceil(2^16 / N): cell / N == (cell * divm) >> 16 for cells < 256
  int32_t tag_r2, vis_r2, time_limit;
  float r_tag, r_step;
  uint32_t key0, key1;
  const uint8_t* tabs;     // [ncells] valid-target counts (u8, 16-B padded) | [ncells][ncells] target lists
  int32_t off_cnt, off_list, tab_bytes;
  uint32_t* st;            // [B] ant | target << 8 | elapsed << 16
  AtSlot* mslot;
  uint32_t* derr;            // device error word (GP_DERR_*)
  const int32_t* rp_choose;  // replay: target move choice [B]
  const int32_t* rp_ant;     // replay: reset ant cell index [B]
  const int32_t* rp_tgt;     // replay: reset target index into the ant cell's valid list [B]
};

__device__ __forceinline__ void stage_tables(const AtDev& p, uint8_t* lds) {
  const uint4* src = (const uint4*)p.tabs;
  uint4* dst = (uint4*)lds;
  for (int i = threadIdx.x; i < p.tab_bytes / 16; i += TPB) dst[i] = src[i];
}

__device__ __forceinline__ int isgn(int v) { return (v > 0) - (v < 0); }
// cell / N without an integer divide (exact for cells < 256, N <= 16)
__device__ __forceinline__ int cdiv(const AtDev& p, int c) { return (int)(((uint32_t)c * p.divm) >> 16); }

// The reset draws of env `env` at `step`: words 1, 2 of its Philox block (word 0 is the target-move
// choice of the same step; `r` passes the block when the caller already has it).
template <bool REPLAY>
__device__ __forceinline__ uint32_t draw_reset(const AtDev& p, const uint8_t* lds, int env, uint64_t step,
                                               const Philox4* have = nullptr) {
  uint32_t ant, k;
  if constexpr (REPLAY) {
    ant = (uint32_t)min(max(p.rp_ant[env], 0), p.ncells - 1);
    k = (uint32_t)max(p.rp_tgt[env], 0);
  } else {
    const Philox4 r = have ? *have
                           : philox4x32_10((uint32_t)env, (uint32_t)step, (uint32_t)(step >> 32), TAG, p.key0, p.key1);
    ant = lemire_value(r.x[1], (uint32_t)p.ncells);
    k = lemire_value(r.x[2], (uint32_t)lds[p.off_cnt + ant]);
  }
  k = min(k, (uint32_t)lds[p.off_cnt + ant] - 1u);
  const uint32_t tgt = lds[p.off_list + ant * p.ncells + k];
  return ant | (tgt << 8);
}

struct StepOut {
  float rew;
  uint8_t term, trunc;
};

template <bool REPLAY>
__device__ __forceinline__ StepOut at_env_step(const AtDev& p, const uint8_t* lds, uint32_t& u, int a, int env,
                                               bool live, uint64_t step, float& rsum, uint32_t& eps, uint32_t& lens) {
  const int N = p.N;
  int ant = (int)(u & 0xFFu), tgt = (int)((u >> 8) & 0xFFu);
  uint32_t el = (u >> 16) + 1u;
  int ay = cdiv(p, ant), ax = ant - ay * N, ty = cdiv(p, tgt), tx = tgt - ty * N;
  // ant move (an action outside [-5, 5) is flagged as the reference's discrete envs would raise, then clamped)
  if (live && action_out_of_range(a, NACT)) flag_bad_action(p.derr);
  if (a < 0) a += NACT;
  a = min(max(a, 0), NACT - 1);
  const int DY[NACT] = {-1, 0, 1, 0, 0}, DX[NACT] = {0, 1, 0, -1, 0};
  const int ny = ay + DY[a], nx = ax + DX[a];
  if (ny >= 0 && ny < N && nx >= 0 && nx < N) { ay = ny; ax = nx; }
  // target move (choose uniform over 4)
  uint32_t choose = 3;
  Philox4 r{};
  if (live) {
    if constexpr (REPLAY) {
      choose = (uint32_t)p.rp_choose[env] & 3u;
    } else {
      r = philox4x32_10((uint32_t)env, (uint32_t)step, (uint32_t)(step >> 32), TAG, p.key0, p.key1);
      choose = r.x[0] >> 30;
    }
  }
  const int dy = ay - ty, dx = ax - tx;
  int vy = 0, vx = 0;
  if (choose == 0) { vy = -dy; vx = -dx; }
  else if (choose == 1) { vy = -dx; vx = dy; }
  else if (choose == 2) { vy = dx; vx = -dy; }
  const int avy = abs(vy), avx = abs(vx);
  const int sy = avy >= avx ? isgn(vy) : 0, sx = avx >= avy ? isgn(vx) : 0;
  const int mty = ty + sy, mtx = tx + sx;
  if (mty >= 0 && mty < N && mtx >= 0 && mtx < N) { ty = mty; tx = mtx; }
  const int ey = ay - ty, ex = ax - tx, d2 = ey * ey + ex * ex;
  StepOut o;
  o.term = d2 <= p.tag_r2 ? 1 : 0;
  o.rew = o.term ? p.r_tag : p.r_step;
  o.trunc = el >= (uint32_t)p.time_limit ? 1 : 0;
  u = (uint32_t)(ay * N + ax) | ((uint32_t)(ty * N + tx) << 8) | (min(el, 0xFFFFu) << 16);
  if (!live) return o;
  rsum += o.rew;
  if (o.term | o.trunc) {
    eps += 1u;
    lens += el;
    u = draw_reset<REPLAY>(p, lds, env, step, &r);
  }
  return o;
}

__device__ __forceinline__ int4 at_obs(const AtDev& p, uint32_t u) {
  const int N = p.N, ant = (int)(u & 0xFFu), tgt = (int)((u >> 8) & 0xFFu);
  const int ay = cdiv(p, ant), ax = ant - ay * N, ty = cdiv(p, tgt), tx = tgt - ty * N;
  const int dy = ay - ty, dx = ax - tx;
  const bool vis = dy * dy + dx * dx < p.vis_r2;
  return make_int4(ay, ax, vis ? ty : -1, vis ? tx : -1);
}

__device__ void at_metrics(const AtDev& p, float rsum, uint32_t eps, uint32_t lens, uint32_t nst) {
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
    AtSlot& m = p.mslot[blockIdx.x];
    m.return_sum += (double)r;
    m.episodes += e;
    m.length_sum += l;
    m.env_steps += n;
  }
}

__device__ __forceinline__ bool quad_ok(const void* base, int env0, int B, int esz) {
  return env0 + 3 < B && ((((uintptr_t)base) + (size_t)env0 * esz) & (size_t)(4 * esz - 1)) == 0;
}

template <bool REPLAY>
#ifndef GP_AT_WAVES
#define GP_AT_WAVES 1  // launch bound: minimum waves per SIMD (register budget of the rollout)
#endif
__global__ __launch_bounds__(TPB, GP_AT_WAVES) void anttag_rollout(AtDev p, int K, uint64_t step0, const int32_t* __restrict__ act,
                                                      int4* __restrict__ obs, float* __restrict__ rew,
                                                      uint8_t* __restrict__ term, uint8_t* __restrict__ trunc) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ int4 s_obs[TPB * EPT];  // per-wave obs transpose: lane-contiguous 16-B obs stores
  stage_tables(p, lds);
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int4* wv = s_obs + wid * 64 * EPT;
  float rsum = 0.f;
  uint32_t eps = 0, lens = 0, nst = 0;
  for (int tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
    const int env0 = tile * EPB + threadIdx.x * EPT;
    uint32_t u[EPT];
    const bool sq = quad_ok(p.st, env0, p.B, 4);
    if (sq) {
      const uint4 q = *reinterpret_cast<const uint4*>(p.st + env0);
      u[0] = q.x; u[1] = q.y; u[2] = q.z; u[3] = q.w;
    } else {
#pragma unroll
      for (int i = 0; i < EPT; ++i) u[i] = env0 + i < p.B ? p.st[env0 + i] : 0u;
    }
    auto load_act = [&](int k, int (&a)[EPT]) {
      const size_t off = (size_t)k * p.B;
      if (quad_ok(act + off, env0, p.B, 4)) {
        const int4 q = *reinterpret_cast<const int4*>(act + off + env0);
        a[0] = q.x; a[1] = q.y; a[2] = q.z; a[3] = q.w;
      } else {
#pragma unroll
        for (int i = 0; i < EPT; ++i) a[i] = env0 + i < p.B ? act[off + env0 + i] : 0;
      }
    };
    int a_nxt[EPT];
    if (K > 0) load_act(0, a_nxt);
    for (int k = 0; k < K; ++k) {
      const size_t off = (size_t)k * p.B;
      int a[EPT];
#pragma unroll
      for (int i = 0; i < EPT; ++i) a[i] = a_nxt[i];
      if (k + 1 < K) load_act(k + 1, a_nxt);  // one step ahead
      float r[EPT];
      uint8_t tm[EPT], tr[EPT];
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        const bool live = env0 + i < p.B;
        StepOut o = at_env_step<REPLAY>(p, lds, u[i], a[i], env0 + i, live, step0 + (uint64_t)k, rsum, eps, lens);
        r[i] = o.rew;
        tm[i] = o.term;
        tr[i] = o.trunc;
        nst += live ? 1u : 0u;
      }
      if (quad_ok(rew + off, env0, p.B, 4) && quad_ok(term + off, env0, p.B, 1) && quad_ok(trunc + off, env0, p.B, 1)) {
        *reinterpret_cast<float4*>(rew + off + env0) = make_float4(r[0], r[1], r[2], r[3]);
        *reinterpret_cast<uint32_t*>(term + off + env0) =
            (uint32_t)tm[0] | ((uint32_t)tm[1] << 8) | ((uint32_t)tm[2] << 16) | ((uint32_t)tm[3] << 24);
        *reinterpret_cast<uint32_t*>(trunc + off + env0) =
            (uint32_t)tr[0] | ((uint32_t)tr[1] << 8) | ((uint32_t)tr[2] << 16) | ((uint32_t)tr[3] << 24);
      } else {
#pragma unroll
        for (int i = 0; i < EPT; ++i)
          if (env0 + i < p.B) { rew[off + env0 + i] = r[i]; term[off + env0 + i] = tm[i]; trunc[off + env0 + i] = tr[i]; }
      }
      // obs: through LDS so that each store instruction writes 64 consecutive envs (1 KB)
#pragma unroll
      for (int i = 0; i < EPT; ++i) wv[lane * EPT + i] = at_obs(p, u[i]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
      const int wenv0 = tile * EPB + wid * 64 * EPT;
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        const int e = wenv0 + j * 64 + lane;
        if (e < p.B) obs[off + e] = wv[j * 64 + lane];
      }
    }
    if (sq) {
      *reinterpret_cast<uint4*>(p.st + env0) = make_uint4(u[0], u[1], u[2], u[3]);
    } else {
#pragma unroll
      for (int i = 0; i < EPT; ++i)
        if (env0 + i < p.B) p.st[env0 + i] = u[i];
    }
  }
  at_metrics(p, rsum, eps, lens, nst);
}

template <bool REPLAY>
__global__ __launch_bounds__(TPB) void anttag_reset(AtDev p, uint64_t step, int4* __restrict__ obs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  stage_tables(p, lds);
  __syncthreads();
  for (int env = blockIdx.x * TPB + threadIdx.x; env < p.B; env += gridDim.x * TPB) {
    const uint32_t u = draw_reset<REPLAY>(p, lds, env, step);
    p.st[env] = u;
    obs[env] = at_obs(p, u);
  }
}

__global__ void anttag_get_state(AtDev p, int32_t* ant, int32_t* tgt, int32_t* el) {
  const int env = blockIdx.x * TPB + threadIdx.x;
  if (env >= p.B) return;
  const uint32_t u = p.st[env];
  if (ant) ant[env] = (int32_t)(u & 0xFFu);
  if (tgt) tgt[env] = (int32_t)((u >> 8) & 0xFFu);
  if (el) el[env] = (int32_t)(u >> 16);
}
__global__ void anttag_set_state(AtDev p, const int32_t* ant, const int32_t* tgt, const int32_t* el) {
  const int env = blockIdx.x * TPB + threadIdx.x;
  if (env >= p.B) return;
  uint32_t u = p.st[env];
  if (ant) u = (u & ~0xFFu) | (uint32_t)min(max(ant[env], 0), p.ncells - 1);
  if (tgt) u = (u & ~0xFF00u) | ((uint32_t)min(max(tgt[env], 0), p.ncells - 1) << 8);
  if (el) u = (u & 0xFFFFu) | ((uint32_t)min(max(el[env], 0), 65535) << 16);
  p.st[env] = u;
}

// ------------------------------------------------------------------ host backend ----
struct AntTagBackend : EnvBackend {
  AtDev d{};
  int grid = 1;
  uint64_t philox_step = 0;
  DevBuf b_tabs, b_st, b_slot;
  DevErr derr;
  const int32_t* rp_choose = nullptr;
  const int32_t* rp_ant = nullptr;
  const int32_t* rp_tgt = nullptr;

  int build(const gp_anttag_config* cfg);
  int seed(const RngHost& r, const uint32_t key[2]) override {
    rng = r;
    d.key0 = key[0];
    d.key1 = key[1];
    philox_step = 0;
    return derr.clear();
  }
  int check() override { return derr.check("anttag"); }
  int set_rng_state(const RngHost&) override {
    gp_set_error("anttag: no numpy stream (build-defined env; philox / replay modes)");
    return GP_E_UNSUPPORTED;
  }
  int get_rng_state(RngHost*) override {
    gp_set_error("anttag: no numpy stream (build-defined env; philox / replay modes)");
    return GP_E_UNSUPPORTED;
  }
  AtDev dev_for_launch() const {
    AtDev dd = d;
    dd.rp_choose = rp_choose;
    dd.rp_ant = rp_ant;
    dd.rp_tgt = rp_tgt;
    return dd;
  }
  int reset(void* obs, hipStream_t s) override {
    GP_HIP_CHECK(hipMemsetAsync(d.mslot, 0, sizeof(AtSlot) * grid, s));
    const AtDev dd = dev_for_launch();
    if (rng_mode == GP_RNG_REPLAY) {
      if (!rp_ant || !rp_tgt) {
        gp_set_error("anttag replay reset needs ant / target indices (gp_set_replay i0/i1)");
        return GP_E_STATE;
      }
      hipLaunchKernelGGL(anttag_reset<true>, dim3(grid), dim3(TPB), d.tab_bytes, s, dd, (uint64_t)0, (int4*)obs);
    } else {
      hipLaunchKernelGGL(anttag_reset<false>, dim3(grid), dim3(TPB), d.tab_bytes, s, dd, philox_step, (int4*)obs);
      ++philox_step;
    }
    GP_HIP_CHECK(hipGetLastError());
    has_reset = true;
    return GP_OK;
  }
  int rollout(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) override {
    if (!has_reset) {
      gp_set_error("step() before reset()");
      return GP_E_STATE;
    }
    if (((uintptr_t)obs & 15) != 0) {
      gp_set_error("anttag: obs buffer must be 16-B aligned");
      return GP_E_INVALID;
    }
    const AtDev dd = dev_for_launch();
    if (rng_mode == GP_RNG_REPLAY) {
      if (!rp_choose || !rp_ant || !rp_tgt) {
        gp_set_error("anttag replay step needs choose (u), ant (i0) and target (i1) draws");
        return GP_E_STATE;
      }
      if (K > 1) return EnvBackend::rollout(K, act, obs, rew, term, trunc, s);
      timer.begin(s);
      hipLaunchKernelGGL(anttag_rollout<true>, dim3(grid), dim3(TPB), d.tab_bytes, s, dd, K, (uint64_t)0,
                         (const int32_t*)act, (int4*)obs, rew, term, trunc);
      timer.end(s);
    } else {
      timer.begin(s);
      hipLaunchKernelGGL(anttag_rollout<false>, dim3(grid), dim3(TPB), d.tab_bytes, s, dd, K, philox_step,
                         (const int32_t*)act, (int4*)obs, rew, term, trunc);
      timer.end(s);
      philox_step += (uint64_t)K;
    }
    GP_HIP_CHECK(hipGetLastError());
    return GP_OK;
  }
  int step(const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) override {
    return rollout(1, act, obs, rew, term, trunc, s);
  }
  int get_state(void* a, void* b, void* c, void*, hipStream_t s) override {
    hipLaunchKernelGGL(anttag_get_state, dim3((unsigned)((B + TPB - 1) / TPB)), dim3(TPB), 0, s, d, (int32_t*)a,
                       (int32_t*)b, (int32_t*)c);
    GP_HIP_CHECK(hipGetLastError());
    return GP_OK;
  }
  int set_state(const void* a, const void* b, const void* c, const void*, hipStream_t s) override {
    hipLaunchKernelGGL(anttag_set_state, dim3((unsigned)((B + TPB - 1) / TPB)), dim3(TPB), 0, s, d,
                       (const int32_t*)a, (const int32_t*)b, (const int32_t*)c);
    GP_HIP_CHECK(hipGetLastError());
    has_reset = true;
    return GP_OK;
  }
  // replay: u -> choose (int32 [B]), i0 -> reset ant cell, i1 -> reset target index in the ant's list
  int set_replay(const void* u, const void* i0, const void* i1, const void*, const void*) override {
    if (rng_mode != GP_RNG_REPLAY) {
      gp_set_error("gp_set_replay requires GP_RNG_REPLAY");
      return GP_E_STATE;
    }
    rp_choose = (const int32_t*)u;
    rp_ant = (const int32_t*)i0;
    rp_tgt = (const int32_t*)i1;
    return GP_OK;
  }
  int metrics(double out[4]) override {
    GP_HIP_CHECK(hipDeviceSynchronize());
    std::vector<AtSlot> m(grid);
    GP_HIP_CHECK(hipMemcpy(m.data(), d.mslot, sizeof(AtSlot) * grid, hipMemcpyDeviceToHost));
    out[0] = out[1] = out[2] = out[3] = 0;
    for (const AtSlot& x : m) {
      out[0] += (double)x.episodes;
      out[1] += x.return_sum;
      out[2] += (double)x.length_sum;
      out[3] += (double)x.env_steps;
    }
    return check();
  }
};

int AntTagBackend::build(const gp_anttag_config* cfg) {
  const int N = cfg->size, nc = N * N;
  if (N < 2 || N > MAX_SIZE) {
    gp_set_error("anttag: size %d outside [2, %d]", N, MAX_SIZE);
    return GP_E_INVALID;
  }
  if (cfg->time_limit < 1 || cfg->time_limit > 65535) {
    gp_set_error("anttag: time_limit %d outside [1, 65535]", cfg->time_limit);
    return GP_E_INVALID;
  }
  std::vector<uint8_t> cnt(nc, 0), list((size_t)nc * nc, 0);
  for (int a = 0; a < nc; ++a) {
    int k = 0;
    for (int t = 0; t < nc; ++t) {
      const int dy = a / N - t / N, dx = a % N - t % N;
      if (dy * dy + dx * dx > cfg->min_start_dist2) list[(size_t)a * nc + k++] = (uint8_t)t;
    }
    if (k == 0) {
      gp_set_error("anttag: no target cell farther than sqrt(%d) from cell %d", cfg->min_start_dist2, a);
      return GP_E_INVALID;
    }
    cnt[a] = (uint8_t)std::min(k, 255);
    if (k > 255) {
      gp_set_error("anttag: too many start cells");
      return GP_E_INVALID;
    }
  }
  std::vector<uint8_t> blob;
  auto put = [&](const std::vector<uint8_t>& v) {
    const size_t off = (blob.size() + 15) & ~(size_t)15;
    blob.resize(off + v.size());
    memcpy(blob.data() + off, v.data(), v.size());
    return (int32_t)off;
  };
  d.off_cnt = put(cnt);
  d.off_list = put(list);
  blob.resize((blob.size() + 15) & ~(size_t)15);
  d.tab_bytes = (int32_t)blob.size();
  int e;
  if ((e = b_tabs.upload(blob))) return e;
  d.tabs = b_tabs.as<uint8_t>();
  d.B = (int32_t)B;
  d.ntiles = (int32_t)((B + EPB - 1) / EPB);
  d.N = N;
  d.divm = (65536u + (uint32_t)N - 1u) / (uint32_t)N;
  d.ncells = nc;
  d.tag_r2 = cfg->tag_radius2;
  d.vis_r2 = cfg->visible_radius2;
  d.time_limit = cfg->time_limit;
  d.r_tag = cfg->tag_reward;
  d.r_step = cfg->step_reward;
  obs_dtype = GP_DTYPE_I32;
  obs_width = 4;
  if ((e = b_st.alloc((size_t)B * 4 + 16))) return e;
  d.st = b_st.as<uint32_t>();
  hipDeviceProp_t prop;
  GP_HIP_CHECK(hipGetDeviceProperties(&prop, device));
  int occ = 0;
  GP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, anttag_rollout<false>, TPB, d.tab_bytes));
  grid = persistent_grid(d.ntiles, prop.multiProcessorCount, occ);
  persist_grid = grid;
  persist_occ = occ;
  if ((e = b_slot.alloc(sizeof(AtSlot) * grid))) return e;
  d.mslot = b_slot.as<AtSlot>();
  if ((e = derr.alloc())) return e;
  d.derr = derr.ptr();
  return GP_OK;
}

}  // namespace

std::unique_ptr<EnvBackend> make_anttag_backend(const gp_anttag_config* cfg, int64_t B, int device, int rng_mode,
                                                int* err) {
  if (rng_mode == GP_RNG_NUMPY) {
    gp_set_error("anttag: rng_mode numpy does not exist for this build-defined env; use philox or replay");
    *err = GP_E_UNSUPPORTED;
    return nullptr;
  }
  if (B < 1 || B > (int64_t)1 << 30) {
    gp_set_error("anttag: num_envs %lld out of range", (long long)B);
    *err = GP_E_INVALID;
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    gp_set_error("anttag: hipSetDevice(%d) failed", device);
    *err = GP_E_HIP;
    return nullptr;
  }
  auto be = std::make_unique<AntTagBackend>();
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
