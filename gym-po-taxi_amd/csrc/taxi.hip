// taxi.hip — the (PO-)Taxi backend (GP_KIND_TAXI): TaxiVecEnv.step / _reset_mask /
// _reset_passenger_and_destination / _obs (gym_po/envs/extended_taxi.py:244-372) for B envs.
//
// The whole Taxi transition is a function of (state, action): no draw is made on a step unless the
// env completes a task or resets. So the host lowers the map once into
//   trans[s*6 + a] = s' | goal << 12 | bad << 13    (move, wall/pseudo-wall check, pickup/dropoff;
//                                                    column 5 = action -1, a no-op)
//   obs_of[s]      = s  or  (hansen[r,c]*(L+1) + p)*L + d
//   cdf[k]         = the exact start-state law of  multinomial(ns, uniform over valid).argmax()
//                    (dist.hip) as 64-bit thresholds over the valid states, ascending
// and the device step is: one LDS lookup, a compare or two, the stores. State per env is ONE packed
// uint32 (s | n_dropoffs << 12 | elapsed << 16) kept in registers across the K steps of a rollout.
//
// RNG: the reference's resets draw multinomial(500, p, b) = ~300 sequential binomial inversions per
// resetting env from ONE numpy stream, with a data-dependent word count, so a parallel exact stream
// is out of reach. Two modes:
//   GP_RNG_PHILOX  Philox4x32-10 (env, step): reset state = CDF search of one 64-bit uniform (the
//                  exact law, not an approximation of it); passenger/destination = Lemire draws with
//                  the reference's "resample d while d == p" law (p uniform, d uniform over the rest).
//   GP_RNG_REPLAY  caller-supplied per-env reset states and p*L+d pairs: bit-exact replay of the
//                  reference stream, which is how parity with the reference is checked.
//
// Kernels: one persistent, grid-stride rollout kernel (tables staged in LDS once per block, 1024-env
// tiles, K steps per tile with the state in registers) for both scalar and one-hot observations; the
// one-hot rows (uint8 [B, n_obs], 320 B/env for Hansen) are written as a wave-contiguous stream of
// 16-B chunks so every store instruction covers 1 KB of consecutive bytes.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "gp_internal.h"
#include "gp_libm.h"

namespace {

constexpr int TPB = 256;
constexpr int EPT = 4;
constexpr int EPB = TPB * EPT;  // envs per tile
constexpr int WAVES = TPB / 64;
constexpr int NACT = 5;         // N, S, W, E, Pickup/Dropoff (extended_taxi.py:154)
constexpr int TCOL = NACT + 1;  // transition-table columns: the 5 actions + the action -1 no-op
constexpr int MAX_NS = 4096;    // s fits 12 bits of the packed state
constexpr uint32_t PHILOX_TAG = 0x74617869u;  // 'taxi'

struct alignas(32) TaxiSlot {
  double return_sum;
  unsigned long long episodes, length_sum, env_steps;
};

struct TaxiDev {
  int32_t B, ntiles;
  int32_t ns, nlocs, lpl;          // lpl = L*(L+1): states per taxi cell
  int32_t n_valid, num_passengers, time_limit;
  int32_t n_obs;                   // observation space size (one-hot width)
  float r_goal, r_bad, r_any;
  uint32_t key0, key1;
  const uint8_t* tabs;             // packed tables (global), staged into LDS
  int32_t off_trans, off_obs, off_cdf, off_valid, tab_bytes;
  uint32_t* st;                    // [B] s | nd << 12 | elapsed << 16
  TaxiSlot* mslot;                 // [grid]
  uint32_t* derr;                  // device error word (GP_DERR_*)
  const int32_t* rp_state;         // replay: reset state per env (GP_RNG_REPLAY)
  const int32_t* rp_pd;            // replay: p*L + d per env
};

__device__ __forceinline__ const uint16_t* l_trans(const uint8_t* l, const TaxiDev& p) {
  return (const uint16_t*)(l + p.off_trans);
}
__device__ __forceinline__ const uint16_t* l_obs(const uint8_t* l, const TaxiDev& p) {
  return (const uint16_t*)(l + p.off_obs);
}
__device__ __forceinline__ const uint64_t* l_cdf(const uint8_t* l, const TaxiDev& p) {
  return (const uint64_t*)(l + p.off_cdf);
}
__device__ __forceinline__ const uint16_t* l_valid(const uint8_t* l, const TaxiDev& p) {
  return (const uint16_t*)(l + p.off_valid);
}

// Cooperative copy of the packed tables into LDS (16-B granules; tab_bytes is a multiple of 16).
__device__ __forceinline__ void stage_tables(const TaxiDev& p, uint8_t* lds) {
  const uint4* src = (const uint4*)p.tabs;
  uint4* dst = (uint4*)lds;
  for (int i = threadIdx.x; i < p.tab_bytes / 16; i += TPB) dst[i] = src[i];
}

// ---- the start-state law: smallest k with w < cdf[k] (cdf[n_valid-1] = 2^64-1, saturating) ----
__device__ __forceinline__ uint32_t sample_reset_state(const TaxiDev& p, const uint8_t* lds, uint64_t w) {
  const uint64_t* cdf = l_cdf(lds, p);
  int lo = 0, hi = p.n_valid - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (w < cdf[mid]) hi = mid; else lo = mid + 1;
  }
  return l_valid(lds, p)[lo];
}

template <bool REPLAY>
__device__ __forceinline__ uint32_t draw_reset(const TaxiDev& p, const uint8_t* lds, int env, uint64_t step) {
  if constexpr (REPLAY) {
    return (uint32_t)min(max(p.rp_state[env], 0), p.ns - 1);
  } else {
    const Philox4 r = philox4x32_10((uint32_t)env, (uint32_t)step, (uint32_t)(step >> 32), PHILOX_TAG, p.key0, p.key1);
    return sample_reset_state(p, lds, ((uint64_t)r.x[0] << 32) | r.x[1]);
  }
}

// extended_taxi.py:354-364: p = integers(L); d = integers(L), resampled while d == p. Its law is
// p uniform and d uniform over the other L-1 locations.
template <bool REPLAY>
__device__ __forceinline__ uint32_t draw_pd(const TaxiDev& p, int env, uint64_t step) {
  if constexpr (REPLAY) {
    const uint32_t pd = (uint32_t)min(max(p.rp_pd[env], 0), p.nlocs * p.nlocs - 1);
    return pd;
  } else {
    const Philox4 r = philox4x32_10((uint32_t)env, (uint32_t)step, (uint32_t)(step >> 32), PHILOX_TAG, p.key0, p.key1);
    const uint32_t pp = lemire_value(r.x[2], (uint32_t)p.nlocs);
    uint32_t dd = lemire_value(r.x[3], (uint32_t)(p.nlocs - 1));
    dd += dd >= pp ? 1u : 0u;
    return pp * (uint32_t)p.nlocs + dd;
  }
}

struct StepOut {
  float rew;
  uint8_t term, trunc;
};

// One env-step of TaxiVecEnv.step (extended_taxi.py:244-287) on the packed state `u`.
template <bool REPLAY>
__device__ __forceinline__ StepOut taxi_env_step(const TaxiDev& p, const uint8_t* lds, uint32_t& u, int a, int env,
                                                 bool live, uint64_t step, float& rsum, uint32_t& eps,
                                                 uint32_t& lens) {
  uint32_t s = u & 0xFFFu, nd = (u >> 12) & 0xFu, el = (u >> 16) + 1u;  // elapsed += 1 (:245)
  // numpy negative indexing of ACTIONS_YX[actions]: -5..-2 are the moves, -1 moves (0,0) but is not
  // a pickup/dropoff (p_or_d = actions == 4, extended_taxi.py:264) -> table column 5 (a no-op).
  // Out-of-range actions raise IndexError in the reference: flagged (GP_DERR_ACTION), then clamped.
  if (live && action_out_of_range(a, NACT)) flag_bad_action(p.derr);
  a = a < 0 ? (a == -1 ? NACT : max(a + NACT, 0)) : min(a, NACT - 1);
  const uint32_t t = l_trans(lds, p)[s * TCOL + (uint32_t)a];
  s = t & 0xFFFu;
  const uint32_t goal = (t >> 12) & 1u, bad = (t >> 13) & 1u;
  nd += goal;                                 // n_dropoffs_completed[goal_move] += 1 (:266)
  StepOut o;
  o.rew = goal ? p.r_goal : (bad ? p.r_bad : p.r_any);
  o.term = (nd == (uint32_t)p.num_passengers) ? 1 : 0;
  o.trunc = (el > (uint32_t)p.time_limit) ? 1 : 0;
  if (!live) return o;                        // padding lane of a ragged batch: no draws, no metrics
  rsum += o.rew;
  if (goal && !(o.term | o.trunc)) {          // task completed, episode continues (:281-284)
    const uint32_t pd = draw_pd<REPLAY>(p, env, step);
    s = (s / (uint32_t)p.lpl) * (uint32_t)p.lpl + pd;  // encode(r, c, p, d): taxi cell kept
  }
  if (o.term | o.trunc) {                     // _reset_mask(done | truncated) (:285, :344-352)
    eps += 1u;
    lens += el;
    s = draw_reset<REPLAY>(p, lds, env, step);
    el = 0u;
    nd = 0u;
  }
  u = s | (nd << 12) | (min(el, 0xFFFFu) << 16);
  return o;
}

// ---- vector I/O (4 consecutive envs per thread) ----
__device__ __forceinline__ bool quad_ok(const void* base, int env0, int B, int esz) {
  return env0 + 3 < B && ((((uintptr_t)base) + (size_t)env0 * esz) & (size_t)(4 * esz - 1)) == 0;
}
__device__ __forceinline__ void ld4_u32(const uint32_t* __restrict__ p, int env0, int B, uint32_t (&v)[4]) {
  if (quad_ok(p, env0, B, 4)) {
    const uint4 q = *reinterpret_cast<const uint4*>(p + env0);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = env0 + i < B ? p[env0 + i] : 0u;
  }
}
__device__ __forceinline__ void st4_u32(uint32_t* __restrict__ p, int env0, int B, const uint32_t (&v)[4]) {
  if (quad_ok(p, env0, B, 4)) {
    *reinterpret_cast<uint4*>(p + env0) = make_uint4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (env0 + i < B) p[env0 + i] = v[i];
  }
}
__device__ __forceinline__ void st4_u8(uint8_t* __restrict__ p, int env0, int B, const uint8_t (&v)[4]) {
  if (quad_ok(p, env0, B, 1)) {
    *reinterpret_cast<uint32_t*>(p + env0) =
        (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) | ((uint32_t)v[3] << 24);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (env0 + i < B) p[env0 + i] = v[i];
  }
}

// ---- one-hot rows as a wave-contiguous chunk stream ----
// The wave owns envs [e0, e0 + n) (lane l holds envs 4l..4l+3), i.e. the byte range
// [e0*W, (e0+n)*W) of the output. Lane l writes chunks q = l, l+64, ... of CS bytes each; the
// host guarantees W % CS == 0 and a CS-aligned range, so a chunk never straddles two rows. The
// hot indices of the wave's envs are exchanged through a per-wave LDS array.
template <int CS>
__device__ __forceinline__ void write_onehot_wave(uint8_t* __restrict__ out, int n, int W, uint16_t* hs,
                                                  const uint32_t (&h)[4], int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) hs[lane * 4 + i] = (uint16_t)h[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int cpe = W / CS;                 // chunks per env row
  const int nchunks = n * cpe;
  // lane's first chunk q = lane: env = lane / cpe, chunk-in-row c = lane % cpe; then += 64 chunks
  int e = lane / cpe, c = lane - e * cpe;
  const int de = 64 / cpe, dc = 64 - de * cpe;
  for (int q = lane; q < nchunks; q += 64) {
    const uint32_t hot = hs[e];
    const int hc = (int)(hot / CS), hb = (int)(hot - (uint32_t)hc * CS);
    uint8_t* dst = out + (size_t)q * CS;
    if constexpr (CS == 16) {
      const uint32_t m = (c == hc) ? (1u << ((hb & 3) * 8)) : 0u;
      const int w = hb >> 2;
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      u32x4 v;
      v.x = w == 0 ? m : 0u; v.y = w == 1 ? m : 0u; v.z = w == 2 ? m : 0u; v.w = w == 3 ? m : 0u;
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
    } else if constexpr (CS == 4) {
      const uint32_t m = (c == hc) ? (1u << (hb * 8)) : 0u;
      __builtin_nontemporal_store(m, reinterpret_cast<uint32_t*>(dst));
    } else {
      *dst = (c == hc) ? 1 : 0;
    }
    e += de;
    c += dc;
    if (c >= cpe) { c -= cpe; e += 1; }
  }
  __builtin_amdgcn_wave_barrier();  // hs is rewritten by the next step
}

// Per-block metrics into the block's own slot (the grid is persistent: block b owns slot b).
template <int NW = WAVES>
__device__ void taxi_metrics(const TaxiDev& p, float rsum, uint32_t eps, uint32_t lens, uint32_t nst) {
  __shared__ float s_r[NW];
  __shared__ uint32_t s_e[NW], s_l[NW], s_n[NW];
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
    for (int w = 0; w < NW; ++w) { r += s_r[w]; e += s_e[w]; l += s_l[w]; n += s_n[w]; }
    TaxiSlot& m = p.mslot[blockIdx.x];
    m.return_sum += (double)r;
    m.episodes += e;
    m.length_sum += l;
    m.env_steps += n;
  }
}

// ---- the rollout kernel: K steps for every env, persistent over 1024-env tiles ----
// OH = 0: scalar int32 obs [K,B]; OH = CS in {16, 4, 1}: one-hot uint8 [K,B,n_obs] in CS-byte chunks.
template <int OH, bool REPLAY>
__global__ __launch_bounds__(TPB) void taxi_rollout(TaxiDev p, int K, uint64_t step0, const int32_t* __restrict__ act,
                                                    void* __restrict__ obs, float* __restrict__ rew,
                                                    uint8_t* __restrict__ term, uint8_t* __restrict__ trunc) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ uint16_t s_hot[WAVES][256];
  stage_tables(p, lds);
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float rsum = 0.f;
  uint32_t eps = 0, lens = 0, nst = 0;
  const uint16_t* obs_of = l_obs(lds, p);
  for (int tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
    const int env0 = tile * EPB + threadIdx.x * EPT;
    uint32_t u[4];
    ld4_u32(p.st, env0, p.B, u);
    for (int k = 0; k < K; ++k) {
      const size_t off = (size_t)k * p.B;
      uint32_t a4[4];
      ld4_u32(reinterpret_cast<const uint32_t*>(act + off), env0, p.B, a4);
      float r[4];
      uint8_t tm[4], tr[4];
      uint32_t h[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool live = env0 + i < p.B;
        StepOut o = taxi_env_step<REPLAY>(p, lds, u[i], (int)a4[i], env0 + i, live, step0 + (uint64_t)k, rsum, eps,
                                          lens);
        r[i] = o.rew;
        tm[i] = o.term;
        tr[i] = o.trunc;
        h[i] = obs_of[u[i] & 0xFFFu];
        nst += live ? 1u : 0u;
      }
      st4_u32(reinterpret_cast<uint32_t*>(rew + off), env0, p.B,
              {__float_as_uint(r[0]), __float_as_uint(r[1]), __float_as_uint(r[2]), __float_as_uint(r[3])});
      st4_u8(term + off, env0, p.B, tm);
      st4_u8(trunc + off, env0, p.B, tr);
      if constexpr (OH == 0) {
        st4_u32(reinterpret_cast<uint32_t*>(obs) + off, env0, p.B, h);
      } else {
        const int we0 = tile * EPB + wid * 256;  // first env of this wave
        const int n = min(256, p.B - we0);
        if (n > 0)
          write_onehot_wave<OH>((uint8_t*)obs + (off + (size_t)we0) * (size_t)p.n_obs, n, p.n_obs, s_hot[wid], h,
                                lane);
      }
    }
    st4_u32(p.st, env0, p.B, u);
  }
  taxi_metrics(p, rsum, eps, lens, nst);
}

// reset(): every env draws a start state (extended_taxi.py:232-242); one step index of the stream.
template <int OH, bool REPLAY>
__global__ __launch_bounds__(TPB) void taxi_reset(TaxiDev p, uint64_t step, void* __restrict__ obs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ uint16_t s_hot[WAVES][256];
  stage_tables(p, lds);
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int tile = blockIdx.x; tile < p.ntiles; tile += gridDim.x) {
    const int env0 = tile * EPB + threadIdx.x * EPT;
    uint32_t u[4], h[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int env = env0 + i;
      u[i] = env < p.B ? draw_reset<REPLAY>(p, lds, env, step) : 0u;
      h[i] = l_obs(lds, p)[u[i]];
    }
    st4_u32(p.st, env0, p.B, u);
    if constexpr (OH == 0) {
      st4_u32(reinterpret_cast<uint32_t*>(obs), env0, p.B, h);
    } else {
      const int we0 = tile * EPB + wid * 256;
      const int n = min(256, p.B - we0);
      if (n > 0) write_onehot_wave<OH>((uint8_t*)obs + (size_t)we0 * p.n_obs, n, p.n_obs, s_hot[wid], h, lane);
    }
  }
}

__global__ void taxi_get_state(TaxiDev p, int32_t* s, int32_t* elapsed, int32_t* nd) {
  const int env = blockIdx.x * TPB + threadIdx.x;
  if (env >= p.B) return;
  const uint32_t u = p.st[env];
  if (s) s[env] = (int32_t)(u & 0xFFFu);
  if (nd) nd[env] = (int32_t)((u >> 12) & 0xFu);
  if (elapsed) elapsed[env] = (int32_t)(u >> 16);
}
__global__ void taxi_set_state(TaxiDev p, const int32_t* s, const int32_t* elapsed, const int32_t* nd) {
  const int env = blockIdx.x * TPB + threadIdx.x;
  if (env >= p.B) return;
  uint32_t u = p.st[env];
  if (s) u = (u & ~0xFFFu) | (uint32_t)min(max(s[env], 0), p.ns - 1);
  if (nd) u = (u & ~0xF000u) | ((uint32_t)min(max(nd[env], 0), 15) << 12);
  if (elapsed) u = (u & 0xFFFFu) | ((uint32_t)min(max(elapsed[env], 0), 65535) << 16);
  p.st[env] = u;
}

// ------------------------------------------------------------------ rendering ----
// TaxiVecEnv.render (extended_taxi.py:289-309) -> str_map_to_img (:121-143) -> tile_images (render_utils.py:63-88):
// one thread per pixel of the tiled frame. Frame k (env k) sits at tile (k / TW, k % TW); its char map is the
// bordered map with 'D' (destination), 'T' (taxi), 'P' (waiting passenger), 'F' (taxi with passenger) and
// "TP" -> 'T' where the waiting passenger shares the taxi's cell (the reference's '<U1' array truncates it).
struct TaxiRender {
  const uint32_t* st;    // packed env state (s | nd << 12 | elapsed << 16)
  const uint8_t* desc;   // [DR][DC] bordered char map
  const int32_t* lrc;    // [L][2] bordered (row, col) of each location
  int32_t DR, DC, C, L, pseudo, n, TW, rows, cols, hansen;
};
__global__ void taxi_render_kernel(TaxiRender p, uint8_t* out) {
  const int pix = blockIdx.x * TPB + threadIdx.x;
  if (pix >= p.rows * p.cols) return;
  const int y = pix / p.cols, x = pix - y * p.cols;
  const int ty = y / p.DR, tx = x / p.DC, r = y - ty * p.DR, c = x - tx * p.DC;
  const int k = ty * p.TW + tx;
  uint8_t rgb[3] = {0, 0, 0};  // padding frames are black
  if (k < p.n) {
    const int s = (int)(p.st[k] & 0xFFFu);
    const int d = s % p.L, t = s / p.L, pp = t % (p.L + 1), t2 = t / (p.L + 1);
    const int tr = t2 / p.C + 1, tc = p.pseudo ? 2 * (t2 % p.C) + 1 : t2 % p.C + 1;
    char ch = (char)p.desc[r * p.DC + c];
    if (r == p.lrc[2 * d] && c == p.lrc[2 * d + 1]) ch = 'D';
    const bool at_taxi = r == tr && c == tc;
    if (at_taxi) ch = 'T';
    if (pp < p.L) {
      const int pr = p.lrc[2 * pp], pc = p.lrc[2 * pp + 1];
      if (r == pr && c == pc) ch = (pr == tr && pc == tc) ? 'T' : 'P';
    } else if (at_taxi) {
      ch = 'F';
    }
    switch (ch) {  // render_utils.py:11-24 palette
      case '|': break;                                          // WALL black
      case 'P': rgb[0] = 128; rgb[2] = 128; break;              // PASSENGER purple
      case 'T': rgb[0] = 128; rgb[1] = 128; break;              // TAXI yellow
      case 'F': rgb[1] = 128; break;                            // FULL_TAXI green
      case 'D': rgb[2] = 128; break;                            // DESTINATION blue
      case ' ': rgb[0] = rgb[1] = rgb[2] = 96; break;           // FLOOR gray_mid_dark
      case ':': rgb[1] = 128; rgb[2] = 128; break;              // FAKE_WALL teal
      default: rgb[0] = rgb[1] = rgb[2] = 191; break;           // LOC gray_light
    }
    // Hansen highlight (:136-142): the taxi's four orthogonal neighbours +64, wrapping
    if (p.hansen && ((r == tr && (c == tc - 1 || c == tc + 1)) || (c == tc && (r == tr - 1 || r == tr + 1))))
      for (int j = 0; j < 3; ++j) rgb[j] = (uint8_t)(rgb[j] + 64);
  }
  uint8_t* o = out + (size_t)pix * 3;
  o[0] = rgb[0]; o[1] = rgb[1]; o[2] = rgb[2];
}

// cv2.resize(..., INTER_AREA) outside the decimation case (OpenCV resizeGeneric_ with area coefficients, 11-bit
// fixed point; restated, see oracle/render.py): per destination pixel and channel.
struct ResizeArea {
  const uint8_t* src;
  const int32_t* xofs;   // [dw] source column
  const int16_t* xa;     // [dw][2]
  const int32_t* yofs;   // [dh] source row
  const int16_t* yb;     // [dh][2]
  int32_t sh, sw, ch, dh, dw, dpitch;
};
__global__ void resize_area_kernel(ResizeArea p, uint8_t* dst) {
  const int i = blockIdx.x * TPB + threadIdx.x;
  if (i >= p.dh * p.dw * p.ch) return;
  const int k = i % p.ch, t = i / p.ch, dx = t % p.dw, dy = t / p.dw;
  const int x0 = p.xofs[dx], x1 = min(x0 + 1, p.sw - 1);
  const int y0 = min(max(p.yofs[dy], 0), p.sh - 1), y1 = min(max(p.yofs[dy] + 1, 0), p.sh - 1);
  const int a0 = p.xa[2 * dx], a1 = p.xa[2 * dx + 1];
  const uint8_t* r0 = p.src + (size_t)y0 * p.sw * p.ch;
  const uint8_t* r1 = p.src + (size_t)y1 * p.sw * p.ch;
  const int S0 = r0[x0 * p.ch + k] * a0 + r0[x1 * p.ch + k] * a1;  // HResizeLinear (int)
  const int S1 = r1[x0 * p.ch + k] * a0 + r1[x1 * p.ch + k] * a1;
  const int b0 = p.yb[2 * dy], b1 = p.yb[2 * dy + 1];
  const int v = (((b0 * (S0 >> 4)) >> 16) + ((b1 * (S1 >> 4)) >> 16) + 2) >> 2;  // VResizeLinear<uchar>
  dst[(size_t)dy * p.dpitch + (size_t)dx * p.ch + k] = (uint8_t)min(max(v, 0), 255);
}

// ------------------------------------------------------------------ numpy mode ----
// rng_mode "numpy": the reference's own stream (extended_taxi.py:281-286, 344-364), draw for draw, so that a seeded
// run reproduces TaxiVecEnv's obs / rewards / dones and its final PCG64 state. One workgroup of NP_TPB threads
// runs K steps per launch:
//  1. transitions of every env (coalesced 1024-env tiles), each tile's task completions (tc) and resets (rs)
//     ranked in env order by a workgroup scan;
//  2. _reset_passenger_and_destination: integers(L, b1) for p, then for d, then the `while d == p` redraws,
//     numpy's buffered 32-bit Lemire draws (distributions.c random_bounded_uint64_fill -> buffered_bounded_lemire_
//     uint32 on next_uint32) -- serial on one lane (a handful per step);
//  3. _reset_mask: multinomial(ns, state_distribution, b2).argmax(-1), numpy's random_multinomial: per valid
//     category in order a random_binomial(p_j / remaining_p, dn) by inversion (random_binomial_inversion, one
//     next_double per try, q^n = exp(n log q) with glibc's exp restated in gp_libm.h), stopping when dn hits 0.
//     A row draws C0 doubles (one per drawn category) unless it stops early or an inversion restarts, so rows are
//     walked SPECULATIVELY: lane (l, delta) walks row r0 + l from stream offset C0 l - delta; lane 0 then chains
//     the rows whose guessed offset was right (delta = the deficit of the rows before) and the next round starts
//     after them. 64 rows x 16 deficits per round; the deficit grows ~0.25 per row.
//  4. the task / episode resets applied, observations written.
// Host tables per category (p_j, q_j = 1 - p_j, log q_j with the C library's log, flipped when p_j > 0.5 as
// random_binomial does) keep every dn-independent value identical to numpy's.
constexpr int NP_TPB = 1024;
constexpr int NP_WAVES = NP_TPB / 64;
constexpr int SPEC_DEF = 16;                   // deficits per speculative row
constexpr int SPEC_ROWS = NP_TPB / SPEC_DEF;   // rows per round
constexpr uint32_t NP_INV_CAP = 1u << 20;      // inversion tries before a row is flagged (numpy would loop on)

struct TaxiNpDev {
  uint64_t* rng;          // [6] state hi, lo, inc hi, lo, has_uint32, uinteger
  const uint8_t* mtab;    // category tables (staged into LDS): pp f64 | q f64 | lq f64 | cat u16 | flip u8
  int32_t off_pp, off_q, off_lq, off_cat, off_flip, mtab_bytes;
  int32_t C0;             // categories a row draws when it neither stops early nor restarts
  int32_t n;              // balls per row (= ns)
  int32_t last;           // the last category (ns - 1): count dn if the row ends with dn > 0
  const PcgJump* jrow;    // [NP_TPB]: jump by C0 l - delta (lane l * SPEC_DEF + delta)
  const PcgJump* jt;      // radix-64 general jump tables
  int32_t* rk;            // [B] this step's rank: -1, tc rank, or rs rank | 1 << 30
  int32_t* vtc;           // [B] tc rank -> p << 16 | d
  uint16_t* vrs;          // [B] rs rank -> start state
};

struct NpRng {
  u128 s, inc;
  uint32_t has, uval;
};
// pcg64_next32: the buffered high half first
__device__ __forceinline__ uint32_t np_next32(NpRng& g) {
  if (g.has) {
    g.has = 0;
    return g.uval;
  }
  g.s = pcg_step(g.s, g.inc);
  const uint64_t x = pcg_output(g.s);
  g.has = 1;
  g.uval = (uint32_t)(x >> 32);
  return (uint32_t)x;
}
// integers(n) with int64 output: random_bounded_uint64_fill(rng = n - 1) -> buffered_bounded_lemire_uint32
__device__ __forceinline__ uint32_t np_integers(NpRng& g, uint32_t n) {
  if (n <= 1) return 0;  // rng == 0: no draw
  uint64_t m = (uint64_t)np_next32(g) * n;
  uint32_t left = (uint32_t)m;
  if (left < n) {
    const uint32_t thr = (0xFFFFFFFFu - (n - 1)) % n;
    while (left < thr) {
      m = (uint64_t)np_next32(g) * n;
      left = (uint32_t)m;
    }
  }
  return (uint32_t)(m >> 32);
}
__device__ __forceinline__ double np_next_double(u128& s, u128 inc) {
  s = pcg_step(s, inc);
  return (double)(pcg_output(s) >> 11) * (1.0 / 9007199254740992.0);
}

struct NpCats {
  const double *pp, *q, *lq;
  const uint16_t* cat;
  const uint8_t* flip;
  const uint64_t* etab;  // exp table (LDS copy)
};

// The host libm's exp build (gp_exp_host_variant: 1 the -mfma build, 0 the plain one), set at create time.
__device__ int g_taxi_exp_fma = 1;

// One multinomial row from state s: the argmax category; `used` = doubles drawn.
__device__ __forceinline__ uint32_t np_row(const TaxiNpDev& q, const NpCats& c, u128 s, u128 inc, uint32_t& used,
                                           uint32_t& flags) {
#pragma clang fp contract(off)
  int64_t dn = q.n, best = -1;
  uint32_t arg = 0, u = 0;
  for (int k = 0; k < q.C0; ++k) {
    const double pp = c.pp[k];
    int64_t X = 0;
    if (pp * (double)dn <= 30.0) {  // random_binomial -> random_binomial_inversion(dn, pp)
      const double qq = c.q[k];
      const double qn = g_taxi_exp_fma ? gp_libm::exp<true>((double)dn * c.lq[k], c.etab)
                                       : gp_libm::exp<false>((double)dn * c.lq[k], c.etab);
      const double np = (double)dn * pp;
      const double bnd = np + 10.0 * __builtin_sqrt(np * qq + 1.0);
      const int64_t bound = (int64_t)((double)dn < bnd ? (double)dn : bnd);
      double px = qn, U = np_next_double(s, inc);
      ++u;
      uint32_t tries = 0;
      while (U > px) {
        ++X;
        if (X > bound) {
          X = 0;
          px = qn;
          U = np_next_double(s, inc);
          ++u;
        } else {
          U -= px;
          px = ((double)(dn - X + 1) * pp * px) / ((double)X * qq);
        }
        if (++tries > NP_INV_CAP) {
          flags |= GP_DERR_BTPE;
          break;
        }
      }
    } else {
      flags |= GP_DERR_BTPE;  // numpy's BTPE: not restated
    }
    if (c.flip[k]) X = dn - X;
    if (X > best) {
      best = X;
      arg = c.cat[k];
    }
    dn -= X;
    if (dn <= 0) break;
  }
  if (dn > 0 && dn > best) arg = (uint32_t)q.last;
  used = u;
  return arg;
}

// Workgroup scan of two flags over one 1024-env tile: ranks below this thread (env order) and the tile totals.
__device__ __forceinline__ void np_tile_scan(bool ftc, bool frs, uint32_t* wcnt, uint32_t& rtc, uint32_t& rrs,
                                             uint32_t& ttc, uint32_t& trs) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t btc = __ballot((int)ftc), brs = __ballot((int)frs);
  if (lane == 0) wcnt[w] = (uint32_t)__builtin_popcountll(btc) | ((uint32_t)__builtin_popcountll(brs) << 16);
  __syncthreads();
  uint32_t pre = 0, tot = 0;
  for (int i = 0; i < NP_WAVES; ++i) {
    const uint32_t v = wcnt[i];
    pre += i < w ? v : 0u;
    tot += v;
  }
  const uint32_t mtc = __builtin_amdgcn_mbcnt_hi((uint32_t)(btc >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)btc, 0u));
  const uint32_t mrs = __builtin_amdgcn_mbcnt_hi((uint32_t)(brs >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)brs, 0u));
  rtc = (pre & 0xFFFFu) + mtc;
  rrs = (pre >> 16) + mrs;
  ttc = tot & 0xFFFFu;
  trs = tot >> 16;
  __syncthreads();  // wcnt is reused by the next tile
}

struct NpShared {
  uint32_t wcnt[NP_WAVES];
  uint32_t b1, b2, r0, flags;
  uint64_t S[2];                // the stream state between phases (hi, lo)
  uint32_t has, uval;
  uint16_t res_arg[NP_TPB];
  uint16_t res_used[NP_TPB];
};

// The rows of this step's b2 resets (ranks 0..b2-1 -> q.vrs), all threads.
__device__ void np_reset_rows(const TaxiDev& p, const TaxiNpDev& q, const NpCats& c, NpShared& sh, uint32_t b2) {
  const int t = threadIdx.x;
  const int l = t / SPEC_DEF, del = t % SPEC_DEF;
  const PcgJump jl = q.jrow[t];
  const u128 inc = mk128(q.rng[2], q.rng[3]);
  uint32_t r0 = 0;
  uint32_t flags = 0;
  while (r0 < b2) {
    const u128 S = mk128(sh.S[0], sh.S[1]);
    if (r0 + (uint32_t)l < b2 && !(l == 0 && del > 0)) {
      uint32_t used = 0;
      const uint32_t a = np_row(q, c, apply_jump(jl, S), inc, used, flags);
      sh.res_arg[t] = (uint16_t)a;
      sh.res_used[t] = (uint16_t)min(used, 65535u);
    }
    __syncthreads();
    if (t == 0) {  // chain the rows whose guessed offset was right
      int32_t D = 0;
      uint32_t n = 0;
      while (r0 + n < b2 && n < (uint32_t)SPEC_ROWS && D >= 0 && D < SPEC_DEF) {
        const int u = (int)n * SPEC_DEF + D;
        q.vrs[r0 + n] = sh.res_arg[u];
        D += q.C0 - (int32_t)sh.res_used[u];
        ++n;
      }
      const u128 S2 = pcg_jump(q.jt, S, (uint32_t)((int64_t)q.C0 * n - D));
      sh.S[0] = hi64(S2);
      sh.S[1] = lo64(S2);
      sh.r0 = r0 + n;
    }
    __syncthreads();
    r0 = sh.r0;
  }
  if (flags) atomicOr(p.derr, flags);
}

// _reset_passenger_and_destination's draws (extended_taxi.py:360-363) across the workgroup. numpy's integers(L, b)
// is b buffered 32-bit Lemire draws (random_bounded_uint64_fill -> buffered_bounded_lemire_uint32), one next_uint32
// each unless a word is rejected (leftover < (2^32 - L) % L: never for L a power of two, p ~ L / 2^32 otherwise).
// So with no rejection half-word k of the stream (the buffered half first) is p of completion k for k < b1, d of
// completion k - b1 for k < 2 b1, and every `while d == p` round gives its colliding completions, in env order, the
// next half-words by rank. Each thread makes the half-words of a contiguous range of positions: one jump from the
// step's state, then LCG steps. Returns false (nothing written to the stream state) when a word in these ranges is
// rejected: the caller then walks the stream serially.
__device__ bool np_pd_parallel(const TaxiDev& p, const TaxiNpDev& q, NpShared& sh, uint32_t b1) {
  __shared__ uint32_t s_cnt[NP_WAVES];
  __shared__ uint32_t s_flag;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t L = (uint32_t)p.nlocs;
  const uint32_t thr = (0xFFFFFFFFu - (L - 1u)) % L;
  const u128 S = mk128(sh.S[0], sh.S[1]), inc = mk128(q.rng[2], q.rng[3]);
  const uint32_t h0 = sh.has, u0 = sh.uval;
  uint16_t* vh = reinterpret_cast<uint16_t*>(q.vtc);  // completion i: [2 i] = d, [2 i + 1] = p
  if (t == 0) s_flag = 0;
  __syncthreads();
  // half-words [k0, k0 + n) of the stream -> f(k, value); rejections flagged
  auto words = [&](uint32_t k0, uint32_t n, auto&& f) {
    if (!n) return;
    uint32_t k = k0, left = n;
    if (h0 && k == 0) {  // the buffered half
      f(k, u0);
      ++k;
      --left;
    }
    if (!left) return;
    const uint32_t j = h0 ? k - 1u : k;  // position among the fresh halves
    u128 st = pcg_jump(q.jt, S, j / 2u + 1u);
    uint64_t x = pcg_output(st);
    bool hi = (j & 1u) != 0;
    for (; left; --left, ++k) {
      f(k, hi ? (uint32_t)(x >> 32) : (uint32_t)x);
      if (hi) {
        st = pcg_step(st, inc);
        x = pcg_output(st);
      }
      hi = !hi;
    }
  };
  auto lemire = [&](uint32_t word, bool& rej) {
    const uint64_t m = (uint64_t)word * L;
    rej |= (uint32_t)m < thr;
    return (uint32_t)(m >> 32);
  };
  bool rej = false;
  {  // p of every completion, then d: half-words 0 .. 2 b1 - 1
    const uint32_t n = 2u * b1, per = (n + NP_TPB - 1u) / NP_TPB;
    const uint32_t k0 = min((uint32_t)t * per, n), k1 = min(k0 + per, n);
    words(k0, k1 - k0, [&](uint32_t k, uint32_t v) {
      const uint32_t x = lemire(v, rej);
      if (k < b1) vh[2 * k + 1] = (uint16_t)x;
      else vh[2 * (k - b1)] = (uint16_t)x;
    });
  }
  uint32_t pos = 2u * b1;
  const uint32_t per = (b1 + NP_TPB - 1u) / NP_TPB;  // completions per thread (env order)
  const uint32_t i0 = min((uint32_t)t * per, b1), i1 = min(i0 + per, b1);
  for (int round = 0; round < 4096; ++round) {
    if (rej) s_flag = 1;  // (benign race: every writer stores 1)
    __threadfence_block();
    __syncthreads();
    if (s_flag) return false;
    // this round's colliding completions (p == d), ranked in env order
    uint32_t c = 0;
    for (uint32_t i = i0; i < i1; ++i) c += vh[2 * i] == vh[2 * i + 1] ? 1u : 0u;
    uint32_t v = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(v, d, 64);
      if (lane >= d) v += y;
    }
    if (lane == 63) s_cnt[w] = v;
    __syncthreads();
    uint32_t base = 0, m = 0;
    for (int x = 0; x < NP_WAVES; ++x) {
      base += x < w ? s_cnt[x] : 0u;
      m += s_cnt[x];
    }
    base += v - c;
    __syncthreads();  // (s_cnt reused next round)
    if (m == 0) break;
    if (c) {  // my colliders take half-words pos + base .. pos + base + c - 1, in order
      uint32_t i = i0;
      words(pos + base, c, [&](uint32_t, uint32_t val) {
        while (vh[2 * i] != vh[2 * i + 1]) ++i;  // the next collider (its d is rewritten below)
        vh[2 * i] = (uint16_t)lemire(val, rej);
        ++i;
      });
    }
    pos += m;
  }
  __threadfence_block();
  __syncthreads();
  if (t == 0) {  // the stream after `pos` half-words
    uint32_t used, h;
    if (h0) {
      used = pos >> 1;
      h = (pos - 1u) & 1u;
    } else {
      used = (pos + 1u) >> 1;
      h = pos & 1u;
    }
    const u128 S2 = used ? pcg_jump(q.jt, S, used) : S;
    sh.S[0] = hi64(S2);
    sh.S[1] = lo64(S2);
    sh.has = h;
    if (used) sh.uval = (uint32_t)(pcg_output(S2) >> 32);  // numpy keeps the last drawn high half (buffered or not)
  }
  __syncthreads();
  return true;
}

// The draws of one step (or of reset(): b1 = 0, every env a reset), between the two env passes.
__device__ void np_draws(const TaxiDev& p, const TaxiNpDev& q, const NpCats& c, NpShared& sh, bool rows = true) {
  const uint32_t b1 = sh.b1, b2 = sh.b2;
  const bool done_pd = b1 && np_pd_parallel(p, q, sh, b1);
  if (threadIdx.x == 0 && !done_pd) {
    NpRng g{mk128(sh.S[0], sh.S[1]), mk128(q.rng[2], q.rng[3]), sh.has, sh.uval};
    if (b1) {  // extended_taxi.py:360-363
      const uint32_t L = (uint32_t)p.nlocs;
      for (uint32_t i = 0; i < b1; ++i) q.vtc[i] = (int32_t)(np_integers(g, L) << 16);
      for (uint32_t i = 0; i < b1; ++i) q.vtc[i] |= (int32_t)np_integers(g, L);
      bool any = true;
      for (uint32_t it = 0; any && it < (1u << 20); ++it) {
        any = false;
        for (uint32_t i = 0; i < b1; ++i) {
          const int32_t v = q.vtc[i];
          if ((v >> 16) == (v & 0xFFFF)) {
            q.vtc[i] = (v & ~0xFFFF) | (int32_t)np_integers(g, L);
            any = true;
          }
        }
      }
    }
    sh.S[0] = hi64(g.s);
    sh.S[1] = lo64(g.s);
    sh.has = g.has;
    sh.uval = g.uval;
  }
  __syncthreads();
  if (b2 && rows) np_reset_rows(p, q, c, sh, b2);
}

// The numpy-mode rollout / reset: one workgroup, K steps (K = 0: reset(), every env draws a start state).
template <bool ONEHOT>
__global__ __launch_bounds__(NP_TPB) void taxi_np_kernel(TaxiDev p, TaxiNpDev q, int K, const int32_t* __restrict__ act,
                                                         void* __restrict__ obs, float* __restrict__ rew,
                                                         uint8_t* __restrict__ term, uint8_t* __restrict__ trunc) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ NpShared sh;
  __shared__ uint64_t etab[256];
  const int t = threadIdx.x;
  {  // tables: the env tables, then the category tables behind them, the exp table
    const uint4* s1 = (const uint4*)p.tabs;
    uint4* d1 = (uint4*)lds;
    for (int i = t; i < p.tab_bytes / 16; i += NP_TPB) d1[i] = s1[i];
    const uint4* s2 = (const uint4*)q.mtab;
    uint4* d2 = (uint4*)(lds + p.tab_bytes);
    for (int i = t; i < q.mtab_bytes / 16; i += NP_TPB) d2[i] = s2[i];
    for (int i = t; i < 256; i += NP_TPB) etab[i] = gp_libm::kExpTab[i];
    if (t == 0) {
      sh.S[0] = q.rng[0];
      sh.S[1] = q.rng[1];
      sh.has = (uint32_t)q.rng[4];
      sh.uval = (uint32_t)q.rng[5];
    }
  }
  __syncthreads();
  const uint8_t* mt = lds + p.tab_bytes;
  const NpCats c{(const double*)(mt + q.off_pp), (const double*)(mt + q.off_q), (const double*)(mt + q.off_lq),
                 (const uint16_t*)(mt + q.off_cat), mt + q.off_flip, etab};
  const uint16_t* obs_of = l_obs(lds, p);
  const int B = p.B, ntile = (B + NP_TPB - 1) / NP_TPB;
  float rsum = 0.f;
  uint32_t eps = 0, lens = 0, nst = 0;
  const int steps = K > 0 ? K : 1;
  for (int k = 0; k < steps; ++k) {
    const size_t off = (size_t)k * B;
    // ---- pass 1: transitions (steps) or every env a reset (reset()), ranked in env order ----
    uint32_t ntc = 0, nrs = 0;
    for (int tile = 0; tile < ntile; ++tile) {
      const int env = tile * NP_TPB + t;
      const bool live = env < B;
      bool ftc = false, frs = false;
      if (K == 0) {
        frs = live;
      } else if (live) {
        uint32_t u = p.st[env];
        uint32_t s = u & 0xFFFu, nd = (u >> 12) & 0xFu, el = (u >> 16) + 1u;
        int a = act[off + env];
        if (action_out_of_range(a, NACT)) flag_bad_action(p.derr);
        a = a < 0 ? (a == -1 ? NACT : max(a + NACT, 0)) : min(a, NACT - 1);
        const uint32_t tr = l_trans(lds, p)[s * TCOL + (uint32_t)a];
        s = tr & 0xFFFu;
        const uint32_t goal = (tr >> 12) & 1u, bad = (tr >> 13) & 1u;
        nd += goal;
        const float r = goal ? p.r_goal : (bad ? p.r_bad : p.r_any);
        const bool dterm = nd == (uint32_t)p.num_passengers, dtrunc = el > (uint32_t)p.time_limit;
        rew[off + env] = r;
        term[off + env] = dterm ? 1 : 0;
        trunc[off + env] = dtrunc ? 1 : 0;
        rsum += r;
        nst += 1u;
        ftc = goal && !(dterm || dtrunc);
        frs = dterm || dtrunc;
        if (frs) {
          eps += 1u;
          lens += el;
        }
        p.st[env] = s | (nd << 12) | (min(el, 0xFFFFu) << 16);
      }
      uint32_t rtc, rrs, ttc, trs;
      np_tile_scan(ftc, frs, sh.wcnt, rtc, rrs, ttc, trs);
      if (live) q.rk[env] = ftc ? (int32_t)(ntc + rtc) : (frs ? (int32_t)((nrs + rrs) | (1u << 30)) : -1);
      ntc += ttc;
      nrs += trs;
    }
    if (t == 0) {
      sh.b1 = ntc;
      sh.b2 = nrs;
    }
    __syncthreads();
    // ---- the draws, in the reference's order ----
    np_draws(p, q, c, sh);
    __syncthreads();
    // ---- pass 2: task / episode resets applied, observations ----
    for (int tile = 0; tile < ntile; ++tile) {
      const int env = tile * NP_TPB + t;
      if (env >= B) continue;
      uint32_t u = p.st[env];
      const int32_t r = q.rk[env];
      if (r >= 0) {
        if (r & (1 << 30)) {
          u = q.vrs[r & ~(1 << 30)];  // _reset_mask: new start state, elapsed 0, dropoffs 0
        } else {
          const int32_t v = q.vtc[r];  // encode(r, c, p, d): taxi cell kept
          const uint32_t s = u & 0xFFFu;
          const uint32_t s2 = (s / (uint32_t)p.lpl) * (uint32_t)p.lpl + (uint32_t)(v >> 16) * (uint32_t)p.nlocs +
                              (uint32_t)(v & 0xFFFF);
          u = (u & ~0xFFFu) | s2;
        }
        p.st[env] = u;
      }
      const uint32_t h = obs_of[u & 0xFFFu];
      if constexpr (!ONEHOT) {
        reinterpret_cast<int32_t*>(obs)[off + env] = (int32_t)h;
      } else {
        uint8_t* row = (uint8_t*)obs + (off + env) * (size_t)p.n_obs;
        for (int i = 0; i < p.n_obs; ++i) row[i] = (uint32_t)i == h ? 1 : 0;
      }
    }
    __syncthreads();
  }
  if (t == 0) {
    q.rng[0] = sh.S[0];
    q.rng[1] = sh.S[1];
    q.rng[4] = sh.has;
    q.rng[5] = sh.uval;
  }
  if (K > 0) taxi_metrics<NP_WAVES>(p, rsum, eps, lens, nst);
}

// ---- numpy mode, grid-wide (B > NPG_MIN_ENVS): the same step as three launches ----
// Only the draws walk the stream (one workgroup, np_draws as above); both env passes run over every CU:
//   taxi_npg_pass1  one 1024-env tile per block: transitions, rewards / flags, and each env's rank among its
//                   tile's task completions (tc) and episode resets (rs) in env order; the tile's two counts;
//   taxi_npg_draws  the tiles' counts -> per-tile prefixes and the step's b1 / b2, then the draws;
//   taxi_npg_pass2  one tile per block: resets applied (rank = tile prefix + rank in the tile), observations.
// (reset(): pass 1 flags every env a reset, pass 2 writes the obs.)
constexpr int NPG_MIN_ENVS = 1024;  // at or below: the one-workgroup kernel (K steps per launch; measured crossover)

struct NpgDev {
  uint32_t* bcnt;   // [ntiles] tile counts: tc | rs << 16
  uint64_t* bpre;   // [ntiles] tile prefixes: tc | rs << 32
  int32_t grid;     // metric slots (p.mslot)
  // the multinomial rows, grid-wide (taxi_npg_rows)
  uint32_t* rres;   // [RW_R * RW_W] row results: arg << 16 | doubles used (0xFFFF: not evaluated)
  uint32_t* rctl;   // [16] 0: barrier arrivals (monotone), 1: b2 (rows of this step), 2: rows done (r0), 3: the mean
                    //      deficit per row x 256 (window centre), 5: the arrival count a launch starts from
  uint64_t* rst;    // [2] the stream state at the round's first row (hi, lo)
  int32_t rgrid;    // blocks of taxi_npg_rows (all resident: one per CU)
};

// Exclusive block scan of a u64 per thread (256 threads); the block total in tot.
__device__ __forceinline__ uint64_t npg_scan64(uint64_t x, uint64_t& tot) {
  __shared__ uint64_t ws[WAVES];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t v = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(v, d, 64);
    if (lane >= d) v += y;
  }
  if (lane == 63) ws[w] = v;
  __syncthreads();
  uint64_t base = 0;
  tot = 0;
#pragma unroll
  for (int i = 0; i < WAVES; ++i) {
    base += i < w ? ws[i] : 0ull;
    tot += ws[i];
  }
  __syncthreads();
  return base + v - x;
}

// Metrics of a block into slot (block mod slots), atomically (more blocks than slots).
__device__ void npg_metrics(const TaxiDev& p, int slots, float rsum, uint32_t eps, uint32_t lens, uint32_t nst) {
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
    TaxiSlot& m = p.mslot[blockIdx.x % (unsigned)slots];
    atomicAdd(&m.return_sum, (double)r);
    atomicAdd(&m.episodes, e);
    atomicAdd(&m.length_sum, l);
    atomicAdd(&m.env_steps, n);
  }
}

// Pass 1 of step k (RESET: reset(), every env flagged a reset).
template <bool RESET>
__global__ __launch_bounds__(TPB) void taxi_npg_pass1(TaxiDev p, TaxiNpDev q, NpgDev g, size_t off,
                                                      const int32_t* __restrict__ act, float* __restrict__ rew,
                                                      uint8_t* __restrict__ term, uint8_t* __restrict__ trunc) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  if (!RESET) stage_tables(p, lds);
  __syncthreads();
  const int tile = blockIdx.x, env0 = tile * EPB + threadIdx.x * EPT;
  float rsum = 0.f;
  uint32_t eps = 0, lens = 0, nst = 0;
  bool ftc[EPT], frs[EPT];
  if (RESET) {
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      ftc[i] = false;
      frs[i] = env0 + i < p.B;
    }
  } else {
    uint32_t u[4], a4[4];
    ld4_u32(p.st, env0, p.B, u);
    ld4_u32(reinterpret_cast<const uint32_t*>(act + off), env0, p.B, a4);
    float r[4];
    uint8_t tm[4], tr[4];
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const bool live = env0 + i < p.B;
      ftc[i] = frs[i] = false;
      r[i] = 0.f;
      tm[i] = tr[i] = 0;
      if (!live) continue;
      uint32_t s = u[i] & 0xFFFu, nd = (u[i] >> 12) & 0xFu, el = (u[i] >> 16) + 1u;
      int a = (int)a4[i];  // extended_taxi.py:344-364 (as taxi_np_kernel's pass 1)
      if (action_out_of_range(a, NACT)) flag_bad_action(p.derr);
      a = a < 0 ? (a == -1 ? NACT : max(a + NACT, 0)) : min(a, NACT - 1);
      const uint32_t t = l_trans(lds, p)[s * TCOL + (uint32_t)a];
      s = t & 0xFFFu;
      const uint32_t goal = (t >> 12) & 1u, bad = (t >> 13) & 1u;
      nd += goal;
      r[i] = goal ? p.r_goal : (bad ? p.r_bad : p.r_any);
      const bool dterm = nd == (uint32_t)p.num_passengers, dtrunc = el > (uint32_t)p.time_limit;
      tm[i] = dterm ? 1 : 0;
      tr[i] = dtrunc ? 1 : 0;
      rsum += r[i];
      nst += 1u;
      ftc[i] = goal && !(dterm || dtrunc);
      frs[i] = dterm || dtrunc;
      if (frs[i]) {
        eps += 1u;
        lens += el;
      }
      u[i] = s | (nd << 12) | (min(el, 0xFFFFu) << 16);
    }
    st4_u32(reinterpret_cast<uint32_t*>(rew + off), env0, p.B,
            {__float_as_uint(r[0]), __float_as_uint(r[1]), __float_as_uint(r[2]), __float_as_uint(r[3])});
    st4_u8(term + off, env0, p.B, tm);
    st4_u8(trunc + off, env0, p.B, tr);
    st4_u32(p.st, env0, p.B, u);
  }
  // ranks in env order within the tile (env0 + i: thread-major, then i)
  uint32_t ctc = 0, crs = 0;
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    ctc += ftc[i] ? 1u : 0u;
    crs += frs[i] ? 1u : 0u;
  }
  uint64_t tot;
  const uint64_t base = npg_scan64((uint64_t)ctc | ((uint64_t)crs << 32), tot);
  uint32_t rtc = (uint32_t)base, rrs = (uint32_t)(base >> 32);
  int32_t rk[4];
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    rk[i] = ftc[i] ? (int32_t)rtc : (frs[i] ? (int32_t)(rrs | (1u << 30)) : -1);
    rtc += ftc[i] ? 1u : 0u;
    rrs += frs[i] ? 1u : 0u;
  }
  st4_u32(reinterpret_cast<uint32_t*>(q.rk), env0, p.B,
          {(uint32_t)rk[0], (uint32_t)rk[1], (uint32_t)rk[2], (uint32_t)rk[3]});
  if (threadIdx.x == 0) g.bcnt[tile] = (uint32_t)tot | ((uint32_t)(tot >> 32) << 16);
  if (!RESET) npg_metrics(p, g.grid, rsum, eps, lens, nst);
}

// ---- the multinomial rows of a step (or of reset()) grid-wide: taxi_npg_rows ----
// A row's start in the stream is the sum of the doubles the rows before it used: C0 each unless a row stops early
// (the last categories empty) or an inversion restarts, so the deficit D_i = C0 i - (start of row i) drifts by a
// few tenths per row. Each round evaluates rows r0 .. r0 + RW_R - 1 at RW_W candidate starts each, centred on
// the drift predicted from earlier rounds (lane (i, j): start C0 i - (base_i + j), base_i = m i - RW_W / 2), one
// row per thread over the whole grid; then block 0 chains them in order from the exact D_0 = 0 (row i's result
// at its true D_i is looked up, D_{i+1} = D_i + C0 - used) until a true start falls outside its candidates or the
// rows run out, and the next round starts at the first unchained row (row r0 is always chained: base_0 <= 0). A
// grid barrier (one counter, bounded spins) separates the evaluation from the chain and the chain from the next
// round's evaluation.
constexpr int RW_W = 64;        // candidate starts per row
constexpr int RW_R = 1024;      // rows per round (RW_R * RW_W threads: one row each)
constexpr int RW_TPB = 256;
constexpr int RW_CHUNK = 128;   // rows block 0 stages in LDS at a time while chaining
constexpr uint32_t RW_SPIN = 1u << 24;

__device__ __forceinline__ void npg_grid_barrier(const TaxiDev& p, uint32_t* ctr, uint32_t target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();  // this block's results / publications before its arrival
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t n = 0;
    while ((int32_t)(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++n > RW_SPIN) {
        atomicOr(p.derr, GP_DERR_TIMEOUT);
        break;
      }
    }
    __threadfence();  // acquire: the others' writes
  }
  __syncthreads();
}

__device__ __forceinline__ int32_t rw_base(uint32_t mdef, uint32_t i) {
  return (int32_t)(((uint64_t)mdef * i) >> 8) - RW_W / 2;
}

// Persistent: every block stages the category tables, then rounds of evaluation + chain until the step's b2 rows
// are placed (q.vrs[r] = start state of reset rank r); block 0 leaves the stream state after the last row in q.rng.
__global__ __launch_bounds__(RW_TPB) void taxi_npg_rows(TaxiDev p, TaxiNpDev q, NpgDev g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ uint64_t etab[256];
  __shared__ uint32_t s_r0, s_n, s_mdef;
  __shared__ int32_t s_D;
  __shared__ uint64_t s_S[2];
  const int t = threadIdx.x;
  {
    const uint4* s2 = (const uint4*)q.mtab;
    uint4* d2 = (uint4*)lds;
    for (int i = t; i < q.mtab_bytes / 16; i += RW_TPB) d2[i] = s2[i];
    for (int i = t; i < 256; i += RW_TPB) etab[i] = gp_libm::kExpTab[i];
  }
  uint32_t* res_lds = reinterpret_cast<uint32_t*>(lds + ((q.mtab_bytes + 15) & ~15));  // block 0: RW_CHUNK x RW_W
  const NpCats c{(const double*)(lds + q.off_pp), (const double*)(lds + q.off_q), (const double*)(lds + q.off_lq),
                 (const uint16_t*)(lds + q.off_cat), lds + q.off_flip, etab};
  const u128 inc = mk128(q.rng[2], q.rng[3]);
  const uint32_t G = gridDim.x;
  const uint32_t b2 = __hip_atomic_load(&g.rctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t r0 = 0, mdef = __hip_atomic_load(&g.rctl[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  u128 S = mk128(__hip_atomic_load(&q.rng[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                 __hip_atomic_load(&q.rng[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  // the barrier counter only grows: this launch's arrivals count from where the last launch left it
  const uint32_t bar0 = __hip_atomic_load(&g.rctl[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t flags = 0, bar = 0;
  __syncthreads();
  while (r0 < b2) {
    // evaluation: thread (block, t) -> lane L -> row i = L / RW_W, candidate j = L % RW_W
    for (uint32_t L = blockIdx.x * RW_TPB + t; L < (uint32_t)(RW_R * RW_W); L += G * RW_TPB) {
      const uint32_t i = L / RW_W, j = L % RW_W;
      uint32_t v = 0xFFFFu;
      if (r0 + i < b2) {
        const int64_t off = (int64_t)q.C0 * i - (int64_t)(rw_base(mdef, i) + (int32_t)j);
        if (off >= 0) {
          uint32_t used = 0;
          const uint32_t a = np_row(q, c, off ? pcg_jump(q.jt, S, (uint32_t)off) : S, inc, used, flags);
          v = (a << 16) | min(used, 0xFFFEu);
        }
      }
      g.rres[L] = v;
    }
    npg_grid_barrier(p, &g.rctl[0], bar0 + G * ++bar);
    if (blockIdx.x == 0) {  // the chain, RW_CHUNK rows at a time from LDS
      int32_t D = 0;
      uint32_t n = 0;
      bool go = true;
      while (go && n < (uint32_t)RW_R && r0 + n < b2) {
        const uint32_t rows = min(min((uint32_t)RW_CHUNK, (uint32_t)RW_R - n), b2 - r0 - n);
        for (uint32_t x = t; x < rows * RW_W; x += RW_TPB) res_lds[x] = g.rres[n * RW_W + x];
        __syncthreads();
        if (t == 0) {
          uint32_t k = 0;
          for (; k < rows; ++k) {
            const int32_t jj = D - rw_base(mdef, n + k);
            if (jj < 0 || jj >= RW_W) break;
            const uint32_t v = res_lds[k * RW_W + (uint32_t)jj];
            if ((v & 0xFFFFu) == 0xFFFFu) break;  // (not evaluated: cannot happen for a chained start)
            q.vrs[r0 + n + k] = (uint16_t)(v >> 16);
            D += q.C0 - (int32_t)(v & 0xFFFFu);
          }
          s_n = k;
          s_D = D;
        }
        __syncthreads();
        const uint32_t k = s_n;
        D = s_D;
        n += k;
        go = k == rows;
        __syncthreads();
      }
      if (t == 0) {
        const u128 S2 = pcg_jump(q.jt, S, (uint32_t)((int64_t)q.C0 * n - D));
        // the drift estimate for the next round: this round's mean deficit per row (x 256), kept when n is small
        uint32_t m2 = mdef;
        if (n >= 32) m2 = (uint32_t)max((int64_t)0, ((int64_t)D << 8) / (int64_t)n);
        g.rst[0] = hi64(S2);
        g.rst[1] = lo64(S2);
        g.rctl[2] = r0 + n;
        g.rctl[3] = m2;
      }
    }
    npg_grid_barrier(p, &g.rctl[0], bar0 + G * ++bar);
    if (t == 0) {
      s_r0 = __hip_atomic_load(&g.rctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_mdef = __hip_atomic_load(&g.rctl[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_S[0] = __hip_atomic_load(&g.rst[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_S[1] = __hip_atomic_load(&g.rst[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (s_r0 <= r0) {  // no progress: a logic error (row r0 is always chained); flag and stop
      if (t == 0 && blockIdx.x == 0) atomicOr(p.derr, GP_DERR_TIMEOUT);
      break;
    }
    r0 = s_r0;
    mdef = s_mdef;
    S = mk128(s_S[0], s_S[1]);
    __syncthreads();
  }
  if (flags) atomicOr(p.derr, flags);
  if (blockIdx.x == 0 && t == 0) {  // the stream after the rows (the 32-bit buffer is untouched: doubles only)
    q.rng[0] = hi64(S);
    q.rng[1] = lo64(S);
    g.rctl[5] = bar0 + G * bar;  // every block made the same `bar` arrivals: the next launch counts from here
  }
}

// The draws of one step (one workgroup of NP_TPB threads): tile prefixes, b1 / b2, then the p / d draws; the step's
// b2 for taxi_npg_rows.
__global__ __launch_bounds__(NP_TPB) void taxi_npg_draws(TaxiDev p, TaxiNpDev q, NpgDev g, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ NpShared sh;
  __shared__ uint64_t etab[256];
  __shared__ uint64_t wsum[NP_WAVES];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  {
    const uint4* s2 = (const uint4*)q.mtab;
    uint4* d2 = (uint4*)lds;
    for (int i = t; i < q.mtab_bytes / 16; i += NP_TPB) d2[i] = s2[i];
    for (int i = t; i < 256; i += NP_TPB) etab[i] = gp_libm::kExpTab[i];
    if (t == 0) {
      sh.S[0] = q.rng[0];
      sh.S[1] = q.rng[1];
      sh.has = (uint32_t)q.rng[4];
      sh.uval = (uint32_t)q.rng[5];
    }
  }
  // per-tile prefixes: thread t sums tiles [t * per, (t + 1) * per), a block scan, then the tiles' own
  const int per = (ntiles + NP_TPB - 1) / NP_TPB;
  uint64_t x = 0;
  for (int j = 0; j < per; ++j) {
    const int tl = t * per + j;
    if (tl < ntiles) {
      const uint32_t c = g.bcnt[tl];
      x += (uint64_t)(c & 0xFFFFu) | ((uint64_t)(c >> 16) << 32);
    }
  }
  uint64_t v = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(v, d, 64);
    if (lane >= d) v += y;
  }
  if (lane == 63) wsum[w] = v;
  __syncthreads();
  uint64_t base = 0, tot = 0;
  for (int i = 0; i < NP_WAVES; ++i) {
    base += i < w ? wsum[i] : 0ull;
    tot += wsum[i];
  }
  base += v - x;
  for (int j = 0; j < per; ++j) {
    const int tl = t * per + j;
    if (tl < ntiles) {
      g.bpre[tl] = base;
      const uint32_t c = g.bcnt[tl];
      base += (uint64_t)(c & 0xFFFFu) | ((uint64_t)(c >> 16) << 32);
    }
  }
  if (t == 0) {
    sh.b1 = (uint32_t)tot;
    sh.b2 = (uint32_t)(tot >> 32);
  }
  __syncthreads();
  const NpCats c{(const double*)(lds + q.off_pp), (const double*)(lds + q.off_q), (const double*)(lds + q.off_lq),
                 (const uint16_t*)(lds + q.off_cat), lds + q.off_flip, etab};
  np_draws(p, q, c, sh, false);  // the p / d draws; the rows are taxi_npg_rows's (after this launch)
  __syncthreads();
  if (t == 0) {
    q.rng[0] = sh.S[0];
    q.rng[1] = sh.S[1];
    q.rng[4] = sh.has;
    q.rng[5] = sh.uval;
    g.rctl[1] = sh.b2;
  }
}

// Pass 2 of step k: the draws applied, the observations (OH as taxi_rollout: 0 scalar, CS one-hot chunks).
template <int OH>
__global__ __launch_bounds__(TPB) void taxi_npg_pass2(TaxiDev p, TaxiNpDev q, NpgDev g, size_t off,
                                                      void* __restrict__ obs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  __shared__ uint16_t s_hot[WAVES][256];
  stage_tables(p, lds);
  __syncthreads();
  const int tile = blockIdx.x, env0 = tile * EPB + threadIdx.x * EPT;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t pre = g.bpre[tile];
  const uint32_t ptc = (uint32_t)pre, prs = (uint32_t)(pre >> 32);
  uint32_t u[4], rk[4], h[4];
  ld4_u32(p.st, env0, p.B, u);
  ld4_u32(reinterpret_cast<const uint32_t*>(q.rk), env0, p.B, rk);
  const uint16_t* obs_of = l_obs(lds, p);
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int32_t r = (int32_t)rk[i];
    if (env0 + i < p.B && r >= 0) {
      if (r & (1 << 30)) {
        u[i] = q.vrs[prs + (uint32_t)(r & ~(1 << 30))];  // _reset_mask: new start state, elapsed 0, dropoffs 0
      } else {
        const int32_t v = q.vtc[ptc + (uint32_t)r];  // encode(r, c, p, d): taxi cell kept
        const uint32_t s = u[i] & 0xFFFu;
        const uint32_t s2 = (s / (uint32_t)p.lpl) * (uint32_t)p.lpl + (uint32_t)(v >> 16) * (uint32_t)p.nlocs +
                            (uint32_t)(v & 0xFFFF);
        u[i] = (u[i] & ~0xFFFu) | s2;
      }
    }
    h[i] = obs_of[u[i] & 0xFFFu];
  }
  st4_u32(p.st, env0, p.B, u);
  if constexpr (OH == 0) {
    st4_u32(reinterpret_cast<uint32_t*>(obs) + off, env0, p.B, h);
  } else {
    const int we0 = tile * EPB + wid * 256;
    const int n = min(256, p.B - we0);
    if (n > 0)
      write_onehot_wave<OH>((uint8_t*)obs + (off + (size_t)we0) * (size_t)p.n_obs, n, p.n_obs, s_hot[wid], h, lane);
  }
}

// ------------------------------------------------------------------ host backend ----
struct TaxiBackend : EnvBackend {
  TaxiDev d{};
  int grid = 1;                 // persistent grid size (= metric slots)
  int one_hot = 0;
  uint64_t philox_step = 0;
  std::vector<double> law;      // P(start state = valid[k])
  DevBuf b_tabs, b_st, b_slot;
  DevErr derr;
  const int32_t* rp_state = nullptr;
  const int32_t* rp_pd = nullptr;

  // numpy mode (rng_mode GP_RNG_NUMPY): the reference's stream on the device
  TaxiNpDev np{};
  DevBuf b_rng, b_mtab, b_jrow, b_jt, b_rk, b_vtc, b_vrs;
  int np_build(const std::vector<uint16_t>& valid);
  int np_upload_rng() {
    GP_HIP_CHECK(hipDeviceSynchronize());
    const uint64_t r6[6] = {hi64(rng.state), lo64(rng.state), hi64(rng.inc), lo64(rng.inc), rng.has_u32, rng.uinteger};
    GP_HIP_CHECK(hipMemcpy(b_rng.p, r6, sizeof(r6), hipMemcpyHostToDevice));
    const std::vector<PcgJump> jt = build_jump_tables(rng.inc);
    GP_HIP_CHECK(hipMemcpy(b_jt.p, jt.data(), jt.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
    std::vector<PcgJump> jr(NP_TPB);
    for (int t = 0; t < NP_TPB; ++t) {
      const int64_t delta = (int64_t)np.C0 * (t / SPEC_DEF) - t % SPEC_DEF;  // negative: never chained
      jr[t] = pcg_jump_params((u128)(delta > 0 ? delta : 0), rng.inc);
    }
    GP_HIP_CHECK(hipMemcpy(b_jrow.p, jr.data(), jr.size() * sizeof(PcgJump), hipMemcpyHostToDevice));
    return GP_OK;
  }

  int build(const gp_taxi_config* cfg);
  int seed(const RngHost& r, const uint32_t key[2]) override {
    rng = r;
    philox_key[0] = key[0];
    philox_key[1] = key[1];
    d.key0 = key[0];
    d.key1 = key[1];
    philox_step = 0;
    if (rng_mode == GP_RNG_NUMPY)
      if (int e = np_upload_rng()) return e;
    return derr.clear();
  }
  int check() override { return derr.check("taxi"); }
  int set_rng_state(const RngHost& r) override {
    if (rng_mode != GP_RNG_NUMPY) {
      gp_set_error("taxi: the PCG64 stream is used on the device only with rng_mode numpy");
      return GP_E_UNSUPPORTED;
    }
    rng = r;
    return np_upload_rng();
  }
  int get_rng_state(RngHost* r) override {
    if (rng_mode != GP_RNG_NUMPY) {
      gp_set_error("taxi: the PCG64 stream is used on the device only with rng_mode numpy");
      return GP_E_UNSUPPORTED;
    }
    GP_HIP_CHECK(hipDeviceSynchronize());
    uint64_t r6[6];
    GP_HIP_CHECK(hipMemcpy(r6, b_rng.p, sizeof(r6), hipMemcpyDeviceToHost));
    r->state = mk128(r6[0], r6[1]);
    r->inc = mk128(r6[2], r6[3]);
    r->has_u32 = (uint32_t)r6[4];
    r->uinteger = (uint32_t)r6[5];
    return check();
  }
  // grid-wide numpy mode (B > npg_min): per step pass 1, the draws, pass 2 (K = 0: reset())
  NpgDev npg{};
  DevBuf b_bcnt, b_bpre, b_rres, b_rctl, b_rst;
  size_t rows_lds() const { return (size_t)((np.mtab_bytes + 15) & ~15) + (size_t)RW_CHUNK * RW_W * 4; }
  int npg_min = NPG_MIN_ENVS;
  template <int OH>
  void launch_npg_pass2(size_t off, void* obs, hipStream_t s) {
    hipLaunchKernelGGL((taxi_npg_pass2<OH>), dim3((unsigned)d.ntiles), dim3(TPB), (size_t)d.tab_bytes, s, d, np, npg,
                       off, obs);
  }
  void launch_npg(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) {
    const int cs = one_hot ? chunk_size(obs, K > 0 ? K : 1) : 0;
    for (int k = 0; k < (K > 0 ? K : 1); ++k) {
      const size_t off = (size_t)k * (size_t)B;
      if (K == 0)
        hipLaunchKernelGGL((taxi_npg_pass1<true>), dim3((unsigned)d.ntiles), dim3(TPB), (size_t)d.tab_bytes, s, d, np,
                           npg, off, (const int32_t*)act, rew, term, trunc);
      else
        hipLaunchKernelGGL((taxi_npg_pass1<false>), dim3((unsigned)d.ntiles), dim3(TPB), (size_t)d.tab_bytes, s, d, np,
                           npg, off, (const int32_t*)act, rew, term, trunc);
      hipLaunchKernelGGL(taxi_npg_draws, dim3(1), dim3(NP_TPB), (size_t)np.mtab_bytes, s, d, np, npg, d.ntiles);
      hipLaunchKernelGGL(taxi_npg_rows, dim3((unsigned)npg.rgrid), dim3(RW_TPB), rows_lds(), s, d, np, npg);
      switch (cs) {
        case 0: launch_npg_pass2<0>(off, obs, s); break;
        case 16: launch_npg_pass2<16>(off, obs, s); break;
        case 4: launch_npg_pass2<4>(off, obs, s); break;
        default: launch_npg_pass2<1>(off, obs, s); break;
      }
    }
  }
  void launch_np(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) {
    if (B > npg_min) {
      launch_npg(K, act, obs, rew, term, trunc, s);
      return;
    }
    const size_t lds = (size_t)d.tab_bytes + (size_t)np.mtab_bytes;
    if (one_hot)
      hipLaunchKernelGGL((taxi_np_kernel<true>), dim3(1), dim3(NP_TPB), lds, s, d, np, K, (const int32_t*)act, obs,
                         rew, term, trunc);
    else
      hipLaunchKernelGGL((taxi_np_kernel<false>), dim3(1), dim3(NP_TPB), lds, s, d, np, K, (const int32_t*)act, obs,
                         rew, term, trunc);
  }
  // Largest chunk size the one-hot stream may use for these buffers.
  int chunk_size(const void* obs, int K) const {
    for (int cs : {16, 4}) {
      if (d.n_obs % cs) continue;
      if (((uintptr_t)obs) % cs) continue;
      if (K > 1 && ((size_t)B * d.n_obs) % cs) continue;
      return cs;
    }
    return 1;
  }
  TaxiDev dev_for_launch() const {
    TaxiDev dd = d;
    dd.rp_state = rp_state;
    dd.rp_pd = rp_pd;
    return dd;
  }
  template <bool REPLAY>
  void launch_rollout(int cs, int K, uint64_t step0, const void* act, void* obs, float* rew, uint8_t* term,
                      uint8_t* trunc, hipStream_t s) {
    const TaxiDev dd = dev_for_launch();
    const dim3 g((unsigned)grid), b(TPB);
    const size_t lds = (size_t)d.tab_bytes;
    const int32_t* a = (const int32_t*)act;
    if (!one_hot)
      hipLaunchKernelGGL((taxi_rollout<0, REPLAY>), g, b, lds, s, dd, K, step0, a, obs, rew, term, trunc);
    else if (cs == 16)
      hipLaunchKernelGGL((taxi_rollout<16, REPLAY>), g, b, lds, s, dd, K, step0, a, obs, rew, term, trunc);
    else if (cs == 4)
      hipLaunchKernelGGL((taxi_rollout<4, REPLAY>), g, b, lds, s, dd, K, step0, a, obs, rew, term, trunc);
    else
      hipLaunchKernelGGL((taxi_rollout<1, REPLAY>), g, b, lds, s, dd, K, step0, a, obs, rew, term, trunc);
  }
  template <bool REPLAY>
  void launch_reset(int cs, uint64_t step, void* obs, hipStream_t s) {
    const TaxiDev dd = dev_for_launch();
    const dim3 g((unsigned)grid), b(TPB);
    const size_t lds = (size_t)d.tab_bytes;
    if (!one_hot) hipLaunchKernelGGL((taxi_reset<0, REPLAY>), g, b, lds, s, dd, step, obs);
    else if (cs == 16) hipLaunchKernelGGL((taxi_reset<16, REPLAY>), g, b, lds, s, dd, step, obs);
    else if (cs == 4) hipLaunchKernelGGL((taxi_reset<4, REPLAY>), g, b, lds, s, dd, step, obs);
    else hipLaunchKernelGGL((taxi_reset<1, REPLAY>), g, b, lds, s, dd, step, obs);
  }
  int reset(void* obs, hipStream_t s) override {
    GP_HIP_CHECK(hipMemsetAsync(d.mslot, 0, sizeof(TaxiSlot) * grid, s));
    const int cs = chunk_size(obs, 1);
    if (rng_mode == GP_RNG_NUMPY) {
      launch_np(0, nullptr, obs, nullptr, nullptr, nullptr, s);
    } else if (rng_mode == GP_RNG_REPLAY) {
      if (!rp_state) {
        gp_set_error("taxi replay reset needs reset states (gp_set_replay i0)");
        return GP_E_STATE;
      }
      launch_reset<true>(cs, 0, obs, s);
    } else {
      launch_reset<false>(cs, philox_step, obs, s);
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
    if (rng_mode == GP_RNG_REPLAY) {
      if (!rp_state || (d.num_passengers > 1 && !rp_pd)) {
        gp_set_error("taxi replay step needs reset states (i0) and, with num_passengers > 1, p/d pairs (i1)");
        return GP_E_STATE;
      }
      if (K > 1) return EnvBackend::rollout(K, act, obs, rew, term, trunc, s);  // one draw set per step
    }
    const int cs = chunk_size(obs, K);
    timer.begin(s);
    if (rng_mode == GP_RNG_NUMPY) launch_np(K, act, obs, rew, term, trunc, s);
    else if (rng_mode == GP_RNG_REPLAY) launch_rollout<true>(cs, K, 0, act, obs, rew, term, trunc, s);
    else launch_rollout<false>(cs, K, philox_step, act, obs, rew, term, trunc, s);
    timer.end(s);
    GP_HIP_CHECK(hipGetLastError());
    if (rng_mode != GP_RNG_REPLAY) philox_step += (uint64_t)K;
    return GP_OK;
  }
  int step(const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) override {
    return rollout(1, act, obs, rew, term, trunc, s);
  }
  int get_state(void* a, void* b, void* c, void* dd, hipStream_t s) override {
    hipLaunchKernelGGL(taxi_get_state, dim3((unsigned)((B + TPB - 1) / TPB)), dim3(TPB), 0, s, d, (int32_t*)a,
                       (int32_t*)b, (int32_t*)c);
    GP_HIP_CHECK(hipGetLastError());
    return GP_OK;
  }
  int set_state(const void* a, const void* b, const void* c, const void* dd, hipStream_t s) override {
    hipLaunchKernelGGL(taxi_set_state, dim3((unsigned)((B + TPB - 1) / TPB)), dim3(TPB), 0, s, d,
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
    rp_state = (const int32_t*)i0;
    rp_pd = (const int32_t*)i1;
    return GP_OK;
  }
  int metrics(double out[4]) override {
    GP_HIP_CHECK(hipDeviceSynchronize());
    std::vector<TaxiSlot> m(grid);
    GP_HIP_CHECK(hipMemcpy(m.data(), d.mslot, sizeof(TaxiSlot) * grid, hipMemcpyDeviceToHost));
    out[0] = out[1] = out[2] = out[3] = 0;
    for (const TaxiSlot& x : m) {
      out[0] += (double)x.episodes;
      out[1] += x.return_sum;
      out[2] += (double)x.length_sum;
      out[3] += (double)x.env_steps;
    }
    return check();
  }
  int reset_distribution(double* out, int cap) const override {
    for (int k = 0; k < (int)law.size() && k < cap; ++k) out[k] = law[k];
    return (int)law.size();
  }
  // rendering: bordered map + location coordinates on the device
  DevBuf b_rdesc, b_rlocs;
  int rDR = 0, rDC = 0, rC = 0, rpseudo = 0;
  int render(int n, int hansen, uint8_t* out, int32_t dims[4], hipStream_t s) override {
    if (n < 1 || n > B || n > 65536) {
      gp_set_error("taxi render: n=%d outside [1, min(num_envs, 65536)]", n);
      return GP_E_INVALID;
    }
    const int TH = (int)std::ceil(std::sqrt((double)n)), TW = (int)std::ceil((double)n / TH);  // tile_images
    dims[0] = TH * rDR;
    dims[1] = TW * rDC;
    dims[2] = rDR;
    dims[3] = rDC;
    if (!out) return GP_OK;
    TaxiRender p{d.st, b_rdesc.as<uint8_t>(), b_rlocs.as<int32_t>(), rDR, rDC, rC, d.nlocs, rpseudo, n, TW,
                 dims[0], dims[1], hansen != 0};
    const int npix = dims[0] * dims[1];
    hipLaunchKernelGGL(taxi_render_kernel, dim3((npix + TPB - 1) / TPB), dim3(TPB), 0, s, p, out);
    GP_HIP_CHECK(hipGetLastError());
    return GP_OK;
  }
};

int TaxiBackend::build(const gp_taxi_config* cfg) {
  const int R = cfg->rows, C = cfg->cols, L = cfg->n_locs;
  const int DR = cfg->desc_rows, DC = cfg->desc_cols;
  if (R < 1 || C < 1 || L < 1 || !cfg->desc || !cfg->locs) {
    gp_set_error("taxi: bad map (rows=%d cols=%d n_locs=%d)", R, C, L);
    return GP_E_INVALID;
  }
  const bool pseudo = cfg->pseudo_walls != 0;
  if (DR != R + 2 || DC != (pseudo ? 2 * C + 1 : C + 2)) {
    gp_set_error("taxi: desc %dx%d does not border a %dx%d grid", DR, DC, R, C);
    return GP_E_INVALID;
  }
  const int ns = R * C * L * (L + 1);
  if (ns > MAX_NS) {
    gp_set_error("taxi: %d states exceed the packed-state limit %d", ns, MAX_NS);
    return GP_E_INVALID;
  }
  if (cfg->num_passengers < 0 || cfg->num_passengers > 15) {
    gp_set_error("taxi: num_passengers %d outside [0, 15]", cfg->num_passengers);
    return GP_E_INVALID;
  }
  if (cfg->num_passengers > 1 && L < 2) {
    gp_set_error("taxi: num_passengers > 1 needs >= 2 locations (the reference's d != p loop never ends)");
    return GP_E_INVALID;
  }
  if (cfg->time_limit < 0 || cfg->time_limit > 65534) {
    gp_set_error("taxi: time_limit %d outside [0, 65534]", cfg->time_limit);
    return GP_E_INVALID;
  }
  if (cfg->obs_kind != GP_OBS_TABLE && cfg->obs_kind != GP_OBS_HANSEN) {
    gp_set_error("taxi: obs_kind must be GP_OBS_TABLE (state) or GP_OBS_HANSEN");
    return GP_E_INVALID;
  }
  auto desc = [&](int r, int c) { return cfg->desc[(size_t)r * DC + c]; };
  auto cc_r = [&](int r) { return r + 1; };
  auto cc_c = [&](int c) { return pseudo ? 2 * c + 1 : c + 1; };
  std::vector<int> loc_r(L + 1), loc_c(L + 1);
  for (int i = 0; i < L; ++i) {
    loc_r[i] = cfg->locs[2 * i];
    loc_c[i] = cfg->locs[2 * i + 1];
  }
  loc_r[L] = loc_c[L] = -1;  // extraneous "in taxi" location (extended_taxi.py:185)
  auto encode = [&](int r, int c, int p, int dd) { return ((r * C + c) * (L + 1) + p) * L + dd; };
  // generate_hansen_map (extended_taxi.py:102-114): N=1, S=2, W=4, E=8
  std::vector<int> hansen((size_t)R * C);
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < C; ++c) {
      const int br = cc_r(r), bc = cc_c(c);
      hansen[(size_t)r * C + c] = (desc(br - 1, bc) == '|') + 2 * (desc(br + 1, bc) == '|') +
                                  4 * (desc(br, bc - 1) == '|') + 8 * (desc(br, bc + 1) == '|');
    }
  static const int AY[NACT] = {-1, 1, 0, 0, 0}, AX[NACT] = {0, 0, -1, 1, 0};
  std::vector<uint16_t> trans((size_t)ns * TCOL), obs_of(ns);
  for (int s = 0; s < ns; ++s) {
    const int dd = s % L, t1 = s / L, p = t1 % (L + 1), t2 = t1 / (L + 1), c = t2 % C, r = t2 / C;
    obs_of[s] = (uint16_t)(cfg->obs_kind == GP_OBS_HANSEN ? (hansen[(size_t)r * C + c] * (L + 1) + p) * L + dd : s);
    for (int a = 0; a < NACT; ++a) {
      // extended_taxi.py:248-260
      const int rn = std::min(std::max(r + AY[a], 0), R - 1), cn = std::min(std::max(c + AX[a], 0), C - 1);
      const int br = cc_r(rn), bc = cc_c(cn);
      bool ok = desc(br, bc) != '|';
      if (AX[a] != 0 && desc(br, bc - AX[a]) == '|') ok = false;
      const int r2 = ok ? rn : r, c2 = ok ? cn : c;
      // extended_taxi.py:262-275 (goal evaluated on the pre-update p; a dropoff keeps p)
      int p2 = p, goal = 0, bad = 0;
      if (a == 4) {
        goal = (p == L) && loc_r[dd] == r2 && loc_c[dd] == c2;
        const int pick = (p < L) && loc_r[p] == r2 && loc_c[p] == c2;
        if (pick) p2 = L;
        bad = !goal && !pick;
      }
      trans[(size_t)s * TCOL + a] = (uint16_t)(encode(r2, c2, p2, dd) | (goal << 12) | (bad << 13));
    }
    trans[(size_t)s * TCOL + NACT] = (uint16_t)s;  // action -1: ACTIONS_YX[-1] = (0,0), not a pickup/dropoff
  }
  // valid start states (extended_taxi.py:208-218), ascending, and the argmax-multinomial law
  std::vector<uint16_t> valid;
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < C; ++c) {
      const char g = desc(cc_r(r), cc_c(c));
      if (g == '|') continue;
      for (int p = 0; p < L; ++p)
        for (int dd = 0; dd < L; ++dd)
          if (dd != p) valid.push_back((uint16_t)encode(r, c, p, dd));
    }
  if (valid.empty()) {
    gp_set_error("taxi: no valid start state");
    return GP_E_INVALID;
  }
  const int V = (int)valid.size();
  law = argmax_multinomial_distribution(V, ns);
  long double tot = 0.0L;
  for (double v : law) tot += v;
  std::vector<uint64_t> cdf(V);
  long double acc = 0.0L;
  const long double two64 = 18446744073709551616.0L;
  for (int k = 0; k < V; ++k) {
    acc += law[k];
    const long double x = acc / tot * two64;
    cdf[k] = (k == V - 1 || x >= two64) ? ~0ull : (uint64_t)x;
  }
  // pack: trans | obs_of | cdf | valid, each 16-B aligned
  auto al16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const size_t o_trans = 0, o_obs = al16(o_trans + trans.size() * 2), o_cdf = al16(o_obs + obs_of.size() * 2),
               o_valid = al16(o_cdf + cdf.size() * 8), total = al16(o_valid + valid.size() * 2);
  std::vector<uint8_t> blob(total, 0);
  memcpy(blob.data() + o_trans, trans.data(), trans.size() * 2);
  memcpy(blob.data() + o_obs, obs_of.data(), obs_of.size() * 2);
  memcpy(blob.data() + o_cdf, cdf.data(), cdf.size() * 8);
  memcpy(blob.data() + o_valid, valid.data(), valid.size() * 2);
  if (int e = b_tabs.upload(blob)) return e;
  d.tabs = b_tabs.as<uint8_t>();
  d.off_trans = (int)o_trans;
  d.off_obs = (int)o_obs;
  d.off_cdf = (int)o_cdf;
  d.off_valid = (int)o_valid;
  d.tab_bytes = (int)total;

  d.B = (int32_t)B;
  d.ntiles = (int32_t)((B + EPB - 1) / EPB);
  d.ns = ns;
  d.nlocs = L;
  d.lpl = L * (L + 1);
  d.n_valid = V;
  d.num_passengers = cfg->num_passengers;
  d.time_limit = cfg->time_limit;
  d.n_obs = cfg->obs_kind == GP_OBS_HANSEN ? 16 * L * (L + 1) : ns;  // compute_obs_space (:72-81)
  d.r_goal = cfg->reward_goal;
  d.r_bad = cfg->reward_bad;
  d.r_any = cfg->reward_any;
  one_hot = cfg->one_hot != 0;
  obs_dtype = one_hot ? GP_DTYPE_U8 : GP_DTYPE_I32;
  obs_width = one_hot ? d.n_obs : 1;

  {  // render tables: the bordered map and each location's bordered (row, col)
    std::vector<uint8_t> rd((size_t)DR * DC);
    for (int r = 0; r < DR; ++r)
      for (int c = 0; c < DC; ++c) rd[(size_t)r * DC + c] = (uint8_t)desc(r, c);
    std::vector<int32_t> rl(2 * L);
    for (int i = 0; i < L; ++i) {
      rl[2 * i] = cc_r(loc_r[i]);
      rl[2 * i + 1] = cc_c(loc_c[i]);
    }
    if (int e = b_rdesc.upload(rd)) return e;
    if (int e = b_rlocs.upload(rl)) return e;
    rDR = DR;
    rDC = DC;
    rC = C;
    rpseudo = pseudo ? 1 : 0;
  }
  if (int e = b_st.alloc((size_t)B * 4 + 16)) return e;
  d.st = b_st.as<uint32_t>();
  // persistent grid: as many blocks as are co-resident, capped by the number of tiles
  hipDeviceProp_t prop;
  GP_HIP_CHECK(hipGetDeviceProperties(&prop, device));
  int occ = 0;
  GP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, taxi_rollout<16, false>, TPB, d.tab_bytes));
  grid = persistent_grid(d.ntiles, prop.multiProcessorCount, occ);
  persist_grid = grid;
  persist_occ = occ;
  if (int e = b_slot.alloc(sizeof(TaxiSlot) * grid)) return e;
  d.mslot = b_slot.as<TaxiSlot>();
  if (int e = derr.alloc()) return e;
  d.derr = derr.ptr();
  if (d.tab_bytes > 64 * 1024) {
    gp_set_error("taxi: tables (%d B) exceed the LDS budget", d.tab_bytes);
    return GP_E_INVALID;
  }
  if (rng_mode == GP_RNG_NUMPY)
    if (int e = np_build(valid)) return e;
  return GP_OK;
}

// numpy mode: random_multinomial's per-category constants for pvals = state_distribution (1/V on the valid states,
// extended_taxi.py:205-218). Category j < ns - 1 with pix_j > 0 draws random_binomial(pix_j / remaining_p, dn);
// remaining_p -= pix_j after each (zeros change nothing). The flip and q = 1 - p are random_binomial's, log q is
// the C library's (random_binomial_inversion: qn = exp(n * log(q))).
int TaxiBackend::np_build(const std::vector<uint16_t>& valid) {
  const int ns = d.ns, V = (int)valid.size();
  const double pix = 1.0 / (double)V;  // state_distribution[valid] += 1; /= sum (exactly V)
  std::vector<double> pp, qv, lq;
  std::vector<uint16_t> cat;
  std::vector<uint8_t> flip;
  double rem = 1.0;
  size_t vi = 0;
  for (int j = 0; j + 1 < ns; ++j) {
    const bool isv = vi < valid.size() && valid[vi] == j;
    if (isv) {
      ++vi;
      const double p = pix / rem;
      const bool fl = p > 0.5;
      const double pb = fl ? 1.0 - p : p;
      pp.push_back(pb);
      qv.push_back(1.0 - pb);
      lq.push_back(std::log(1.0 - pb));
      cat.push_back((uint16_t)j);
      flip.push_back(fl ? 1 : 0);
      rem -= pix;
    }
  }
  const int C0 = (int)pp.size();
  if (C0 < 1) {
    gp_set_error("taxi numpy mode: no category to draw");
    return GP_E_INVALID;
  }
  auto al16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const size_t o_pp = 0, o_q = al16(o_pp + 8 * (size_t)C0), o_lq = al16(o_q + 8 * (size_t)C0),
               o_cat = al16(o_lq + 8 * (size_t)C0), o_flip = al16(o_cat + 2 * (size_t)C0), tot = al16(o_flip + C0);
  if ((size_t)d.tab_bytes + tot > 96 * 1024) {
    gp_set_error("taxi numpy mode: tables (%zu B) exceed the LDS budget", (size_t)d.tab_bytes + tot);
    return GP_E_INVALID;
  }
  std::vector<uint8_t> blob(tot, 0);
  memcpy(blob.data() + o_pp, pp.data(), 8 * (size_t)C0);
  memcpy(blob.data() + o_q, qv.data(), 8 * (size_t)C0);
  memcpy(blob.data() + o_lq, lq.data(), 8 * (size_t)C0);
  memcpy(blob.data() + o_cat, cat.data(), 2 * (size_t)C0);
  memcpy(blob.data() + o_flip, flip.data(), (size_t)C0);
  int e;
  if ((e = b_mtab.upload(blob)) || (e = b_rng.alloc(64)) || (e = b_jrow.alloc(sizeof(PcgJump) * NP_TPB)) ||
      (e = b_jt.alloc(sizeof(PcgJump) * JT_LEVELS * JT_RADIX)) || (e = b_rk.alloc((size_t)B * 4 + 16)) ||
      (e = b_vtc.alloc((size_t)B * 4 + 16)) || (e = b_vrs.alloc((size_t)B * 2 + 16)))
    return e;
  np.rng = b_rng.as<uint64_t>();
  np.mtab = b_mtab.as<uint8_t>();
  np.off_pp = (int)o_pp;
  np.off_q = (int)o_q;
  np.off_lq = (int)o_lq;
  np.off_cat = (int)o_cat;
  np.off_flip = (int)o_flip;
  np.mtab_bytes = (int)tot;
  np.C0 = C0;
  np.n = ns;
  np.last = ns - 1;
  np.jrow = b_jrow.as<PcgJump>();
  np.jt = b_jt.as<PcgJump>();
  np.rk = b_rk.as<int32_t>();
  np.vtc = b_vtc.as<int32_t>();
  np.vrs = b_vrs.as<uint16_t>();
  if (gp_debug_knobs().taxi_npg_min >= 0) npg_min = gp_debug_knobs().taxi_npg_min;
  if ((e = b_bcnt.alloc(sizeof(uint32_t) * (size_t)d.ntiles + 16)) ||
      (e = b_bpre.alloc(sizeof(uint64_t) * (size_t)d.ntiles + 16)))
    return e;
  npg.bcnt = b_bcnt.as<uint32_t>();
  npg.bpre = b_bpre.as<uint64_t>();
  npg.grid = grid;
  // the grid-wide rows: one block per CU, all resident (its barrier waits on every block)
  if ((e = b_rres.alloc(sizeof(uint32_t) * RW_R * RW_W)) || (e = b_rctl.alloc(sizeof(uint32_t) * 16)) ||
      (e = b_rst.alloc(sizeof(uint64_t) * 2)))
    return e;
  npg.rres = b_rres.as<uint32_t>();
  npg.rctl = b_rctl.as<uint32_t>();
  npg.rst = b_rst.as<uint64_t>();
  {
    const uint32_t m0 = 64;  // the drift's first estimate: 0.25 doubles per row (x 256); each round re-measures it
    GP_HIP_CHECK(hipMemcpy(npg.rctl + 3, &m0, sizeof(m0), hipMemcpyHostToDevice));
    int cus = 0, occ = 0;
    GP_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    GP_HIP_CHECK(hipFuncSetAttribute((const void*)taxi_npg_rows, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)rows_lds()));
    GP_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, taxi_npg_rows, RW_TPB, rows_lds()));
    if (occ < 1) {
      gp_set_error("taxi: the grid-wide row kernel does not fit a CU (%zu B of LDS)", rows_lds());
      return GP_E_UNSUPPORTED;
    }
    npg.rgrid = cus;
  }
  return np_upload_rng();
}

}  // namespace

std::unique_ptr<EnvBackend> make_taxi_backend(const gp_taxi_config* cfg, int64_t B, int device, int rng_mode,
                                              int* err) {
  if (B < 1 || B > (int64_t)1 << 30) {
    gp_set_error("taxi: num_envs %lld out of range", (long long)B);
    *err = GP_E_INVALID;
    return nullptr;
  }
  auto be = std::make_unique<TaxiBackend>();
  be->B = B;
  be->device = device;
  be->rng_mode = rng_mode;
  if (hipSetDevice(device) != hipSuccess) {
    gp_set_error("taxi: hipSetDevice(%d) failed", device);
    *err = GP_E_HIP;
    return nullptr;
  }
  int e = be->build(cfg);
  if (e) {
    *err = e;
    return nullptr;
  }
  if (rng_mode == GP_RNG_NUMPY) {  // numpy's q^n = exp(n log q) from the host's libm build
    const int fma = gp_exp_host_variant() == 0 ? 0 : 1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_taxi_exp_fma), &fma, sizeof(fma)) != hipSuccess) {
      gp_set_error("taxi: hipMemcpyToSymbol(exp variant) failed");
      *err = GP_E_HIP;
      return nullptr;
    }
  }
  return be;
}

// ------------------------------------------------------------------ C ABI: resize ----
// OpenCV resizeGeneric_ coefficient setup for INTER_AREA outside decimation (resize.cpp: sx = floor(dx*scale),
// fx = (float)((dx+1) - (sx+1)*inv_scale), fx = fx <= 0 ? 0 : fx - floor(fx); alpha = saturate_cast<short>
// (c * 2048)); `clamp`: the horizontal setup pins the last source column.
static void area_coeffs(int ssize, int dsize, bool clamp, std::vector<int32_t>& ofs, std::vector<int16_t>& a) {
#pragma clang fp contract(off)
  const double inv_scale = (double)dsize / ssize, scale = 1. / inv_scale;
  ofs.resize(dsize);
  a.resize(2 * (size_t)dsize);
  for (int dx = 0; dx < dsize; ++dx) {
    int sx = (int)std::floor(dx * scale);
    float fx = (float)((dx + 1) - (sx + 1) * inv_scale);
    fx = fx <= 0 ? 0.f : fx - (float)std::floor(fx);
    if (clamp && sx >= ssize - 1) {
      fx = 0.f;
      sx = ssize - 1;
    }
    ofs[dx] = sx;
    a[2 * dx] = (int16_t)std::lrint((1.f - fx) * 2048.f);
    a[2 * dx + 1] = (int16_t)std::lrint(fx * 2048.f);
  }
}

extern "C" int gp_resize_area_u8(const uint8_t* src, int sh, int sw, int ch, uint8_t* dst, int dh, int dw,
                                 int dst_pitch, void* stream) {
  if (!src || !dst || sh < 1 || sw < 1 || ch < 1 || ch > 4 || dh < 1 || dw < 1 || dst_pitch < dw * ch) {
    gp_set_error("gp_resize_area_u8: bad arguments");
    return GP_E_INVALID;
  }
  if (dh <= sh && dw <= sw && !(dh == sh && dw == sw)) {
    gp_set_error("gp_resize_area_u8: INTER_AREA decimation (both axes shrink) is not implemented");
    return GP_E_UNSUPPORTED;
  }
  std::vector<int32_t> xo, yo;
  std::vector<int16_t> xa, yb;
  area_coeffs(sw, dw, true, xo, xa);
  area_coeffs(sh, dh, false, yo, yb);
  DevBuf bx, bxa, by, byb;
  if (int e = bx.upload(xo)) return e;
  if (int e = bxa.upload(xa)) return e;
  if (int e = by.upload(yo)) return e;
  if (int e = byb.upload(yb)) return e;
  const hipStream_t s = (hipStream_t)stream;
  ResizeArea p{src, bx.as<int32_t>(), bxa.as<int16_t>(), by.as<int32_t>(), byb.as<int16_t>(), sh, sw, ch, dh, dw,
               dst_pitch};
  const int n = dh * dw * ch;
  hipLaunchKernelGGL(resize_area_kernel, dim3((n + TPB - 1) / TPB), dim3(TPB), 0, s, p, dst);
  GP_HIP_CHECK(hipGetLastError());
  GP_HIP_CHECK(hipStreamSynchronize(s));  // the coefficient buffers are freed on return
  return GP_OK;
}
