// Launch-footprint probe: what a launch with the headline kernel's footprint costs when the
// kernel does (almost) nothing, beside the real wgrid_rollout<8,4> at K = 1 / 20 in the same process
// (tools/launch_floor.py drives it; built by that script with hipcc -shared).
//
// Variants (all 52-B kernel arguments: a pointer, an int and five pointers, like wgrid_rollout):
//   0 trivial     256 x 64 threads, no LDS, few registers
//   1 footprint   G x 704 threads, `lds` bytes of dynamic LDS, 155 VGPRs / 100 SGPRs pinned (asm clobbers)
//   2 + outputs   as 1, and every env lane writes one step of outputs (obs i32, reward f32, term u8, trunc u8 for
//                 E envs per block) with non-temporal stores, as the launch's last step does (dirty lines at the end)
//   3 + wt out    as 2 with write-through (sc1) stores
//   4 + tables    as 1, and the control / store waves copy `tab` bytes of a device image into LDS (the table staging)
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int TPB = 704;

__device__ __forceinline__ void pin_regs() {
  asm volatile("" ::: "v154", "s99");
}

__global__ __launch_bounds__(64) void lf_trivial(const void* P, int K, const int32_t* act, int32_t* obs, float* rew,
                                                 uint8_t* term, uint8_t* trunc) {
  if (K == -12345 && threadIdx.x == 0) obs[blockIdx.x] = act[0];
}

template <int MODE>
__global__ __launch_bounds__(TPB) void lf_footprint(const void* P, int K, const int32_t* act, int32_t* obs, float* rew,
                                                    uint8_t* term, uint8_t* trunc) {
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  pin_regs();
  const int tid = threadIdx.x, wid = tid >> 6;
  if constexpr (MODE == 4) {  // table staging: waves 8..10 copy K bytes of the image P into LDS
    if (wid >= 8) {
      const uint4* s = reinterpret_cast<const uint4*>(P);
      uint4* d = reinterpret_cast<uint4*>(dyn);
      for (int i = tid - 512; i < (K >> 4); i += 192) d[i] = s[i];
    }
    __syncthreads();
    if (tid == 0 && dyn[1] == 123 && dyn[7] == 45) obs[blockIdx.x] = 1;
  } else if constexpr (MODE == 2 || MODE == 3) {  // one step of outputs from the env lanes (8 slots x 512 lanes)
    if (wid < 8) {
      const size_t e0 = (size_t)blockIdx.x * 4096;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const size_t e = e0 + (size_t)s * 512 + tid;
        const int32_t o = (int32_t)(e * 2654435761u);
        if constexpr (MODE == 2) {
          __builtin_nontemporal_store(o, obs + e);
          __builtin_nontemporal_store(-1.0f, rew + e);
          __builtin_nontemporal_store((uint8_t)(o & 1), term + e);
          __builtin_nontemporal_store((uint8_t)((o >> 1) & 1), trunc + e);
        } else {
          __hip_atomic_store(obs + e, o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(reinterpret_cast<uint32_t*>(rew) + e, 0xBF800000u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(term + e, (uint8_t)(o & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(trunc + e, (uint8_t)((o >> 1) & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  } else {
    if (K == -12345 && tid == 0) obs[blockIdx.x] = act[0] + (int)dyn[tid];
  }
}
}  // namespace

extern "C" {
// Allow `lds` bytes of dynamic LDS for every variant; returns hipError_t.
int lf_setup(int lds) {
  int e = 0;
  e |= (int)hipFuncSetAttribute((const void*)lf_footprint<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  e |= (int)hipFuncSetAttribute((const void*)lf_footprint<2>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  e |= (int)hipFuncSetAttribute((const void*)lf_footprint<3>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  e |= (int)hipFuncSetAttribute((const void*)lf_footprint<4>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  return e;
}
// One launch of variant v on `stream` (a hipStream_t). G blocks; P / K: the table image and its bytes (variant 4).
int lf_launch(int v, int G, int lds, void* stream, const void* P, int K, const int32_t* act, int32_t* obs, float* rew,
              uint8_t* term, uint8_t* trunc) {
  hipStream_t s = (hipStream_t)stream;
  switch (v) {
    case 0: hipLaunchKernelGGL(lf_trivial, dim3(256), dim3(64), 0, s, P, K, act, obs, rew, term, trunc); break;
    case 1: hipLaunchKernelGGL(lf_footprint<1>, dim3(G), dim3(TPB), lds, s, P, K, act, obs, rew, term, trunc); break;
    case 2: hipLaunchKernelGGL(lf_footprint<2>, dim3(G), dim3(TPB), lds, s, P, K, act, obs, rew, term, trunc); break;
    case 3: hipLaunchKernelGGL(lf_footprint<3>, dim3(G), dim3(TPB), lds, s, P, K, act, obs, rew, term, trunc); break;
    case 4: hipLaunchKernelGGL(lf_footprint<4>, dim3(G), dim3(TPB), lds, s, P, K, act, obs, rew, term, trunc); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
}
