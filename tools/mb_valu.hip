// Issue cost of the integer VALU instructions the PCG64 arithmetic is made of, on gfx950:
// v_mad_u64_u32, v_mul_lo_u32, v_mul_hi_u32, v_add_u32, v_mul_u32_u24 (8 independent chains per lane,
// 1 or 2 waves per SIMD, cycles from s_memtime per wave).
//   hipcc --offload-arch=gfx950 -O3 tools/mb_valu.hip -o /tmp/mb_valu && /tmp/mb_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int N = 512;

template <int OP>
__global__ void k(uint32_t* out, uint64_t* cyc, uint32_t seed) {
  uint32_t a[8];
  uint64_t w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = seed * (threadIdx.x + 1) + j;
    w[j] = a[j] * 0x9E3779B97F4A7C15ull;
  }
  const uint32_t c = seed | 1u;
  __syncthreads();
  const uint64_t t0 = clock64();
  for (int i = 0; i < N; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (OP == 0) w[j] = (uint64_t)a[j] * c + w[j];            // v_mad_u64_u32
      if constexpr (OP == 1) a[j] = a[j] * c;                              // v_mul_lo_u32
      if constexpr (OP == 2) a[j] = __umulhi(a[j], c) + j;                 // v_mul_hi_u32 (+ add)
      if constexpr (OP == 3) a[j] = (a[j] + c) ^ j;                        // v_add + v_xor
      if constexpr (OP == 4) a[j] = __umul24(a[j], c) + 1;                 // v_mul_u32_u24 (+ add: mad24)
      if constexpr (OP == 0) a[j] = (uint32_t)(w[j] >> 32);
    }
  }
  const uint64_t t1 = clock64();
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r ^= a[j] ^ (uint32_t)w[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
void run(const char* name, int tpb) {
  uint32_t* out;
  uint64_t* cyc;
  const int G = 256;
  hipMalloc(&out, sizeof(uint32_t) * G * tpb);
  hipMalloc(&cyc, sizeof(uint64_t) * G * (tpb / 64));
  hipLaunchKernelGGL(k<OP>, dim3(G), dim3(tpb), 0, 0, out, cyc, 12345u);
  hipLaunchKernelGGL(k<OP>, dim3(G), dim3(tpb), 0, 0, out, cyc, 12345u);
  hipDeviceSynchronize();
  uint64_t h[G * 16];
  hipMemcpy(h, cyc, sizeof(uint64_t) * G * (tpb / 64), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < G * (tpb / 64); ++i) s += (double)h[i];
  s /= G * (tpb / 64);
  // s_memtime counts at the shader clock on gfx950? report raw units per (iteration x chain)
  printf("%-28s waves/SIMD %d: %.2f clock64 units per op per wave (%.0f per wave total)\n", name, tpb / 256,
         s / (N * 8.0), s);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int tpb : {256, 512}) {
    run<0>("v_mad_u64_u32 (+shift)", tpb);
    run<1>("v_mul_lo_u32", tpb);
    run<2>("v_mul_hi_u32 + v_add", tpb);
    run<3>("v_add_u32 + v_xor", tpb);
    run<4>("v_mad_u32_u24", tpb);
  }
  return 0;
}
