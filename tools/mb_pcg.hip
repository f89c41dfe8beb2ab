// Throughput of numpy's PCG64 (XSL-RR 128/64) word generation on gfx950: every thread of a 256-block grid steps its
// own 128-bit LCG state N times and folds the outputs (the form a window fill takes: one per-lane jump, then
// consecutive steps), at 4, 8 and 12 waves per CU. Reports chip-wide words/s and cycles per wave-word per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_pcg.hip -o tools/mb_pcg.bin && tools/mb_pcg.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../gym-po-taxi_amd/csrc/gp_common.h"

constexpr int N = 1024;

template <int ILP>
__global__ void gen(uint64_t* out, uint64_t inc_hi, uint64_t inc_lo, uint64_t* cyc) {
  const u128 inc = mk128(inc_hi, inc_lo);
  u128 s[ILP];
#pragma unroll
  for (int j = 0; j < ILP; ++j) s[j] = mk128(blockIdx.x * 977 + j, threadIdx.x * 0x9E3779B97F4A7C15ull + j);
  uint64_t acc = 0;
  const uint64_t t0 = clock64();
  for (int i = 0; i < N / ILP; ++i) {
#pragma unroll
    for (int j = 0; j < ILP; ++j) {
      s[j] = pcg_step(s[j], inc);
      acc ^= pcg_output(s[j]);
    }
  }
  const uint64_t t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
}

// One general affine jump per word (runtime multiplier and increment, as a window base or a radix jump).
__global__ void jumps(uint64_t* out, const PcgJump* jt, uint64_t* cyc) {
  u128 s = mk128(blockIdx.x, threadIdx.x * 0x9E3779B97F4A7C15ull);
  const PcgJump j = jt[threadIdx.x & 63];
  uint64_t acc = 0;
  const uint64_t t0 = clock64();
  for (int i = 0; i < N / 4; ++i) {
    s = apply_jump(j, s);
    acc ^= pcg_output(s);
  }
  const uint64_t t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
}

template <class F>
void timeit(const char* name, int tpb, int words_per_thread, F launch) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch();
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(a);
    launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  const double words = 256.0 * tpb * words_per_thread;
  // cycles per wave-word per SIMD at 2.4 GHz: (time * 2.4e9) / (words / 64 / (256 CUs * 4 SIMDs))
  const double cpw = best * 1e-3 * 2.4e9 / (words / 64.0 / 1024.0);
  printf("%-28s tpb %4d: %.3f ms, %.3g words/s, %.1f cycles per wave-word per SIMD (2.4 GHz)\n", name, tpb, best,
         words / (best * 1e-3), cpw);
}

int main() {
  uint64_t *out, *cyc;
  PcgJump* jt;
  (void)hipMalloc(&out, sizeof(uint64_t) * 256 * 1024);
  (void)hipMalloc(&cyc, sizeof(uint64_t) * 256 * 16);
  (void)hipMalloc(&jt, sizeof(PcgJump) * 64);
  PcgJump h[64];
  const u128 inc = mk128(0x1234567ull, 0x89abcdef0123457ull);
  for (int i = 0; i < 64; ++i) h[i] = pcg_jump_params((u128)(1000 + 37 * i), inc);
  (void)hipMemcpy(jt, h, sizeof(h), hipMemcpyHostToDevice);
  for (int tpb : {256, 512, 768}) {
    timeit("lcg step ILP1", tpb, N, [&] { hipLaunchKernelGGL(gen<1>, dim3(256), dim3(tpb), 0, 0, out, hi64(inc), lo64(inc), cyc); });
    timeit("lcg step ILP2", tpb, N, [&] { hipLaunchKernelGGL(gen<2>, dim3(256), dim3(tpb), 0, 0, out, hi64(inc), lo64(inc), cyc); });
    timeit("lcg step ILP4", tpb, N, [&] { hipLaunchKernelGGL(gen<4>, dim3(256), dim3(tpb), 0, 0, out, hi64(inc), lo64(inc), cyc); });
    timeit("general jump per word", tpb, N / 4, [&] { hipLaunchKernelGGL(jumps, dim3(256), dim3(tpb), 0, 0, out, jt, cyc); });
  }
  return 0;
}
