// Dependent-chain LATENCY of the integer VALU instructions the PCG64 128-bit multiply is made of, and of an
// LDS round trip, on gfx950: ONE wave per CU, a single dependent chain, clock64() cycles per op.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_lat.hip -o tools/mb_lat.bin && tools/mb_lat.bin
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int N = 512;

template <int OP>
__global__ void k(uint32_t* out, uint64_t* cyc, uint32_t seed) {
  __shared__ uint32_t lds[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) lds[i] = (uint32_t)i * 7u & 1023u;
  __syncthreads();
  uint32_t a = seed * (threadIdx.x + 1), c = seed | 1u;
  uint64_t w = (uint64_t)a * 0x9E3779B97F4A7C15ull;
  const uint64_t t0 = clock64();
  for (int i = 0; i < N; ++i) {
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(c));
    else if constexpr (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(c));
    else if constexpr (OP == 2) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w) : "v"((uint32_t)w), "v"(c) : "vcc");
    else if constexpr (OP == 3) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(w) : "v"(w));
    else if constexpr (OP == 4) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, %2, %1, vcc" : "+v"(a), "+v"(c) : : "vcc");
    else if constexpr (OP == 5) { a = lds[a & 1023u]; }
    else if constexpr (OP == 6) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a) : "v"(c));
  }
  const uint64_t t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ (uint32_t)w ^ c;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
double run() {
  uint32_t* out;
  uint64_t* cyc;
  const int G = 64;
  (void)hipMalloc(&out, sizeof(uint32_t) * G * 64);
  (void)hipMalloc(&cyc, sizeof(uint64_t) * G);
  hipLaunchKernelGGL(k<OP>, dim3(G), dim3(64), 0, 0, out, cyc, 12345u);
  hipLaunchKernelGGL(k<OP>, dim3(G), dim3(64), 0, 0, out, cyc, 12345u);
  (void)hipDeviceSynchronize();
  uint64_t h[64];
  (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < G; ++i) s += (double)h[i];
  (void)hipFree(out);
  (void)hipFree(cyc);
  return s / G / N;
}

int main() {
  const char* names[] = {"v_add_u32", "v_mul_lo_u32", "v_mad_u64_u32 (chained via addend)", "v_lshl_add_u64",
                         "v_add_co + v_addc_co", "ds_read_b32 (dependent address)", "v_mul_hi_u32"};
  double r[7] = {run<0>(), run<1>(), run<2>(), run<3>(), run<4>(), run<5>(), run<6>()};
  for (int i = 0; i < 7; ++i) printf("%-36s %7.2f clock64 units per dependent op\n", names[i], r[i]);
  return 0;
}
