// Issue cost of the integer VALU instructions the PCG64 draw is made of, on gfx950 (inline asm, so the
// compiler can neither fold nor reorder them): 8 independent chains per lane, 1 or 2 waves per SIMD,
// cycles from clock64() per wave, reported relative to v_add_u32 (a full-rate op).
//   hipcc --offload-arch=gfx950 -O3 tools/mb_valu.hip -o tools/mb_valu.bin && tools/mb_valu.bin
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int N = 256;

#define CH8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
template <int OP>
__global__ void k(uint32_t* out, uint64_t* cyc, uint32_t seed) {
  uint32_t a0, a1, a2, a3, a4, a5, a6, a7;
  uint64_t w0, w1, w2, w3, w4, w5, w6, w7;
  const uint32_t c = seed | 1u;
#define INIT(j) a##j = seed * (threadIdx.x + 1) + j; w##j = (uint64_t)a##j * 0x9E3779B97F4A7C15ull;
  CH8(INIT)
  __syncthreads();
  const uint64_t t0 = clock64();
  for (int i = 0; i < N; ++i) {
    if constexpr (OP == 0) {
#define OPX(j) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##j) : "v"(c));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 1) {
#define OPX(j) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a##j) : "v"(c));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 2) {
#define OPX(j) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a##j) : "v"(c));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 3) {
#define OPX(j) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w##j) : "v"(a##j), "v"(c) : "vcc");
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 4) {
#define OPX(j) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(w##j) : "v"(c));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 5) {
#define OPX(j) asm volatile("v_alignbit_b32 %0, %0, %1, %1" : "+v"(a##j) : "v"(c));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 6) {
#define OPX(j) asm volatile("v_cmp_gt_u64 vcc, %0, %1\n\tv_cndmask_b32 %2, %2, %3, vcc" : : "v"(w##j), "v"(w0), "v"(a##j), "v"(c) : "vcc");
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 7) {
#define OPX(j) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %2, %2, %3, vcc" : : "v"(a##j), "v"(c), "v"(a##j), "v"(c) : "vcc");
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 8) {
#define OPX(j) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(w##j) : "v"(w0));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 9) {
#define OPX(j) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, %2, %1, vcc" : "+v"(a##j) : "v"(c), "v"(a0) : "vcc");
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 10) {
#define OPX(j) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a##j) : "v"(c));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 11) {
#define OPX(j) asm volatile("v_log_f32 %0, %0" : "+v"(a##j));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 12) {
#define OPX(j) asm volatile("v_sin_f32 %0, %0" : "+v"(a##j));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 13) {
#define OPX(j) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a##j));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 14) {
#define OPX(j) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(w##j) : "v"(w0));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 15) {
#define OPX(j) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(w##j) : "v"(w0));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 16) {
#define OPX(j) asm volatile("v_floor_f64 %0, %0" : "+v"(w##j));
      CH8(OPX)
#undef OPX
    } else if constexpr (OP == 17) {
#define OPX(j) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a##j) : "v"(c));
      CH8(OPX)
#undef OPX
    }
  }
  const uint64_t t1 = clock64();
  uint32_t r = 0;
#define FIN(j) r ^= a##j ^ (uint32_t)w##j;
  CH8(FIN)
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
double run(int tpb) {
  uint32_t* out;
  uint64_t* cyc;
  const int G = 256;
  (void)hipMalloc(&out, sizeof(uint32_t) * G * tpb);
  (void)hipMalloc(&cyc, sizeof(uint64_t) * G * (tpb / 64));
  hipLaunchKernelGGL(k<OP>, dim3(G), dim3(tpb), 0, 0, out, cyc, 12345u);
  hipLaunchKernelGGL(k<OP>, dim3(G), dim3(tpb), 0, 0, out, cyc, 12345u);
  (void)hipDeviceSynchronize();
  static uint64_t h[256 * 16];
  (void)hipMemcpy(h, cyc, sizeof(uint64_t) * G * (tpb / 64), hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < G * (tpb / 64); ++i) s += (double)h[i];
  (void)hipFree(out);
  (void)hipFree(cyc);
  return s / (G * (tpb / 64)) / (N * 8.0);
}

int main() {
  const char* names[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_lshlrev_b64",
                         "v_alignbit_b32", "v_cmp_gt_u64 + v_cndmask", "v_cmp_gt_u32 + v_cndmask",
                         "v_lshl_add_u64", "v_add_co + v_addc_co", "v_bitop3_b32", "v_log_f32", "v_sin_f32",
                         "v_sqrt_f32", "v_fma_f64", "v_mul_f64", "v_floor_f64", "v_fma_f32"};
  for (int tpb : {256, 512}) {
    double r[18] = {run<0>(tpb), run<1>(tpb), run<2>(tpb), run<3>(tpb), run<4>(tpb), run<5>(tpb),
                    run<6>(tpb), run<7>(tpb), run<8>(tpb), run<9>(tpb), run<10>(tpb), run<11>(tpb),
                    run<12>(tpb), run<13>(tpb), run<14>(tpb), run<15>(tpb), run<16>(tpb), run<17>(tpb)};
    for (int i = 0; i < 18; ++i)
      printf("waves/SIMD %d  %-28s %6.2f clock64 units per wave-op  (%.2fx v_add_u32)\n", tpb / 256, names[i], r[i],
             r[i] / r[0]);
  }
  return 0;
}
