// Launch-cost probe: the event-timed duration and host wall (launch + sync) of an EMPTY kernel with the fused
// numpy rollout's geometry (256 blocks x 704 threads, ~98 KB dynamic LDS), vs smaller geometries. The part of a
// short launch's event time that no wave sees (dispatch before the first wave, completion after the last).
//   hipcc --offload-arch=gfx950 -O3 tools/mb_launch.hip -o tools/mb_launch.bin && ./tools/mb_launch.bin
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

__global__ void empty_kernel(int* out) {
  extern __shared__ char dyn[];
  if (out && threadIdx.x == 0 && blockIdx.x == 0) out[0] = (int)dyn[0];
}

struct Big {
  uint64_t w[80];  // 640 B of kernel arguments, like the fused kernel's GridDev by value
};
__global__ void big_arg_kernel(Big b, int* out) {
  if (out && threadIdx.x == 0 && blockIdx.x == 0 && b.w[79] == 12345) out[2] = (int)b.w[3];
}

__global__ void touch_kernel(int* out, const int* in, int n) {  // every thread reads 16 B, block 0 writes one word
  extern __shared__ char dyn[];
  const int i = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  int4 v = i + 3 < n ? *reinterpret_cast<const int4*>(in + i) : int4{0, 0, 0, 0};
  if (v.x == 12345 && v.y == 1) out[1] = v.z + (int)dyn[0];
}

int main() {
  int *d, *in;
  const int n = 1 << 22;
  hipMalloc(&d, 64);
  hipMalloc(&in, (size_t)n * 4);
  hipMemset(in, 0, (size_t)n * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  struct G { int blocks, threads, lds; bool touch; };
  const G gs[] = {{256, 256, 0, false}, {256, 704, 0, false}, {256, 704, 98 * 1024, false},
                  {256, 704, 98 * 1024, true}, {1024, 256, 0, false}};
  hipFuncSetAttribute((const void*)empty_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
  hipFuncSetAttribute((const void*)touch_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
  hipFuncSetAttribute((const void*)big_arg_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
  for (const G& g : gs) {
    std::vector<double> ev, wall;
    for (int r = 0; r < 120; ++r) {
      hipDeviceSynchronize();
      const auto t0 = std::chrono::steady_clock::now();
      hipEventRecord(a, 0);
      if (g.touch)
        hipLaunchKernelGGL(touch_kernel, dim3(g.blocks), dim3(g.threads), g.lds, 0, d, in, n);
      else
        hipLaunchKernelGGL(empty_kernel, dim3(g.blocks), dim3(g.threads), g.lds, 0, d);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      const auto t1 = std::chrono::steady_clock::now();
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (r >= 20) {
        ev.push_back(ms * 1e3);
        wall.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      }
    }
    std::sort(ev.begin(), ev.end());
    std::sort(wall.begin(), wall.end());
    printf("blocks %4d threads %4d lds %6d %s: event median %.2f us, host wall median %.2f us\n", g.blocks,
           g.threads, g.lds, g.touch ? "read 16 B/thread" : "empty          ", ev[ev.size() / 2],
           wall[wall.size() / 2]);
  }
  // host cost of the launch call itself (enqueue), small vs 640-B kernel arguments, idle stream
  Big big{};
  for (int variant = 0; variant < 2; ++variant) {
    std::vector<double> call, wall;
    for (int r = 0; r < 220; ++r) {
      hipDeviceSynchronize();
      const auto t0 = std::chrono::steady_clock::now();
      if (variant == 0)
        hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(704), 98 * 1024, 0, d);
      else
        hipLaunchKernelGGL(big_arg_kernel, dim3(256), dim3(704), 98 * 1024, 0, big, d);
      const auto t1 = std::chrono::steady_clock::now();
      hipDeviceSynchronize();
      const auto t2 = std::chrono::steady_clock::now();
      if (r >= 20) {
        call.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        wall.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
      }
    }
    std::sort(call.begin(), call.end());
    std::sort(wall.begin(), wall.end());
    printf("%s kernel arguments: hipLaunchKernel call median %.2f us, launch + hipDeviceSynchronize median %.2f us\n",
           variant ? "640-B" : "8-B  ", call[call.size() / 2], wall[wall.size() / 2]);
  }
  return 0;
}
