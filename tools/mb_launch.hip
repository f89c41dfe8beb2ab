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
  return 0;
}
