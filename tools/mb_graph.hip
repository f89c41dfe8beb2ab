// Dependent-launch cost, stream vs hipGraph replay: a chain of small kernels, each reading what the previous one
// wrote (64K ints, the C-ROOMS exact-mode step's per-env arrays at 65,536 envs), 5 kernels per "step" x 20 steps,
// launched one by one on a stream vs captured once into a graph and replayed. Per-kernel time = event span / 100.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_graph.hip -o tools/mb_graph.bin && ./tools/mb_graph.bin
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

__global__ void chain_kernel(int* __restrict__ dst, const int* __restrict__ src, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i] + 1;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));                \
      return 1;                                                            \
    }                                                                      \
  } while (0)

static void enqueue(hipStream_t s, int* buf0, int* buf1, int n, int blocks, int launches) {
  for (int k = 0; k < launches; ++k) {
    int* dst = (k & 1) ? buf0 : buf1;
    const int* src = (k & 1) ? buf1 : buf0;
    hipLaunchKernelGGL(chain_kernel, dim3(blocks), dim3(256), 0, s, dst, src, n);
  }
}

int main() {
  const int launches = 100;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int sizes[] = {65536, 180224, 1 << 20};
  for (int n : sizes) {
    int *buf0, *buf1;
    CK(hipMalloc(&buf0, (size_t)n * 4));
    CK(hipMalloc(&buf1, (size_t)n * 4));
    CK(hipMemset(buf0, 0, (size_t)n * 4));
    CK(hipMemset(buf1, 0, (size_t)n * 4));
    const int blocks = (n + 255) / 256;
    // the graph: the same 100 launches captured once
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    enqueue(s, buf0, buf1, n, blocks, launches);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int mode = 0; mode < 3; ++mode) {  // 0 stream, 1 graph, 2 one kernel alone
      std::vector<double> us;
      for (int r = 0; r < 60; ++r) {
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(a, s));
        if (mode == 0) enqueue(s, buf0, buf1, n, blocks, launches);
        else if (mode == 1) CK(hipGraphLaunch(ge, s));
        else enqueue(s, buf0, buf1, n, blocks, 1);
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 10) us.push_back(ms * 1e3 / (mode == 2 ? 1 : launches));
      }
      std::sort(us.begin(), us.end());
      printf("n %8d blocks %5d %-26s: median %.2f us per kernel (p10 %.2f, p90 %.2f)\n", n, blocks,
             mode == 0 ? "stream, 100 dependent" : mode == 1 ? "hipGraph replay, 100 dep." : "one kernel alone",
             us[us.size() / 2], us[us.size() / 10], us[us.size() * 9 / 10]);
    }
    int check = -1;
    CK(hipMemcpy(&check, buf0, 4, hipMemcpyDeviceToHost));
    printf("  (chain value %d)\n", check);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipFree(buf0));
    CK(hipFree(buf1));
  }
  return 0;
}
