// Scan-primitive probe for the multi-workgroup exact C-ROOMS draw calls: the cost of a block ticket (one device
// atomic per block), of the single-pass decoupled look-back (wave 0 reads 64 predecessors per round), and of a
// reduce-by-reading prefix (each block sums its predecessors' counts), per launch, at the grid sizes a 2^16 and a
// 2^21-env normal call use.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_scan.hip -o tools/mb_scan.bin && ./tools/mb_scan.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int T = 256;

struct Scan {
  uint64_t* status;
  unsigned long long* ticket;
  unsigned long long tbase;
  uint32_t tag;
};

__device__ __forceinline__ int ticket(const Scan& sc) {
  __shared__ int tk;
  if (threadIdx.x == 0) tk = (int)(atomicAdd(sc.ticket, 1ull) - sc.tbase);
  __syncthreads();
  return tk;
}

__device__ __forceinline__ uint32_t lookback(const Scan& sc, int bid, uint32_t agg) {
  __shared__ uint32_t pre;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const uint64_t tg = (uint64_t)sc.tag << 32;
    if (bid == 0) {
      if (lane == 0) {
        __hip_atomic_store(&sc.status[0], tg | (2ull << 30) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pre = 0;
      }
    } else {
      if (lane == 0)
        __hip_atomic_store(&sc.status[bid], tg | (1ull << 30) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t run = 0;
      for (int top = bid - 1;;) {
        const int idx = top - lane;
        bool ready = true, inc = false;
        uint32_t val = 0;
        if (idx >= 0) {
          const uint64_t v = __hip_atomic_load(&sc.status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint32_t f = (uint32_t)(v >> 30) & 3u;
          ready = (v >> 32) == sc.tag && f != 0;
          inc = ready && f == 2u;
          val = (uint32_t)(v & 0x3FFFFFFFu);
        }
        const uint64_t incm = __ballot(inc);
        const int first = incm ? __builtin_ctzll(incm) : 64;
        const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
        if (__ballot(!ready) & need) {
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        uint32_t x = lane <= first ? val : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        run += x;
        if (first < 64) break;
        top -= 64;
      }
      if (lane == 0) {
        __hip_atomic_store(&sc.status[bid], tg | (2ull << 30) | (run + agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        pre = run;
      }
    }
  }
  __syncthreads();
  return pre;
}

// mode 0: plain (write one word), 1: ticket, 2: ticket + look-back, 3: blockIdx + look-back,
// 4: read-prefix (sum of counts[0, bid) by the whole block), 5: counts written by this launch (producer half)
__global__ __launch_bounds__(T) void probe(int mode, Scan sc, uint32_t* out, const uint32_t* counts) {
  int bid = blockIdx.x;
  uint32_t pre = 0;
  if (mode == 1 || mode == 2) bid = ticket(sc);
  if (mode == 2 || mode == 3) pre = lookback(sc, bid, 256);
  if (mode == 4) {
    __shared__ uint32_t ws[T / 64];
    uint32_t x = 0;
    for (int j = threadIdx.x; j < bid; j += T) x += counts[j];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = x;
    __syncthreads();
    pre = ws[0] + ws[1] + ws[2] + ws[3];
  }
  if (threadIdx.x == 0) out[bid] = pre + 1;
}

int main() {
  const int maxb = 1 << 15;
  uint64_t* status;
  unsigned long long* tk;
  uint32_t *out, *counts;
  hipMalloc(&status, maxb * 8);
  hipMalloc(&tk, 8);
  hipMalloc(&out, maxb * 4);
  hipMalloc(&counts, maxb * 4);
  hipMemset(status, 0, maxb * 8);
  hipMemset(tk, 0, 8);
  hipMemset(counts, 1, maxb * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  unsigned long long tbase = 0;
  uint32_t tag = 0;
  const char* names[] = {"plain", "ticket", "ticket+lookback", "blockIdx+lookback", "read-prefix"};
  const int grids[] = {182, 576, 2048, 16800};
  for (int g : grids) {
    for (int mode = 0; mode < 5; ++mode) {
      if (mode == 4 && g > 4096) continue;
      const int reps = 200;
      for (int r = 0; r < reps + 20; ++r) {
        if (r == 20) hipEventRecord(a, 0);
        Scan sc{status, tk, tbase, ++tag};
        if (mode == 1 || mode == 2) tbase += g;
        hipLaunchKernelGGL(probe, dim3(g), dim3(T), 0, 0, mode, sc, out, counts);
      }
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      uint32_t last = 0;
      hipMemcpy(&last, out + g - 1, 4, hipMemcpyDeviceToHost);
      printf("blocks %6d %-18s %7.2f us/launch (last block's prefix %u)\n", g, names[mode], ms * 1e3 / reps, last);
    }
  }
  return 0;
}
