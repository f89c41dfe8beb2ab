// gp_internal.h — handle layout shared by the per-kind backends (not part of the C ABI).
#pragma once
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/gym_po_amd.h"
#include "gp_common.h"

// numpy Generator(PCG64) state as the host sees it.
struct RngHost {
  u128 state = 0, inc = 1;
  uint32_t has_u32 = 0, uinteger = 0;
};

// SeedSequence(entropy, spawn_key).generate_state(n, uint64) — numpy bit_generator.pyx restated.
std::vector<uint64_t> seed_sequence_u64(const std::vector<uint32_t>& entropy, const std::vector<uint32_t>& spawn_key,
                                        int n_words64);
RngHost pcg64_from_seed(const std::vector<uint32_t>& entropy, const std::vector<uint32_t>& spawn_key);
// P(argmax = k) for Multinomial(n, uniform over m) counts, ties -> first (taxi reset law).
std::vector<double> argmax_multinomial_distribution(int m, int n);
// Radix-64 jump tables (JT_LEVELS x 64) for increment `inc`.
std::vector<PcgJump> build_jump_tables(u128 inc);

// Diagnostic knobs (gp_debug_set), read by the backends at gp_create.
struct GpDebugKnobs {
  int disable_fused = 0, no_staging = 0, xmode = 1, fault_block = -1;
  int fused_tile = 0;       // GRID fused kernel: envs per tile (512 / 1024 / 2048); 0 = chosen by size
  uint32_t spin_limit = 0;  // 0 = the kernel's default
  int generic_kernels = 0;  // CROOMS: 1 = never the compile-time-specialised philox rollout (A/B and parity tests)
  int no_spw = 0;           // GRID fused kernel: 1 = no speculative word windows (A/B and parity tests)
  int no_wgrid = 0;         // GRID: 1 = never the windowed kernel (wgrid.hip): the older fused kernel instead
  int wg_halo = 0;          // GRID windowed kernel: window halo (256 or 512 draws); 0 = default
  int wg_bias = 0;          // GRID windowed kernel: added to the predicted reset count (forces window misses)
  int wg_tmode = 0;         // GRID windowed kernel: timing-study variants (wgrid.hip TM_*); some give wrong results
  int wg_kmax = -1;         // GRID: longest launch (steps) on the windowed kernel; longer ones on the fused kernel (-1 default)
  int xg_min_envs = -1;      // CROOMS exact mode: largest B on the one-workgroup kernel (-1 = crooms.hip XG_MIN_ENVS)
  int xg_ppt_min = -1;       // CROOMS exact mode: normal calls above this many 256-position blocks take 4 per thread
  int xg_spb_min = -1;       // CROOMS exact mode: env kernels above this many env blocks take 4 per workgroup
  int taxi_npg_min = -1;    // TAXI numpy mode: largest B on the one-workgroup kernel (-1 = taxi.hip NPG_MIN_ENVS)
  int64_t fused_step = -1;  // GRID: the fused kernel's tag counter (GridCtl::step) set at every seed (-1 = kept)
  int wg_block_envs = 0;    // GRID windowed kernel: the smallest envs per block to use (0 = the smallest that fits)
  int wg_fill_simd = 0;     // GRID windowed kernel: per-SIMD window-row deltas, 4 signed nibbles (0 = WG_FILL_SIMD)
  int64_t wg_fill_wave = 0; // GRID windowed kernel: per-wave deltas on top, 8 signed nibbles (wave 0 lowest)
  int persist_bpc = 0;      // TAXI / CROOMS / ANT-TAG streaming rollouts: blocks per CU (0 = every resident block, persistent_grid)
};
const GpDebugKnobs& gp_debug_knobs();

// Grid of a persistent grid-stride tile loop (the Taxi / C-ROOMS / Ant-Tag rollouts: K steps per tile with the
// tile's state in registers): every resident block (occupancy x CUs), capped by the tiles. An equal number of
// tiles per block measured slower (round 6, profiles/r06_persist_grid.txt: C-ROOMS at 2^21 envs 17.4 us/step with
// 1,024 blocks of 4 tiles vs 15.7 with 1,280 blocks of 3-4; Ant-Tag 14.6 vs 13.9): per-wave latency, not the
// SIMDs' issue rate, bounds these loops, so more resident waves win even with a ragged last round. The knob
// persist_bpc forces the blocks per CU (A/Bs).
inline int persistent_grid(int ntiles, int cus, int occ) {
  const int forced = gp_debug_knobs().persist_bpc;
  const int bpc = forced > 0 ? forced : (occ < 1 ? 1 : (occ > 8 ? 8 : occ));
  const int g = cus * bpc;
  return ntiles < g ? (ntiles > 0 ? ntiles : 1) : g;
}

// Per-kind backend interface; gp_env owns one.
// hipEvent pairs around the step-kernel launches (gp_set_profiling / gp_profile_read).
struct KernelTimer {
  bool on = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  size_t used = 0;
  double acc_ms = 0;
  int64_t acc_n = 0;
  void begin(hipStream_t s);
  void end(hipStream_t s);
  int read(double* ms, int64_t* n);
  ~KernelTimer();
};

struct EnvBackend {
  KernelTimer timer;   // the step kernel (K1 / fused rollout)
  KernelTimer timer2;  // the reset resolver (K2, numpy mode)
  int64_t B = 0;
  int device = 0;
  int rng_mode = GP_RNG_NUMPY;
  int persist_grid = 0;  // blocks of the persistent rollout grid (Taxi / C-ROOMS / Ant-Tag; gp_query "persist_blocks")
  int persist_occ = 0;   // resident blocks per CU of that rollout kernel (the occupancy query)
  int obs_dtype = GP_DTYPE_I32;
  int obs_width = 1;
  bool has_reset = false;
  RngHost rng;                 // host copy of the numpy-mode RNG state (authoritative until uploaded)
  uint32_t philox_key[2] = {0, 0};
  virtual ~EnvBackend() {}
  virtual int seed(const RngHost& r, const uint32_t key[2]) = 0;
  virtual int set_rng_state(const RngHost& r) = 0;
  virtual int get_rng_state(RngHost* r) = 0;
  virtual int reset(void* obs, hipStream_t s) = 0;
  virtual int step(const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) = 0;
  virtual int rollout(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s);
  virtual int get_state(void* a, void* b, void* c, void* d, hipStream_t s) = 0;
  virtual int set_state(const void* a, const void* b, const void* c, const void* d, hipStream_t s) = 0;
  virtual int set_replay(const void* u, const void* i0, const void* i1, const void* f0, const void* f1) {
    gp_set_error("replay mode not supported by this env kind");
    return GP_E_UNSUPPORTED;
  }
  virtual int valid_cells(int which, int32_t* out, int cap) const { return 0; }
  virtual int metrics(double out[4]) = 0;
  // Syncs and reports device-side failures of earlier launches (GP_E_DEVICE); kinds without
  // cross-block waits have none.
  virtual int check() { return GP_OK; }
  // Introspection (gp_query): kernel geometry of this handle.
  virtual int query(const char* key, int64_t* v) const {
    if (!strcmp(key, "num_envs")) *v = B;
    else if (!strcmp(key, "rng_mode")) *v = rng_mode;
    else if (!strcmp(key, "persist_blocks")) *v = persist_grid;
    else if (!strcmp(key, "persist_occupancy")) *v = persist_occ;
    else {
      gp_set_error("gp_query: unknown key '%s'", key);
      return GP_E_INVALID;
    }
    return GP_OK;
  }
  virtual int debug_stamps(unsigned long long* out, int cap) { return 0; }
  // gp_autotune: pick the faster of interchangeable kernels for K-step launches on this device (no-op here)
  virtual int autotune(int K, int reps, int* chosen) {
    if (chosen) *chosen = -1;
    return GP_OK;
  }
  virtual int reset_distribution(double* out, int cap) const {
    gp_set_error("no reset distribution for this env kind");
    return GP_E_UNSUPPORTED;
  }
  // rgb_array frames of envs 0..n-1, tiled (gp_taxi_render)
  virtual int render(int n, int hansen, uint8_t* out, int32_t dims[4], hipStream_t s) {
    gp_set_error("rendering is not available for this env kind (the reference does not render it either)");
    return GP_E_UNSUPPORTED;
  }
  size_t obs_elem_size() const { return obs_dtype == GP_DTYPE_U8 ? 1 : (obs_dtype == GP_DTYPE_F64 ? 8 : 4); }
  virtual size_t rollout_action_bytes_per_env() const { return 4; }
};

std::unique_ptr<EnvBackend> make_grid_backend(const gp_grid_config* cfg, int64_t B, int device, int rng_mode, int* err);
std::unique_ptr<EnvBackend> make_taxi_backend(const gp_taxi_config* cfg, int64_t B, int device, int rng_mode, int* err);
std::unique_ptr<EnvBackend> make_crooms_backend(const gp_crooms_config* cfg, int64_t B, int device, int rng_mode,
                                                int* err);
std::unique_ptr<EnvBackend> make_anttag_backend(const gp_anttag_config* cfg, int64_t B, int device, int rng_mode,
                                                int* err);

// Small device-buffer owner.
struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  DevBuf() {}
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  int alloc(size_t bytes) {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = bytes;
    if (bytes == 0) return GP_OK;
    GP_HIP_CHECK(hipMalloc(&p, bytes));
    GP_HIP_CHECK(hipMemset(p, 0, bytes));
    return GP_OK;
  }
  template <class T>
  int upload(const std::vector<T>& v) {
    int e = alloc(v.size() * sizeof(T) + 16);
    if (e) return e;
    if (!v.empty()) GP_HIP_CHECK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return GP_OK;
  }
  template <class T>
  T* as() const {
    return (T*)p;
  }
};

// The per-handle device error word of the kinds without a control block (taxi, ant-tag, C-ROOMS philox /
// replay): kernels OR GP_DERR_* bits into it; check() syncs, reads it and reports GP_E_DEVICE.
struct DevErr {
  DevBuf buf;
  int alloc() { return buf.alloc(16); }
  uint32_t* ptr() const { return buf.as<uint32_t>(); }
  int clear();                       // on seed: a new stream, earlier errors no longer apply
  int check(const char* kind) const;  // GP_OK or GP_E_DEVICE with gp_last_error() text
};

