// api.hip — the extern "C" boundary (include/gym_po_amd.h), numpy-compatible seeding, and the
// PCG64 jump-table builder shared by the backends.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "gp_internal.h"

struct gp_env {
  int kind = 0;
  std::unique_ptr<EnvBackend> be;
};

static thread_local char g_err[1024] = "";

void gp_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

const char* gp_derr_text(uint32_t flags) {
  static thread_local char buf[512];
  buf[0] = 0;
  if (flags & GP_DERR_ACTION)
    strncat(buf, "an action outside [-n, n) was given (the reference raises IndexError there; the device clamped it); ",
            sizeof(buf) - strlen(buf) - 1);
  if (flags & GP_DERR_TIMEOUT)
    strncat(buf, "a persistent kernel's cross-block wait timed out (blocks not co-resident?); ",
            sizeof(buf) - strlen(buf) - 1);
  if (flags & GP_DERR_OVERFLOW)
    strncat(buf, "more rejected choice() words in one step than the windowed kernel lists; ", sizeof(buf) - strlen(buf) - 1);
  if (flags & GP_DERR_BTPE)
    strncat(buf, "a Taxi numpy-mode reset needed numpy's BTPE binomial (not restated on the device); ",
            sizeof(buf) - strlen(buf) - 1);
  if (flags & GP_DERR_STREAM)
    strncat(buf, "a numpy normal needed more words than one stream window holds; ", sizeof(buf) - strlen(buf) - 1);
  return buf;
}

static GpDebugKnobs g_dbg;
const GpDebugKnobs& gp_debug_knobs() { return g_dbg; }
extern int gp_xg_graph_knob;  // crooms.hip: exact mode's K-step launch sequence as a hipGraph (-1 / 0 / 1)

int DevErr::clear() {
  if (!buf.p) return GP_OK;
  GP_HIP_CHECK(hipDeviceSynchronize());
  GP_HIP_CHECK(hipMemset(buf.p, 0, sizeof(uint32_t)));
  return GP_OK;
}

int DevErr::check(const char* kind) const {
  GP_HIP_CHECK(hipDeviceSynchronize());
  if (!buf.p) return GP_OK;
  uint32_t f = 0;
  GP_HIP_CHECK(hipMemcpy(&f, buf.p, sizeof(f), hipMemcpyDeviceToHost));
  if (!f) return GP_OK;
  gp_set_error("%s: device error flags 0x%x: %sthe outputs and env state since the last seed are invalid "
               "(reseed to clear)", kind, f, gp_derr_text(f));
  return GP_E_DEVICE;
}

// ------------------------------------------------------------------ SeedSequence ----
// numpy/random/bit_generator.pyx (SeedSequence.mix_entropy / generate_state), restated.
namespace {
constexpr uint32_t INIT_A = 0x43b0d7e5u, MULT_A = 0x931e8875u, INIT_B = 0x8b51f9ddu, MULT_B = 0x58f38dedu;
constexpr uint32_t MIX_MULT_L = 0xca01f9ddu, MIX_MULT_R = 0x4973f715u;
constexpr int XSHIFT = 16, POOL = 4;

std::vector<uint32_t> seed_pool(const std::vector<uint32_t>& entropy, const std::vector<uint32_t>& spawn_key) {
  uint32_t hash_const = INIT_A;
  auto hashmix = [&](uint32_t v) {
    v ^= hash_const;
    hash_const *= MULT_A;
    v *= hash_const;
    v ^= v >> XSHIFT;
    return v;
  };
  auto mix = [](uint32_t x, uint32_t y) {
    uint32_t r = MIX_MULT_L * x - MIX_MULT_R * y;
    r ^= r >> XSHIFT;
    return r;
  };
  std::vector<uint32_t> run = entropy.empty() ? std::vector<uint32_t>{0u} : entropy;
  if (!spawn_key.empty()) {
    if (run.size() < (size_t)POOL) run.resize(POOL, 0u);
    run.insert(run.end(), spawn_key.begin(), spawn_key.end());
  }
  std::vector<uint32_t> mixer(POOL);
  for (int i = 0; i < POOL; ++i) mixer[i] = hashmix(i < (int)run.size() ? run[i] : 0u);
  for (int s = 0; s < POOL; ++s)
    for (int d = 0; d < POOL; ++d)
      if (s != d) mixer[d] = mix(mixer[d], hashmix(mixer[s]));
  for (size_t s = POOL; s < run.size(); ++s)
    for (int d = 0; d < POOL; ++d) mixer[d] = mix(mixer[d], hashmix(run[s]));
  return mixer;
}
}  // namespace

std::vector<uint64_t> seed_sequence_u64(const std::vector<uint32_t>& entropy, const std::vector<uint32_t>& spawn_key,
                                        int n_words64) {
  std::vector<uint32_t> pool = seed_pool(entropy, spawn_key);
  uint32_t hash_const = INIT_B;
  std::vector<uint32_t> w32(2 * n_words64);
  for (int i = 0; i < 2 * n_words64; ++i) {
    uint32_t v = pool[i % POOL];
    v ^= hash_const;
    hash_const *= MULT_B;
    v *= hash_const;
    v ^= v >> XSHIFT;
    w32[i] = v;
  }
  std::vector<uint64_t> out(n_words64);
  for (int i = 0; i < n_words64; ++i) out[i] = (uint64_t)w32[2 * i] | ((uint64_t)w32[2 * i + 1] << 32);
  return out;
}

// numpy PCG64.__init__ -> pcg64_set_seed -> pcg_setseq_128_srandom_r.
RngHost pcg64_from_seed(const std::vector<uint32_t>& entropy, const std::vector<uint32_t>& spawn_key) {
  std::vector<uint64_t> w = seed_sequence_u64(entropy, spawn_key, 4);
  const u128 initstate = mk128(w[0], w[1]);
  const u128 initseq = mk128(w[2], w[3]);
  RngHost r;
  r.inc = (initseq << 1) | 1;
  r.state = 0;
  r.state = r.state * pcg_mult() + r.inc;
  r.state += initstate;
  r.state = r.state * pcg_mult() + r.inc;
  r.has_u32 = 0;
  r.uinteger = 0;
  return r;
}

std::vector<PcgJump> build_jump_tables(u128 inc) {
  std::vector<PcgJump> t((size_t)JT_LEVELS * JT_RADIX);
  for (int L = 0; L < JT_LEVELS; ++L) {
    const u128 unit = (u128)1 << (JT_RADIX_BITS * L);
    for (int d = 0; d < JT_RADIX; ++d) t[(size_t)L * JT_RADIX + d] = pcg_jump_params(unit * (u128)d, inc);
  }
  return t;
}

// Default K-step rollout: K step launches on the stream.
int EnvBackend::rollout(int K, const void* act, void* obs, float* rew, uint8_t* term, uint8_t* trunc, hipStream_t s) {
  for (int k = 0; k < K; ++k) {
    const size_t off = (size_t)k * B;
    const size_t act_stride = rollout_action_bytes_per_env();
    int e = step((const uint8_t*)act + off * act_stride, (uint8_t*)obs + off * obs_width * obs_elem_size(),
                 rew + off, term + off, trunc + off, s);
    if (e) return e;
  }
  return GP_OK;
}

// ------------------------------------------------------------------ kernel timer ----
void KernelTimer::begin(hipStream_t s) {
  if (!on) return;
  if (used == ev.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
    ev.push_back({a, b});
  }
  (void)hipEventRecord(ev[used].first, s);
}
void KernelTimer::end(hipStream_t s) {
  if (!on || used >= ev.size()) return;
  (void)hipEventRecord(ev[used].second, s);
  ++used;
  if (used == ev.size() && used >= 4096) {  // bound the pool: fold finished pairs into the sums
    double ms;
    int64_t n;
    read(&ms, &n);
    acc_ms += ms;
    acc_n += n;
  }
}
int KernelTimer::read(double* ms, int64_t* n) {
  double t = 0;
  for (size_t i = 0; i < used; ++i) {
    GP_HIP_CHECK(hipEventSynchronize(ev[i].second));
    float x = 0;
    GP_HIP_CHECK(hipEventElapsedTime(&x, ev[i].first, ev[i].second));
    t += x;
  }
  *ms = t;
  *n = (int64_t)used;
  used = 0;
  return GP_OK;
}
KernelTimer::~KernelTimer() {
  for (auto& p : ev) {
    (void)hipEventDestroy(p.first);
    (void)hipEventDestroy(p.second);
  }
}

// ------------------------------------------------------------------ extern "C" ----
extern "C" {

const char* gp_last_error(void) { return g_err; }

int gp_debug_set(const char* key, int64_t value) {
  if (!key) {
    gp_set_error("gp_debug_set: null key");
    return GP_E_INVALID;
  }
  if (!strcmp(key, "disable_fused")) g_dbg.disable_fused = value != 0;
  else if (!strcmp(key, "no_staging")) g_dbg.no_staging = value != 0;
  else if (!strcmp(key, "xmode")) g_dbg.xmode = (int)value;
  else if (!strcmp(key, "spin_limit")) g_dbg.spin_limit = value > 0 ? (uint32_t)value : 0u;
  else if (!strcmp(key, "fault_block")) g_dbg.fault_block = (int)value;
  else if (!strcmp(key, "fused_tile")) g_dbg.fused_tile = (int)value;
  else if (!strcmp(key, "generic_kernels")) g_dbg.generic_kernels = value != 0;
  else if (!strcmp(key, "no_spw")) g_dbg.no_spw = value != 0;
  else if (!strcmp(key, "no_wgrid")) g_dbg.no_wgrid = value != 0;
  else if (!strcmp(key, "wg_halo")) g_dbg.wg_halo = (int)value;
  else if (!strcmp(key, "wg_bias")) g_dbg.wg_bias = (int)value;
  else if (!strcmp(key, "wg_tmode")) g_dbg.wg_tmode = (int)value;
  else if (!strcmp(key, "wg_kmax")) g_dbg.wg_kmax = (int)value;
  else if (!strcmp(key, "taxi_npg_min")) g_dbg.taxi_npg_min = (int)value;
  else if (!strcmp(key, "xg_min_envs")) g_dbg.xg_min_envs = (int)value;
  else if (!strcmp(key, "fused_step")) g_dbg.fused_step = value;
  else if (!strcmp(key, "wg_block_envs")) g_dbg.wg_block_envs = (int)value;
  else if (!strcmp(key, "wg_fill_simd")) g_dbg.wg_fill_simd = (int)value;
  else if (!strcmp(key, "wg_fill_wave")) g_dbg.wg_fill_wave = value;
  else if (!strcmp(key, "xg_ppt_min")) g_dbg.xg_ppt_min = (int)value;
  else if (!strcmp(key, "xg_spb_min")) g_dbg.xg_spb_min = (int)value;
  else if (!strcmp(key, "persist_bpc")) g_dbg.persist_bpc = (int)value;
  else if (!strcmp(key, "xg_graph")) gp_xg_graph_knob = (int)value;  // (crooms.hip: read at create)
  else {
    gp_set_error("gp_debug_set: unknown key '%s'", key);
    return GP_E_INVALID;
  }
  return GP_OK;
}
void gp_debug_reset(void) {
  g_dbg = GpDebugKnobs{};
  gp_xg_graph_knob = -1;
}
int gp_abi_version(void) { return GP_ABI_VERSION; }

// Makes the env's device current for one C-ABI call and gives the calling thread its own current device back on
// return (a caller whose current device is another GPU, e.g. torch's, must not find it switched afterwards).
struct DeviceGuard {
  int prev = -1;
  bool ok = true;  // false: the env's device could not be made current (the call must not run on another one)
  explicit DeviceGuard(int dev) {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) {
      ok = hipSetDevice(dev) == hipSuccess;
    } else if (cur != dev) {
      ok = hipSetDevice(dev) == hipSuccess;
      if (ok) prev = cur;
    }
    if (!ok) gp_set_error("hipSetDevice(%d) failed", dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

int gp_create(int kind, const void* config, int64_t num_envs, int device, int rng_mode, gp_env** out) {
  if (!out || !config) {
    gp_set_error("gp_create: null argument");
    return GP_E_INVALID;
  }
  *out = nullptr;
  if (rng_mode < GP_RNG_NUMPY || rng_mode > GP_RNG_REPLAY) {
    gp_set_error("gp_create: bad rng_mode %d", rng_mode);
    return GP_E_INVALID;
  }
  int ndev = 0;
  GP_HIP_CHECK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    gp_set_error("gp_create: device %d not present (%d devices)", device, ndev);
    return GP_E_INVALID;
  }
  DeviceGuard guard(device);
  if (!guard.ok) return GP_E_HIP;
  int err = GP_OK;
  std::unique_ptr<EnvBackend> be;
  switch (kind) {
    case GP_KIND_GRID: be = make_grid_backend((const gp_grid_config*)config, num_envs, device, rng_mode, &err); break;
    case GP_KIND_TAXI: be = make_taxi_backend((const gp_taxi_config*)config, num_envs, device, rng_mode, &err); break;
    case GP_KIND_CROOMS:
      be = make_crooms_backend((const gp_crooms_config*)config, num_envs, device, rng_mode, &err);
      break;
    case GP_KIND_ANTTAG:
      be = make_anttag_backend((const gp_anttag_config*)config, num_envs, device, rng_mode, &err);
      break;
    default: gp_set_error("gp_create: unknown kind %d", kind); return GP_E_INVALID;
  }
  if (!be) return err ? err : GP_E_INVALID;
  gp_env* e = new gp_env();
  e->kind = kind;
  e->be = std::move(be);
  *out = e;
  return GP_OK;
}

void gp_destroy(gp_env* env) { delete env; }

#define GP_REQUIRE_ENV()                 \
  if (!env || !env->be) {                \
    gp_set_error("null env handle");     \
    return GP_E_INVALID;                 \
  }                                      \
  DeviceGuard gp_device_guard_(env->be->device); \
  if (!gp_device_guard_.ok) return GP_E_HIP

int gp_obs_info(const gp_env* env, int* dtype, int* width) {
  if (!env || !env->be) {
    gp_set_error("null env handle");
    return GP_E_INVALID;
  }
  if (dtype) *dtype = env->be->obs_dtype;
  if (width) *width = env->be->obs_width;
  return GP_OK;
}

int64_t gp_num_envs(const gp_env* env) { return env && env->be ? env->be->B : -1; }

int gp_seed_words(gp_env* env, const uint32_t* entropy, int n_entropy, const uint32_t* spawn_key, int n_spawn) {
  GP_REQUIRE_ENV();
  std::vector<uint32_t> ent(entropy, entropy + (n_entropy > 0 ? n_entropy : 0));
  std::vector<uint32_t> sk(spawn_key, spawn_key + (n_spawn > 0 ? n_spawn : 0));
  if (ent.empty()) ent.push_back(0u);
  RngHost r = pcg64_from_seed(ent, sk);
  // Philox key for the counter mode: SeedSequence state words 8-9 (not used by PCG64's seeding).
  std::vector<uint64_t> w = seed_sequence_u64(ent, sk, 5);
  uint32_t key[2] = {(uint32_t)w[4], (uint32_t)(w[4] >> 32)};
  return env->be->seed(r, key);
}

int gp_seed(gp_env* env, uint64_t seed) {
  uint32_t words[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  return gp_seed_words(env, words, (seed >> 32) ? 2 : 1, nullptr, 0);
}

int gp_set_rng_state(gp_env* env, const uint64_t st[6]) {
  GP_REQUIRE_ENV();
  RngHost r;
  r.state = mk128(st[0], st[1]);
  r.inc = mk128(st[2], st[3]);
  r.has_u32 = (uint32_t)st[4];
  r.uinteger = (uint32_t)st[5];
  return env->be->set_rng_state(r);
}

int gp_get_rng_state(gp_env* env, uint64_t st[6]) {
  GP_REQUIRE_ENV();
  RngHost r;
  int e = env->be->get_rng_state(&r);
  st[0] = hi64(r.state);
  st[1] = lo64(r.state);
  st[2] = hi64(r.inc);
  st[3] = lo64(r.inc);
  st[4] = r.has_u32;
  st[5] = r.uinteger;
  return e;
}

int gp_reset(gp_env* env, void* obs, void* stream) {
  GP_REQUIRE_ENV();
  if (!obs) {
    gp_set_error("gp_reset: null obs");
    return GP_E_INVALID;
  }
  return env->be->reset(obs, (hipStream_t)stream);
}

int gp_step(gp_env* env, const void* actions, void* obs, float* rew, uint8_t* term, uint8_t* trunc, void* stream) {
  GP_REQUIRE_ENV();
  if (!actions || !obs || !rew || !term || !trunc) {
    gp_set_error("gp_step: null buffer");
    return GP_E_INVALID;
  }
  return env->be->step(actions, obs, rew, term, trunc, (hipStream_t)stream);
}

int gp_rollout(gp_env* env, int K, const void* actions, void* obs, float* rew, uint8_t* term, uint8_t* trunc,
               void* stream) {
  GP_REQUIRE_ENV();
  if (K < 0 || !actions || !obs || !rew || !term || !trunc) {
    gp_set_error("gp_rollout: bad arguments");
    return GP_E_INVALID;
  }
  if (K == 0) return GP_OK;
  return env->be->rollout(K, actions, obs, rew, term, trunc, (hipStream_t)stream);
}

struct gp_plan {
  gp_env* env;
  int K;
  const void* act;
  void* obs;
  float* rew;
  uint8_t* term;
  uint8_t* trunc;
  hipStream_t stream;
};

int gp_plan_create(gp_env* env, int K, const void* actions, void* obs, float* rew, uint8_t* term, uint8_t* trunc,
                   void* stream, gp_plan** out) {
  GP_REQUIRE_ENV();
  if (!out || K < 1 || !actions || !obs || !rew || !term || !trunc) {
    gp_set_error("gp_plan_create: bad arguments");
    return GP_E_INVALID;
  }
  *out = new gp_plan{env, K, actions, obs, rew, term, trunc, (hipStream_t)stream};
  return GP_OK;
}

int gp_plan_run(gp_plan* plan) {
  if (!plan || !plan->env || !plan->env->be) {
    gp_set_error("gp_plan_run: null plan");
    return GP_E_INVALID;
  }
  DeviceGuard guard(plan->env->be->device);  // the env's device, whatever the calling thread's current one is
  return plan->env->be->rollout(plan->K, plan->act, plan->obs, plan->rew, plan->term, plan->trunc, plan->stream);
}

void gp_plan_destroy(gp_plan* plan) { delete plan; }

int gp_get_state(gp_env* env, void* a, void* b, void* c, void* d, void* stream) {
  GP_REQUIRE_ENV();
  return env->be->get_state(a, b, c, d, (hipStream_t)stream);
}

int gp_set_state(gp_env* env, const void* a, const void* b, const void* c, const void* d, void* stream) {
  GP_REQUIRE_ENV();
  return env->be->set_state(a, b, c, d, (hipStream_t)stream);
}

int gp_set_replay(gp_env* env, const void* u, const void* i0, const void* i1, const void* f0, const void* f1) {
  GP_REQUIRE_ENV();
  return env->be->set_replay(u, i0, i1, f0, f1);
}

int gp_valid_cells(const gp_env* env, int which, int32_t* out, int cap) {
  if (!env || !env->be) {
    gp_set_error("null env handle");
    return GP_E_INVALID;
  }
  return env->be->valid_cells(which, out, cap);
}

#ifdef GP_STAMPS
// Diagnostic builds only (libgympo_amd_stamps.so): per-block per-step phase stamps of the fused kernel.
int gp_debug_stamps(gp_env* env, unsigned long long* out, int cap) {
  GP_REQUIRE_ENV();
  return env->be->debug_stamps(out, cap);
}
#endif

int gp_metrics(gp_env* env, double out[4]) {
  GP_REQUIRE_ENV();
  return env->be->metrics(out);
}

int gp_check(gp_env* env) {
  GP_REQUIRE_ENV();
  return env->be->check();
}

int gp_autotune(gp_env* env, int K, int reps, int* chosen) {
  GP_REQUIRE_ENV();
  return env->be->autotune(K, reps, chosen);
}

int gp_query(const gp_env* env, const char* key, int64_t* value) {
  if (!env || !env->be || !key || !value) {
    gp_set_error("gp_query: null argument");
    return GP_E_INVALID;
  }
  return env->be->query(key, value);
}

int gp_taxi_reset_distribution(const gp_env* env, double* out, int cap) {
  if (!env || !env->be) {
    gp_set_error("null env handle");
    return GP_E_INVALID;
  }
  return env->be->reset_distribution(out, cap);
}

int gp_taxi_render(gp_env* env, int n, int hansen_highlight, uint8_t* out, int32_t dims[4], void* stream) {
  GP_REQUIRE_ENV();
  if (!dims) {
    gp_set_error("gp_taxi_render: dims is required");
    return GP_E_INVALID;
  }
  return env->be->render(n, hansen_highlight, out, dims, (hipStream_t)stream);
}

int gp_set_profiling(gp_env* env, int enable) {
  GP_REQUIRE_ENV();
  env->be->timer.on = enable != 0;
  env->be->timer2.on = enable != 0;
  return GP_OK;
}

int gp_profile_read_resolver(gp_env* env, double* total_ms, int64_t* n_launches) {
  GP_REQUIRE_ENV();
  double ms = 0;
  int64_t n = 0;
  int e = env->be->timer2.read(&ms, &n);
  if (total_ms) *total_ms = ms + env->be->timer2.acc_ms;
  if (n_launches) *n_launches = n + env->be->timer2.acc_n;
  env->be->timer2.acc_ms = 0;
  env->be->timer2.acc_n = 0;
  return e;
}

int gp_profile_read(gp_env* env, double* total_ms, int64_t* n_launches) {
  GP_REQUIRE_ENV();
  double ms = 0;
  int64_t n = 0;
  int e = env->be->timer.read(&ms, &n);
  if (total_ms) *total_ms = ms + env->be->timer.acc_ms;
  if (n_launches) *n_launches = n + env->be->timer.acc_n;
  env->be->timer.acc_ms = 0;
  env->be->timer.acc_n = 0;
  return e;
}

int gp_pcg64_seed_state(const uint32_t* entropy, int n_entropy, const uint32_t* spawn_key, int n_spawn,
                        uint64_t out[6]) {
  std::vector<uint32_t> ent(entropy, entropy + (n_entropy > 0 ? n_entropy : 0));
  std::vector<uint32_t> sk(spawn_key, spawn_key + (n_spawn > 0 ? n_spawn : 0));
  if (ent.empty()) ent.push_back(0u);
  RngHost r = pcg64_from_seed(ent, sk);
  out[0] = hi64(r.state);
  out[1] = lo64(r.state);
  out[2] = hi64(r.inc);
  out[3] = lo64(r.inc);
  out[4] = r.has_u32;
  out[5] = r.uinteger;
  return GP_OK;
}

int gp_argmax_multinomial_distribution(int m, int n, double* out) {
  if (m < 1 || n < 1 || !out) {
    gp_set_error("gp_argmax_multinomial_distribution: bad arguments");
    return GP_E_INVALID;
  }
  std::vector<double> p = argmax_multinomial_distribution(m, n);
  for (int k = 0; k < m; ++k) out[k] = p[k];
  return m;
}

}  // extern "C"
