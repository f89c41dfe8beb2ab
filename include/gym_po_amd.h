/*
 * gym_po_amd — C ABI of the MI355X-native vectorised env engine for gym_po's POMDP gridworlds.
 *
 * This is the drop-in boundary: a plain C shared library (libgympo_amd.so; no torch types,
 * plain pointers and sizes). Every device pointer below is a HIP device pointer owned by the
 * CALLER (e.g. a torch-ROCm tensor's data_ptr()); env state and lookup tables are owned by the
 * handle. All calls are asynchronous on the given hipStream_t (passed as void*; NULL = the
 * default stream) unless documented otherwise. A handle is not re-entrant; use one per
 * stream/thread. Every entry point returns 0 on success, a negative GP_E* code otherwise, and
 * gp_last_error() returns thread-local text for the last failure.
 *
 * Reference interfaces replaced (paths relative to DavidSlayback/gym-po-taxi):
 *   gp_create(GP_KIND_GRID)   MultistoryFourRoomsEnv.__init__   gym_po/envs/rooms/msrooms.py:266-367
 *                             RoomsEnv.__init__                  gym_po/envs/rooms/rooms.py:84-175
 *   gp_create(GP_KIND_TAXI)   TaxiVecEnv.__init__                gym_po/envs/extended_taxi.py:158-230
 *   gp_create(GP_KIND_CROOMS) CRoomsEnv.__init__                 gym_po/envs/rooms/crooms.py:104-244
 *   gp_create(GP_KIND_ANTTAG) AntTagEnv task rules (grid restatement, build-defined)
 *                                                                gym_po/envs/ant_tag.py:88-157
 *   gp_seed / gp_seed_words   gymnasium Env.reset(seed=) -> seeding.np_random(seed)
 *                             (msrooms.py:376, rooms.py:184, extended_taxi.py:239, crooms.py:246-249)
 *   gp_reset                  *.reset()      msrooms.py:369-381, rooms.py:177-189,
 *                                            extended_taxi.py:232-242, crooms.py:251-266
 *   gp_step                   *.step()       msrooms.py:390-413, rooms.py:198-222,
 *                                            extended_taxi.py:244-287, crooms.py:276-298
 *   gp_rollout                K x step() in one call (agent rollout loop, tester.py:24-26)
 *   gp_get_state/gp_set_state the env's array state (agent_zyx/goal_zyx/elapsed, s/elapsed/...)
 *   gp_set_replay             replaces env.np_random's draws with pre-decided per-env values
 */
#ifndef GYM_PO_AMD_H
#define GYM_PO_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GP_ABI_VERSION 1

/* ---- status codes ---- */
#define GP_OK 0
#define GP_E_INVALID (-1)   /* bad argument / config (reference would raise)           */
#define GP_E_HIP (-2)       /* HIP runtime error                                         */
#define GP_E_UNSUPPORTED (-3)/* mode not available for this env kind                     */
#define GP_E_STATE (-4)     /* call order (e.g. step before reset)                       */
#define GP_E_DEVICE (-5)    /* a device-side failure of an earlier asynchronous launch (a persistent
                               kernel's cross-block wait timed out): outputs and env state since the
                               last seed are invalid; reported by gp_check / gp_metrics /
                               gp_get_rng_state, cleared by reseeding                          */

/* ---- env kinds ---- */
#define GP_KIND_GRID 1   /* FourRooms (multistory) and ROOMS: discrete cell gridworlds */
#define GP_KIND_TAXI 2
#define GP_KIND_CROOMS 3
#define GP_KIND_ANTTAG 4

/* ---- RNG modes ---- */
#define GP_RNG_NUMPY 0   /* seed-identical to numpy Generator(PCG64(SeedSequence(seed))): GRID, CROOMS, TAXI */
#define GP_RNG_PHILOX 1  /* counter-based Philox4x32-10 keyed by (seed, env, step): fusable rollouts */
#define GP_RNG_REPLAY 2  /* pre-decided per-env draws supplied by gp_set_replay each step       */

/* ---- observation dtypes reported by gp_obs_info ---- */
#define GP_DTYPE_I32 0
#define GP_DTYPE_U8 1
#define GP_DTYPE_F32 2
#define GP_DTYPE_F64 3

/* ---- GRID config (FourRooms / ROOMS) ---- */
#define GP_FLAVOR_ROOMS 0      /* rooms.py: wall == -1, binary Hansen (observations.py:44-71)       */
#define GP_FLAVOR_MULTISTORY 1 /* msrooms.py: wall == 0, stairs 2/3, ternary Hansen (msrooms.py:162) */

#define GP_OBS_HANSEN 0     /* scalar Hansen index x goal multiplier            int32 [B]       */
#define GP_OBS_HANSEN_VEC 1 /* per-direction codes                              uint8 [B,n]     */
#define GP_OBS_TABLE 2      /* table[agent] + table2[goal] (mdp / room scalars)  int32 [B]       */
#define GP_OBS_COORDS 3     /* agent (and goal) coordinates                     int32 [B,d|2d]  */
#define GP_OBS_WINDOW 4     /* n x n local window (observations.py:74-103)      uint8 [B,n,n]   */
#define GP_OBS_ONEHOT 5     /* one-hot of the scalar obs (taxi)                 uint8 [B,space] */
#define GP_OBS_F32 6        /* float observation (crooms coords)                float [B,d]     */

typedef struct gp_grid_config {
  int32_t flavor;          /* GP_FLAVOR_*                                                       */
  int32_t depth, height, width; /* grid shape (depth = floors; 1 for ROOMS)                     */
  const int32_t* cells;    /* [depth*height*width] C-order cell values (room id / walk code)    */
  int32_t n_actions;       /* 4 (cardinal N,E,S,W) or 8 (ordinal N,NE,...,NW) (action_utils.py)  */
  double action_failure_probability;
  int32_t obs_kind;        /* GP_OBS_HANSEN / _HANSEN_VEC / _TABLE / _COORDS / _WINDOW          */
  int32_t obs_dirs;        /* Hansen directions: 4 or 8                                         */
  int32_t obs_goal;        /* include goal information (obs_type contains "goal")               */
  int32_t obs_n;           /* window size for GP_OBS_WINDOW                                     */
  const int32_t* obs_table;  /* GP_OBS_TABLE: per-cell value for the agent    [ncells]          */
  const int32_t* obs_table2; /* GP_OBS_TABLE: per-cell value for the goal (may be NULL) [ncells] */
  int32_t fixed_goal;      /* flat cell index, or -1 = random over valid goal cells; a value
                              >= ncells is an unreachable goal (ROOMS "32" ENDS quirk)          */
  int32_t fixed_agent;     /* flat cell index, or -1 = random over valid agent cells            */
  int32_t time_limit;      /* truncated = elapsed > time_limit                                  */
  float step_reward, wall_reward, goal_reward;
} gp_grid_config;

typedef struct gp_taxi_config {
  int32_t rows, cols;      /* navigable grid (5x5 TAXI_MAP, 8x8 EXTENDED_TAXI_MAP)              */
  int32_t desc_rows, desc_cols;
  const char* desc;        /* [desc_rows*desc_cols] bordered char map ('|' walls, ':' pseudo)   */
  int32_t pseudo_walls;    /* 1 if the map uses ':' columns (cc(r,c) = (r+1, 2c+1))            */
  int32_t n_locs;
  const int32_t* locs;     /* [n_locs*2] (row, col) of R,G,Y,B in row-major order               */
  int32_t num_passengers;
  int32_t time_limit;
  int32_t obs_kind;        /* GP_OBS_TABLE (raw state s, extended_taxi.py:368) or GP_OBS_HANSEN
                              ((hansen[r,c]*(L+1)+p)*L+d, extended_taxi.py:370-372)              */
  int32_t one_hot;         /* 1: emit that index one-hot, uint8 [B, n_obs] (GP_OBS_ONEHOT layout;
                              a build-side encoding, the reference has none)                     */
  float reward_goal, reward_bad, reward_any;
} gp_taxi_config;

typedef struct gp_crooms_config {
  int32_t height, width;
  const int32_t* cells;    /* room-id grid, wall == -1 (layouts.py np_to_grid)                    */
  int32_t use_velocity;    /* crooms.py:304-310: v = clip(v + a, +-5), proposed = agent + v        */
  double cell_size;        /* >= 1 (smaller cells index past the grid: the reference raises)       */
  int32_t action_kind;     /* 0 = continuous (y,x) [B,2]; 4 / 8 = discrete cardinal / ordinal [B]  */
  int32_t action_f64;      /* continuous actions are float64 [B,2] (1) or float32 [B,2] (0)        */
  double action_failure_probability;
  double action_std, action_power;
  int32_t obs_kind;        /* GP_OBS_F32 (vector mdp: agent [+ goal] y,x) or GP_OBS_HANSEN /
                              _HANSEN_VEC / _TABLE / _WINDOW evaluated on floor(coord / cell_size)  */
  int32_t obs_f64;         /* GP_OBS_F32 emitted as float64 (GP_DTYPE_F64) instead of float32       */
  int32_t obs_dirs, obs_goal, obs_n;
  const int32_t* obs_table;  /* GP_OBS_TABLE: per-cell value for the agent [height*width]         */
  const int32_t* obs_table2; /* GP_OBS_TABLE: per-cell value for the goal (may be NULL)           */
  int32_t goal_fixed;      /* 1: goal cell (goal_y, goal_x) every reset (may lie off the grid)    */
  int32_t goal_y, goal_x;
  int32_t agent_fixed;     /* 1: agent cell (agent_y, agent_x) every reset                         */
  int32_t agent_y, agent_x;
  int32_t time_limit;
  float step_reward, wall_reward, goal_reward;
  double goal_threshold;   /* terminated = ||agent - goal||_2 <= goal_threshold (float64)         */
} gp_crooms_config;

typedef struct gp_anttag_config {
  int32_t size;            /* arena cells per side (interior)                                   */
  int32_t tag_radius2;     /* squared Chebyshev/Euclid radius (cells^2) for a tag              */
  int32_t visible_radius2; /* squared radius under which the target is observed                */
  int32_t min_start_dist2; /* squared minimum start separation                                 */
  int32_t time_limit;
  float tag_reward, step_reward;
} gp_anttag_config;

typedef struct gp_env gp_env;

const char* gp_last_error(void);
int gp_abi_version(void);

/* kind = GP_KIND_*, config points to the matching gp_*_config. Tables are built and uploaded
 * to `device` synchronously. rng_mode = GP_RNG_*. */
int gp_create(int kind, const void* config, int64_t num_envs, int device, int rng_mode, gp_env** out);
void gp_destroy(gp_env* env);

/* obs layout: dtype = GP_DTYPE_*, width = elements per env (1 for scalar obs). */
int gp_obs_info(const gp_env* env, int* dtype, int* width);
int64_t gp_num_envs(const gp_env* env);

/* numpy-compatible seeding: SeedSequence(entropy, spawn_key) -> PCG64 (and the Philox key).
 * entropy = little-endian uint32 words of a non-negative integer (numpy's convention). */
int gp_seed_words(gp_env* env, const uint32_t* entropy, int n_entropy, const uint32_t* spawn_key, int n_spawn);
int gp_seed(gp_env* env, uint64_t seed);
/* raw PCG64 state: {state_hi, state_lo, inc_hi, inc_lo, has_uint32, uinteger}. get syncs. */
int gp_set_rng_state(gp_env* env, const uint64_t st[6]);
int gp_get_rng_state(gp_env* env, uint64_t st[6]);

/* Reset every env (reset()), writing the initial observation to `obs` (device). */
int gp_reset(gp_env* env, void* obs, void* stream);

/* One batched step with same-step autoreset. actions: int32 [B] (discrete) or float [B,2]
 * (continuous C-ROOMS); obs as gp_obs_info; rew float [B]; term/trunc uint8 [B]. */
int gp_step(gp_env* env, const void* actions, void* obs, float* rew, uint8_t* term, uint8_t* trunc,
            void* stream);

/* K consecutive steps. actions [K,B(,2)], outputs [K,B,...]. Philox mode, and numpy mode on GRID
 * (persistent kernel with a per-step grid exchange; 16-B aligned buffers, B % 4 == 0), fuse the K
 * steps in one launch with the state in registers; other cases issue K step launches. */
int gp_rollout(gp_env* env, int K, const void* actions, void* obs, float* rew, uint8_t* term, uint8_t* trunc,
               void* stream);
/* A prepared gp_rollout (the agent loop's allocation-free hot path, bench.py's timed call): the arguments are
 * validated and bound once; gp_plan_run(plan) enqueues the K steps with nothing to marshal per call (one
 * pointer across the FFI instead of eight). The buffers must outlive the plan; gp_plan_destroy frees it. */
typedef struct gp_plan gp_plan;
int gp_plan_create(gp_env* env, int K, const void* actions, void* obs, float* rew, uint8_t* term, uint8_t* trunc,
                   void* stream, gp_plan** out);
int gp_plan_run(gp_plan* plan);
void gp_plan_destroy(gp_plan* plan);

/* Canonical state (device pointers, int32 unless noted). GRID: agent cell, goal cell, elapsed
 * [B] each. TAXI: s, elapsed, n_dropoffs. CROOMS: agent yx f64[B,2], goal cell yx i32[B,2],
 * velocity f64[B,2], elapsed i32[B]. ANTTAG: agent cell, target cell, elapsed. */
int gp_get_state(gp_env* env, void* a, void* b, void* c, void* d, void* stream);
int gp_set_state(gp_env* env, const void* a, const void* b, const void* c, const void* d, void* stream);

/* Replay mode: device pointers holding this step's pre-decided per-env draws (read by the next
 * gp_step). GRID: uniform k53 uint64 [B] (u = k*2^-53), goal index int32 [B], agent index
 * int32 [B] (indices into the valid-cell lists). TAXI: reset state int32 [B], passenger/dest
 * pair int32 [B] (p*n_locs+d). CROOMS: action noise f64 [B,2] (the value numpy's
 * normal(scale=action_std) returned), wall noise f64 [B,2] (normal(scale=0.5)), goal/agent index
 * int32 [B] each, uniform k53 uint64 [B] for discrete action failures. */
int gp_set_replay(gp_env* env, const void* u, const void* i0, const void* i1, const void* f0, const void* f1);

/* Valid-cell lists (host copies) used by the index draws: which = 0 goal, 1 agent. */
int gp_valid_cells(const gp_env* env, int which, int32_t* out, int cap);

/* On-device episode statistics since the last gp_reset (syncs): {episodes, return_sum,
 * length_sum, env_steps}. */
int gp_metrics(gp_env* env, double out[4]);

/* Syncs the handle's device and returns GP_E_DEVICE if any launch since the last seed failed on the
 * device (numpy-mode GRID: a persistent kernel's cross-block wait timed out; any kind: an action outside
 * [-n, n) was given, where the reference raises IndexError at msrooms.py:400 / rooms.py:208 /
 * extended_taxi.py:248 — the device clamps it and flags the handle), else GP_OK. The
 * asynchronous step/rollout calls cannot report such failures themselves; gp_metrics and
 * gp_get_rng_state run the same check. (No reference counterpart: numpy steps are synchronous.) */
int gp_check(gp_env* env);
/* Chooses, on this handle's device, the faster of interchangeable kernels for launches of K steps. Numpy-mode GRID
 * with both the windowed (wgrid_rollout) and the fused (grid_rollout_numpy) kernel eligible: their results are
 * identical, and which is faster at short launches differs between MI355X boards. Times `reps` K-step launches of
 * each on scratch actions / outputs from the current state, restores that state exactly (env state, stream
 * state, metrics), and sends K-step launches to the faster. *chosen (host, may be NULL) = 1 windowed, 0 fused,
 * -1 not applicable (other kinds / modes: a no-op). After gp_reset; syncs. (No reference counterpart.) */
int gp_autotune(gp_env* env, int K, int reps, int* chosen);
/* Introspection of a handle (host-only, no sync): key = "num_envs", "rng_mode", and for GRID
 * "fused_blocks" (persistent grid size of the fused numpy rollout, 0 = not eligible),
 * "fused_tiles_per_block", "fused_staged" (1 = LDS-staged outputs + store waves),
 * "fused_tile_envs". Unknown keys return GP_E_INVALID. */
int gp_query(const gp_env* env, const char* key, int64_t* value);
/* ---- the normal sampler of rng_mode=philox (C-ROOMS noise), diagnostics ----
 * Replaces numpy's Generator.standard_normal (numpy/random/src/distributions/distributions.c,
 * random_standard_normal; the reference draws rng.normal at gym_po/envs/rooms/crooms.py:175-178, :324).
 * gp_standard_normal_words: numpy's algorithm (256-layer ziggurat) over the caller's u64 word stream, in
 *   order, on one device lane: words device u64[nwords], out device f64[n] (NaN for every normal whose
 *   words run out, mid-draw included),
 *   *used (host) = words consumed. Over numpy's raw PCG64 words it returns numpy's normals.
 * gp_normal_tail_counts: n normals of the philox-mode sampler keyed by `key` (gp_seed's Philox key words),
 *   never stored: counts[j] = #{|z| > thr[j]} (host arrays, nthr <= 8), moments = {sum z, sum z^2}. Syncs. */
int gp_standard_normal_words(const uint64_t* words, int64_t nwords, double* out, int64_t n, int64_t* used,
                             void* stream);
int gp_normal_tail_counts(uint64_t key, int64_t n, const double* thr, int nthr, uint64_t* counts,
                          double moments[2], void* stream);

/* Device-side start-state law of TAXI resets (host copy): P(state index k) over valid states. */
int gp_taxi_reset_distribution(const gp_env* env, double* out, int cap);

/* rgb_array frames of TAXI envs 0..n-1 (replaces TaxiVecEnv.render(idx=arange(n)), extended_taxi.py:289-309,
 * up to and including str_map_to_img's colouring and Hansen highlight :126-142 and tile_images
 * render_utils.py:63-88): uint8 RGB, frames tiled ceil(sqrt(n)) x ceil(n / ceil(sqrt(n))), zero padding.
 * dims (host, out) = {rows, cols, frame_rows, frame_cols}; out (device, rows*cols*3) may be NULL to query dims.
 * Other env kinds: GP_E_UNSUPPORTED (the reference renders none of them). Asynchronous on `stream`. */
int gp_taxi_render(gp_env* env, int n, int hansen_highlight, uint8_t* out, int32_t dims[4], void* stream);
/* cv2.resize(src, (dw, dh), interpolation=cv2.INTER_AREA) for uint8 sh x sw x ch device images when at least
 * one axis is enlarged (the resize of str_map_to_img, extended_taxi.py:144-146): OpenCV's generic resize path
 * restated (cv2 is absent here: parity unpinned). dst rows are dst_pitch bytes apart. Synchronises `stream`. */
int gp_resize_area_u8(const uint8_t* src, int sh, int sw, int ch, uint8_t* dst, int dh, int dw, int dst_pitch,
                      void* stream);

/* Kernel timing: when enabled, hipEvents bracket every launch of the env's step kernel on its
 * stream; gp_profile_read syncs and returns the summed kernel time (ms) and launch count since
 * the last read (then clears). Used by bench.py for the live roofline measurement. */
int gp_set_profiling(gp_env* env, int enable);
int gp_profile_read(gp_env* env, double* total_ms, int64_t* n_launches);
/* Same for the numpy-mode reset resolver kernel that follows each step kernel. */
int gp_profile_read_resolver(gp_env* env, double* total_ms, int64_t* n_launches);

/* ---- diagnostics (never needed in production; no reference counterpart) ----
 * Process-wide test / tuning knobs, read by gp_create (handles created earlier keep their values):
 *   "disable_fused" (GRID numpy mode: 1 = the two-kernel path only; CROOMS numpy mode: 1 = two launches per
 *   draw call), "no_staging" (1 = the fused kernel's env waves store outputs directly), "xmode" (fused exchange variant, default 1), "spin_limit" (polls
 *   before a cross-block wait gives up, 0 = default), "fault_block" (this block never publishes: forces
 *   the timeout path; -1 = off), "fused_tile" (GRID fused kernel envs per tile: 512, 1024 or 2048; 0 = by
 *   size), "no_spw" (GRID fused kernel: 1 = no speculative word windows), "generic_kernels" (CROOMS: 1 = the
 *   generic philox rollout even where a compile-time-specialised one exists), "no_wgrid" (GRID numpy mode: 1 =
 *   never the windowed kernel csrc/wgrid.hip), "wg_halo" (its window halo: 256 or 512 draws), "wg_bias" (added
 *   to its predicted reset count: forces window regenerations), "wg_tmode" (its timing-study variants, TM_* in
 *   csrc/wgrid.hip; results invalid for some). gp_debug_reset restores the defaults. Unknown key: GP_E_INVALID. */
int gp_debug_set(const char* key, int64_t value);
void gp_debug_reset(void);

/* ---- host-only helpers (no device needed) ---- */
/* PCG64 state {state_hi, state_lo, inc_hi, inc_lo, has_uint32, uinteger} that numpy's
 * Generator(PCG64(SeedSequence(entropy, spawn_key))) starts from. */
int gp_pcg64_seed_state(const uint32_t* entropy, int n_entropy, const uint32_t* spawn_key, int n_spawn,
                        uint64_t out[6]);
/* log1p(-u[i]) for u in [0, 1) exactly as the C library computes it (glibc 2.35 __log1p restated, the version
 * the C-ROOMS exact mode's ziggurat tail uses on the device: numpy's random_standard_normal calls npy_log1p ->
 * libm, distributions.c). Host-only check entry for the CPU tests. */
int gp_zig_log1p_neg(const double* u, double* out, int64_t n);
/* exp(x[i]) exactly as the C library computes it (glibc 2.35 __exp restated, csrc/gp_libm.h: the device copy the
 * exact-stream paths use where numpy calls libm's exp, e.g. random_binomial_inversion's q^n = exp(n log q),
 * distributions.c). fma != 0: the -mfma build glibc selects on CPUs with FMA (x86-64 ifunc), else the plain one.
 * Host-only check entry for the CPU tests. */
int gp_exp_libm(const double* x, double* out, int64_t n, int fma);
/* Philox4x32-R blocks (R = rounds: 7 or 10) of n counters ctr[6 i .. 6 i + 5] = {c0, c1, c2, c3, k0, k1} into
 * out[4 i .. 4 i + 3], computed by the header the philox-mode kernels inline (gp_common.h philox4x32<R>).
 * Host-only check entry for the CPU tests (oracle/philox.py is checked against it). */
int gp_philox_blocks(const uint32_t* ctr, int rounds, uint32_t* out, int64_t n);
/* Which build of the C library's exp this host runs (the one numpy's distributions get): 1 = the -mfma build,
 * 0 = the plain build, -1 = neither restatement matches (exact-stream exp-dependent branches then follow the FMA
 * build: parity unpinned). Decided once per process by comparing libm with both restatements where they differ;
 * the exact-stream kernels (Taxi numpy-mode resets, C-ROOMS exact-mode wedge) use that build on the device. */
int gp_exp_host_variant(void);
/* P(argmax = k), k < m, for Multinomial(n, uniform over m) counts, ties to the first index:
 * the law of TaxiVecEnv._reset_mask (extended_taxi.py:344-352). Returns m. */
int gp_argmax_multinomial_distribution(int m, int n, double* out);

#ifdef __cplusplus
}
#endif
#endif /* GYM_PO_AMD_H */
