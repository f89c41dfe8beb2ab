// grid_shared.h — device-side structures shared by the GRID backend (grid.hip) and the windowed numpy-exact
// rollout (wgrid.hip): the numpy-mode control block, the per-block metric slots, and the windowed kernel's
// parameter block. Not part of the C ABI.
#pragma once
#include "gp_common.h"

// numpy-mode RNG state between launches (one per handle, device memory).
struct alignas(64) GridCtl {
  uint64_t s_hi, s_lo, inc_hi, inc_lo;  // numpy-mode PCG64 state at step start, increment
  uint32_t has_u32, uinteger;           // numpy's buffered 32-bit half
  uint32_t epoch;                       // K2 launches so far (tags the per-block flags)
  uint32_t err;                         // bit0: spin timeout
  uint32_t b_total;                     // resets resolved by the last K2 (diagnostic)
  uint32_t step;                        // fused kernel: its own steps taken (its granule tags; only fused launches
                                        //   advance it, so its steps stay contiguous when windowed launches interleave)
  uint32_t fb_last;                     // fused kernels: resets b of the last step (next launch's window centre)
  uint32_t wstep;                       // windowed kernel: its own steps taken (its granule tags)
};

// Per-block metric accumulators (each persistent block owns one slot).
struct alignas(32) MetricSlot {
  double return_sum;
  unsigned long long episodes, length_sum, env_steps;
};

// ---------------------------------------------------------------- windowed fused rollout (wgrid.hip) ----
// The envs are cut into G blocks of E = 512 * NS consecutive envs (one workgroup per CU). Parameters live in
// device memory (WgParams, refreshed on every seed); the launch passes a pointer and the per-call buffers.
constexpr int WG_HMAX = 512;  // largest halo (u64 draws on each side of a predicted window)

struct WgLds {  // byte offsets of the tables in the LDS image (WgParams::limg, copied verbatim into LDS)
  int32_t j32, jt8, move, thr, ocell, avalid, total;
};

struct WgParams {
  int32_t B, G, E, NS;          // envs, blocks, envs per block, env slots per env lane (E / 512)
  int32_t nact, ncells, n_agent, goal;
  uint32_t thr_agent;           // Lemire rejection threshold of choice(n_agent)
  int32_t time_limit, halo;     // episode limit; window halo H (u64 draws each side, multiple of 256, <= WG_HMAX)
  float r_step, r_wall, r_goal;
  uint32_t spin_limit;          // polls before a cross-block wait gives up (flags GridCtl::err)
  int32_t fault_block;          // test knob: this block never publishes (-1 off)
  int32_t rw_words;             // 64-word rows of a window: (E + 2H) / 64
  int32_t fill_row0[8], fill_rows[8];  // env wave w fills rows fill_row0[w] .. + fill_rows[w] - 1 of each window
  int32_t wg_bias;              // test knob: added to the predicted reset count (forces window misses); 0
  int32_t tmode;                // timing-study knob (gp_debug_set wg_tmode; 0 in production): see wgrid.hip TM_*
  WgLds lds;
  const char* limg;             // [lds.total] LDS image of the tables
  // Per-lane / per-block constant jumps, all applied to S(x_t), the state at a step's start (B = num envs):
  const PcgJump* jlane;         // [512][2]: by 64 fill_row0[w] + lane (lg = 64 w + lane: the lane's first window word from
                                //   the window base) and by B + 32 lg + 1 (coarse state lg)
  const PcgJump* jrej;          // [G][64]: by B + 62 beta + l + 1 (rejection-check slice of block beta, lane l)
  const PcgJump* jblk;          // [G][2]: by B + E beta - H (beta > 0; B for beta 0): the next window's base after
                                //   the choice() draws; by E beta - H + 1 (beta > 0; 0 for beta 0): a launch's first
  const PcgJump* jfirst;        // [2][512]: by 1 + lg (block 0) / by H + lg (blocks > 0) from the first window's base:
                                //   a launch's step-0 word of env slot 0 of lane lg
  const PcgJump* jt64;          // radix-64 general jump tables (JT_LEVELS x 64) for the rare paths
  PcgJump jB, jrow, j512;       // jump by B (random(B)), by 64 (a lane's next window word: the next row), by 512 (the
                                //   next env slot's step-0 word)
  GridCtl* ctl;
  MetricSlot* mslot;            // [G]
  uint32_t* ae;                 // [B] agent cell | elapsed << 16
  uint64_t* slots;              // [2 step parities][2 round parities][G] tagged granules
  unsigned long long* dbg;      // GP_STAMPS builds: [G][1024] step stamps (wgrid.hip ST_*), then [G][8] launch stamps
};

struct WgArgs {  // one launch: K steps, caller-owned action [K][B] and output [K][B] buffers
  const WgParams* P;
  int32_t K;
  const int32_t* act;
  int32_t* obs;
  float* rew;
  uint8_t* term;
  uint8_t* trunc;
};

// Dynamic LDS bytes of a launch (tables + window + coarse states + staging).
__host__ __device__ constexpr int wg_dyn_bytes(int tables, int E, int H) {
#ifndef WG_NSTG
#define WG_NSTG 3
#endif
  return tables + (E + 2 * H) * 8 + 2 * 512 * 16 + WG_NSTG * E * 4;
}
// Launch on `s` (host; csrc/wgrid.hip). Returns hipError_t as int.
int wgrid_launch(const WgArgs& a, int NS, int NA, int G, size_t dyn_lds, hipStream_t s);
// Can this device run a block of the windowed kernel with `dyn_lds` dynamic LDS? (occupancy >= 1)
int wgrid_fits(int NS, int NA, size_t dyn_lds);
