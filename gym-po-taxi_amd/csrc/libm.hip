// libm.hip — host copies of the device restatements of C library functions (gp_libm.h), for the CPU tests that pin
// them against this machine's libm; and the host copy of the Philox block (gp_common.h) for the oracle's check.
#include <cmath>

#include "gp_internal.h"
#include "gp_libm.h"

extern "C" int gp_exp_libm(const double* x, double* out, int64_t n, int fma) {
  if (!x || !out || n < 0) {
    gp_set_error("gp_exp_libm: bad arguments");
    return GP_E_INVALID;
  }
  for (int64_t i = 0; i < n; ++i) out[i] = fma ? gp_libm::exp<true>(x[i]) : gp_libm::exp<false>(x[i]);
  return GP_OK;
}

// The host libm's exp build: probe seeded inputs until 64 of them give different results under the two
// restatements, then ask libm. Cached for the process.
extern "C" int gp_exp_host_variant(void) {
  static int variant = -2;
  if (variant != -2) return variant;
  bool is_fma = true, is_plain = true;
  int diffs = 0;
  uint64_t s = 0x9E3779B97F4A7C15ull;
  double (*volatile libm_exp)(double) = ::exp;  // the library's symbol, never a compiler builtin
  for (int i = 0; i < (1 << 20) && diffs < 64; ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    const double x = -60.0 + 80.0 * (double)(s >> 11) * 0x1.0p-53;
    const double a = gp_libm::exp<true>(x), b = gp_libm::exp<false>(x);
    if (a == b) continue;
    ++diffs;
    const double r = libm_exp(x);
    is_fma &= r == a;
    is_plain &= r == b;
  }
  variant = diffs == 0 ? -1 : (is_fma ? 1 : (is_plain ? 0 : -1));
  return variant;
}

// Philox4x32-R blocks (gp_common.h philox4x32<R>, R = 7 or 10) of n counters ctr[6 i ..] = {c0, c1, c2, c3, k0, k1}
// into out[4 i ..]: the header the kernels inline, compiled for the host.
extern "C" int gp_philox_blocks(const uint32_t* ctr, int rounds, uint32_t* out, int64_t n) {
  if (!ctr || !out || n < 0 || (rounds != 7 && rounds != 10)) {
    gp_set_error("gp_philox_blocks: bad arguments");
    return GP_E_INVALID;
  }
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t* c = ctr + 6 * i;
    const Philox4 r = rounds == 7 ? philox4x32<7>(c[0], c[1], c[2], c[3], c[4], c[5])
                                  : philox4x32<10>(c[0], c[1], c[2], c[3], c[4], c[5]);
    for (int j = 0; j < 4; ++j) out[4 * i + j] = r.x[j];
  }
  return GP_OK;
}
