// libm.hip — host copies of the device restatements of C library functions (gp_libm.h), for the CPU tests that pin
// them against this machine's libm.
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
