// libm.hip — host copies of the device restatements of C library functions (gp_libm.h), for the CPU tests that pin
// them against this machine's libm.
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
