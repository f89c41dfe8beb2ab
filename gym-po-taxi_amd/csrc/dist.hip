// dist.hip — host: exact start-state law of TaxiVecEnv resets.
//
// extended_taxi.py:344-352 resets with  s = multinomial(ns, uniform over the V valid states).argmax()
// i.e. throw n = ns balls into V bins uniformly and take the first fullest bin. The law of that
// argmax is a fixed distribution over the V valid states (low indices ~2x, high ~0.5x uniform),
// computed here once, exactly up to float64 rounding, by Poissonization: with N_j iid
// Poisson(n/V), the counts conditioned on sum = n are that multinomial, hence
//   P(argmax = k) = sum_c pois(c) [x^(n-c)] Q_{c-1}(x)^k Q_c(x)^(V-1-k) / P(sum = n),
//   Q_b(x) = sum_{i<=b} pois(i) x^i.
// The device samples this law with one uniform + a CDF search instead of n categorical draws.
#include <cmath>
#include <vector>

#include "gp_internal.h"

std::vector<double> argmax_multinomial_distribution(int m, int n) {
  const double lam = (double)n / m;
  std::vector<double> pois(n + 1);
  for (int i = 0; i <= n; ++i) pois[i] = std::exp(-lam + i * std::log(lam) - std::lgamma(i + 1.0));
  const double p_sum_n = std::exp(-n + n * std::log((double)n) - std::lgamma(n + 1.0));
  std::vector<double> out(m, 0.0);
  for (int c = 1; c <= n; ++c) {
    if (c > lam + 3 && pois[c] / p_sum_n * m < 1e-19) break;
    const int deg = n - c;
    if (deg < 0) break;
    // pw_lo[k] = Q_{c-1}^k, pw_hi[k] = Q_c^k, truncated at degree deg
    std::vector<double> lo((size_t)m * (deg + 1), 0.0), hi((size_t)m * (deg + 1), 0.0);
    lo[0] = hi[0] = 1.0;
    for (int k = 1; k < m; ++k) {
      const double* pl = &lo[(size_t)(k - 1) * (deg + 1)];
      const double* ph = &hi[(size_t)(k - 1) * (deg + 1)];
      double* ql = &lo[(size_t)k * (deg + 1)];
      double* qh = &hi[(size_t)k * (deg + 1)];
      const int top = std::min(deg, k * c);
      for (int i = 0; i <= top; ++i) {
        double sl = 0.0, sh = 0.0;
        const int jmax = std::min(i, c);
        for (int j = 0; j <= jmax; ++j) {
          if (j < c) sl += pl[i - j] * pois[j];
          sh += ph[i - j] * pois[j];
        }
        ql[i] = sl;
        qh[i] = sh;
      }
    }
    for (int k = 0; k < m; ++k) {
      const double* a = &lo[(size_t)k * (deg + 1)];
      const double* b = &hi[(size_t)(m - 1 - k) * (deg + 1)];
      double s = 0.0;
      for (int i = 0; i <= deg; ++i) s += a[i] * b[deg - i];
      out[k] += pois[c] * s;
    }
  }
  for (double& v : out) v /= p_sum_n;
  return out;
}
