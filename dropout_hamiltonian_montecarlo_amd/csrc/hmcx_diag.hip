// hmcx_diag.hip — cross-chain convergence diagnostics on the device: per parameter,
// R̂ from per-chain moments, split-R̂ and the bulk effective sample size from the gathered thinned
// traces, computed where the RCCL all-gather leaves them (include/hmcx.h hmcx_chain_diagnostics).
//
// The reference has no diagnostics (its multi-chain modules concatenate the workers' posteriors,
// hamiltonian/inference/cpu/sghmc_multicore.py:86-94; the reader is hmc.py:132-138).  Definitions
// (BDA3 §11.4-11.5), the same as the host implementation diagnostics.py:
//   split-R̂: chains split in halves (first ⌊T/2⌋ and last ⌊T/2⌋ draws), m = 2C sequences of n draws;
//            W = mean of the sequences' variances (ddof 1), B = n·var(sequence means, ddof 1),
//            R̂ = sqrt(((n − 1)/n·W + B/n) / W)
//   ESS:     ρ_t = 1 − (W − mean_c acov_c(t)) / var⁺, var⁺ = (n − 1)/n·W + var(means); acov the biased
//            autocovariance of each sequence; Geyer's initial positive, monotone sequence over lag
//            pairs; ESS = m·n / max(τ, 1/log10(m·n + 10)), τ = −1 + 2·Σ pairs
//   R̂ (moments): W = mean_c M2_c/(N − 1), var⁺ = (N − 1)/N·W + var_c(mean_c)
// One thread per parameter; a thread reads its parameter's draws (stride P: consecutive threads read
// consecutive addresses) and stops the autocovariance sum at Geyer's truncation lag.
#include "hmcx_internal.h"
#include <cmath>

namespace hmcx {

struct DiagArgs {
  int C, T, P;
  const double* trace;      // [C][T][P]
  const double* means;      // [C][P] per-chain means of the moments, or null
  const double* M2;         // [C][P]
  int64_t n_mom;            // draws behind the moments
  double* seq_mean;         // scratch [2C][P]
  double* out;              // [3][P]: R̂ (moments), split-R̂, ESS
};

__global__ __launch_bounds__(256) void k_chain_diag(DiagArgs a) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= a.P) return;
  const int C = a.C, T = a.T, P = a.P, n = T / 2, m = 2 * C;
  const double nan = __builtin_nan("");
  // sequence s < C: chain s, draws [0, n); s ≥ C: chain s − C, draws [T − n, T)
  auto x = [&](int s, int i) -> double {
    const int c = s < C ? s : s - C, t = s < C ? i : T - n + i;
    return a.trace[((size_t)c * T + t) * P + p];
  };
  double* smean = a.seq_mean + p;
  // sequence means and variances
  double W = 0.0;
  for (int s = 0; s < m; ++s) {
    double mu = 0.0;
    for (int i = 0; i < n; ++i) mu += x(s, i);
    mu /= n;
    double ss = 0.0;
    for (int i = 0; i < n; ++i) {
      const double d = x(s, i) - mu;
      ss += d * d;
    }
    smean[(size_t)s * P] = mu;
    W += ss / (n - 1);
  }
  W /= m;
  double mm = 0.0;
  for (int s = 0; s < m; ++s) mm += smean[(size_t)s * P];
  mm /= m;
  double vb = 0.0;
  for (int s = 0; s < m; ++s) {
    const double d = smean[(size_t)s * P] - mm;
    vb += d * d;
  }
  vb = m > 1 ? vb / (m - 1) : 0.0;                       // var(sequence means), ddof 1
  const double var_hat = (double)(n - 1) / n * W + vb;    // = (n−1)/n·W + B/n with B = n·vb
  a.out[(size_t)P + p] = W > 0.0 ? sqrt(var_hat / W) : nan;

  // ESS: ρ_t from the mean autocovariance over the sequences, summed lag pair by lag pair
  const double var_plus = var_hat;
  double ess = nan;
  if (var_plus > 0.0) {
    auto rho = [&](int t) -> double {
      if (t == 0) return 1.0;
      double ac = 0.0;
      for (int s = 0; s < m; ++s) {
        const double mu = smean[(size_t)s * P];
        double q = 0.0;
        for (int i = 0; i + t < n; ++i) q += (x(s, i) - mu) * (x(s, i + t) - mu);
        ac += q / n;
      }
      ac /= m;
      return 1.0 - (W - ac) / var_plus;
    };
    double sum = 0.0, prev = __builtin_inf();
    for (int t = 0; t < n - 1; t += 2) {
      double pair = rho(t) + rho(t + 1);
      if (!(pair >= 0.0)) break;
      pair = fmin(pair, prev);
      sum += pair;
      prev = pair;
    }
    const double tau = -1.0 + 2.0 * sum;
    ess = (double)m * n / fmax(tau, 1.0 / log10((double)m * n + 10.0));
  }
  a.out[2 * (size_t)P + p] = ess;

  // R̂ from the per-chain moments
  double r = nan;
  if (a.means) {
    const double N = (double)a.n_mom;
    double Wm = 0.0, mu = 0.0;
    for (int c = 0; c < C; ++c) {
      Wm += a.M2[(size_t)c * P + p] / (N - 1.0);
      mu += a.means[(size_t)c * P + p];
    }
    Wm /= C;
    mu /= C;
    double vm = 0.0;
    for (int c = 0; c < C; ++c) {
      const double d = a.means[(size_t)c * P + p] - mu;
      vm += d * d;
    }
    vm = C > 1 ? vm / (C - 1) : 0.0;
    const double vh = (N - 1.0) / N * Wm + vm;
    r = Wm > 0.0 ? sqrt(vh / Wm) : nan;
  }
  a.out[p] = r;
}

}  // namespace hmcx

using namespace hmcx;

extern "C" int hmcx_chain_diagnostics(hmcx_ctx* ctx, int C, int T, int P, const double* trace, const double* means,
                                      const double* M2, int64_t n_moments, double* out) {
  if (!ctx) return HMCX_EINVAL;
  if (C < 1 || T < 4 || P < 1 || !trace || !out || (means && (!M2 || n_moments < 2)))
    return set_error(ctx, HMCX_EINVAL, "chain diagnostics: need C >= 1, T >= 4 draws, P >= 1 (and M2, n >= 2 with means)");
  Workspace ws(ctx);
  double* sm;
  do {
    ws.reset();
    sm = ws.take<double>((size_t)2 * C * P);
  } while (ws.retry());
  if (ws.failed) return set_error(ctx, HMCX_ENOMEM, "chain diagnostics: workspace");
  DiagArgs a{C, T, P, trace, means, M2, n_moments, sm, out};
  hipLaunchKernelGGL(k_chain_diag, dim3((P + 255) / 256), dim3(256), 0, ctx->stream, a);
  HMCX_HIP(ctx, hipGetLastError());
  return HMCX_OK;
}
