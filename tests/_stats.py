"""Moment comparison of two chain ensembles (test infrastructure for tests/test_gpu_statistics.py).

Two views, both as per-parameter z-scores (difference ÷ combined Monte-Carlo standard error):

* ``ens_*`` — the ensembles' states after the last step: one independent draw per chain, so the
  standard error of the mean is sd/√C and that of the variance √((m4 − v²)/C) (delta method);
* ``run_*`` — the running posterior over the second half of every chain, pooled over chains, with
  MCSE = sd/√ESS (ESS: diagnostics.ess, multi-chain split ESS; for the variance the ESS and sd of the
  squared deviations).

SURVEY §8(c) states the tolerance as 3·MCSE per parameter.  Over thousands of parameters a 3σ
band is exceeded by chance at a rate of ≈0.27 % per statistic, so the tests apply it as: at most
1 % of the parameters beyond 3 standard errors, and none beyond 6 (a family-wise bound over up to
~78k parameters with t-distributed ensemble statistics: oracle-vs-oracle runs reach 5.8).
"""
import numpy as np

from dropout_hamiltonian_montecarlo_amd import diagnostics


def _z(num, den):
    den = np.asarray(den, dtype=np.float64)
    num = np.asarray(num, dtype=np.float64)
    out = np.zeros_like(num)
    ok = den > 0
    out[ok] = num[ok] / den[ok]
    out[~ok & (np.abs(num) > 0)] = np.inf
    return out


def _ens(x):
    C = x.shape[0]
    m = x.mean(0)
    v = x.var(0, ddof=1)
    m4 = ((x - m) ** 4).mean(0)
    return m, v, v / C, np.maximum(m4 - v * v, 0.0) / C


def _run(x, chunk=4096):
    """Running-posterior moments and their MCSE, parameters in chunks (bounded FFT workspace)."""
    P = x.shape[2]
    out = [np.empty(P) for _ in range(4)]
    for p0 in range(0, P, chunk):
        xc = x[:, :, p0:p0 + chunk]
        m = xc.mean((0, 1))
        sd = xc.std((0, 1))
        e = diagnostics.ess(xc)
        e = np.where(np.isfinite(e) & (e > 0), e, 1.0)
        d2 = (xc - m) ** 2
        e2 = diagnostics.ess(d2)
        e2 = np.where(np.isfinite(e2) & (e2 > 0), e2, 1.0)
        for o, v in zip(out, (m, d2.mean((0, 1)), (sd ** 2) / e, d2.var((0, 1)) / e2)):
            o[p0:p0 + chunk] = v
    return tuple(out)


def compare(a, b):
    """a, b: draws [C, T, P] of two ensembles → dict of per-parameter z-scores."""
    ma, va, sma, sva = _ens(a[:, -1, :])
    mb, vb, smb, svb = _ens(b[:, -1, :])
    out = {"ens_mean": _z(ma - mb, np.sqrt(sma + smb)), "ens_var": _z(va - vb, np.sqrt(sva + svb))}
    h = a.shape[1] // 2
    ma, va, sma, sva = _run(a[:, h:, :])
    mb, vb, smb, svb = _run(b[:, h:, :])
    out["run_mean"] = _z(ma - mb, np.sqrt(sma + smb))
    out["run_var"] = _z(va - vb, np.sqrt(sva + svb))
    return out


def summary(z):
    return {k: (float(np.mean(np.abs(v) > 3.0)), float(np.max(np.abs(v)))) for k, v in z.items()}


def assert_same_moments(z, frac3=0.01, zmax=6.0):
    s = summary(z)
    bad = {k: v for k, v in s.items() if v[0] > frac3 or v[1] > zmax}
    assert not bad, "moments differ beyond 3·MCSE: %s (all: %s)" % (bad, s)
