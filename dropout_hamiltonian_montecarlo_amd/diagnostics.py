"""Convergence diagnostics for independent chains: split-R̂ and effective sample size.

The reference has no diagnostics (its multi-chain modules only concatenate posteriors,
/root/reference/hamiltonian/inference/cpu/sghmc_multicore.py:86-94); BASELINE config 4 asks for
the cross-chain R̂/ESS gather.  Standard definitions (Gelman et al., BDA3 §11.4-11.5):
split-R̂ over chain halves, ESS with Geyer's initial monotone sequence.  Host NumPy on the
gathered (small) chain summaries — this runs once per sampling run, not on the hot path.
"""
import numpy as np


def _split(chains):
    chains = np.asarray(chains, dtype=np.float64)
    if chains.ndim == 1:
        chains = chains[None]
    C, T = chains.shape[:2]
    h = T // 2
    if h < 2:
        raise ValueError("need at least 4 draws per chain")
    return np.concatenate([chains[:, :h], chains[:, T - h:]], axis=0)


def split_rhat(chains):
    """chains: [C, T, ...] draws → split-R̂ per trailing index."""
    x = _split(chains)
    m, n = x.shape[:2]
    means = x.mean(axis=1)
    W = x.var(axis=1, ddof=1).mean(axis=0)
    B = n * means.var(axis=0, ddof=1)
    var_hat = (n - 1) / n * W + B / n
    with np.errstate(divide='ignore', invalid='ignore'):
        r = np.sqrt(var_hat / W)
    return np.where(W > 0, r, np.nan)


def _autocov(x):
    """Autocovariance of x along axis 0 (FFT), biased estimator."""
    n = x.shape[0]
    xc = x - x.mean(axis=0)
    nfft = 1 << (2 * n - 1).bit_length()
    f = np.fft.rfft(xc, n=nfft, axis=0)
    ac = np.fft.irfft(f * np.conj(f), n=nfft, axis=0)[:n]
    return ac / n


def ess(chains):
    """chains: [C, T, ...] → bulk effective sample size per trailing index (split chains)."""
    x = _split(chains)
    m, n = x.shape[:2]
    flat = x.reshape(m, n, -1)
    out = np.empty(flat.shape[2])
    for p in range(flat.shape[2]):
        acov = np.stack([_autocov(flat[c, :, p]) for c in range(m)])   # [m, n]
        chain_var = acov[:, 0] * n / (n - 1)
        W = chain_var.mean()
        mean_c = flat[:, :, p].mean(axis=1)
        B_over_n = mean_c.var(ddof=1) if m > 1 else 0.0
        var_plus = W * (n - 1) / n + B_over_n
        if var_plus <= 0:
            out[p] = np.nan
            continue
        rho = 1.0 - (W - acov.mean(axis=0)) / var_plus
        rho[0] = 1.0
        # Geyer initial positive / monotone sequence over pairs
        t = 0
        s = 0.0
        prev = np.inf
        while t + 1 < n:
            pair = rho[t] + rho[t + 1]
            if pair < 0:
                break
            pair = min(pair, prev)
            s += pair
            prev = pair
            t += 2
        tau = -1.0 + 2.0 * s
        out[p] = m * n / max(tau, 1.0 / np.log10(m * n + 10))
    shape = x.shape[2:]
    return out.reshape(shape) if shape else out[0]
