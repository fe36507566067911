"""Convergence diagnostics for independent chains: split-R̂ and effective sample size.

The reference has no diagnostics (its multi-chain modules only concatenate posteriors,
/root/reference/hamiltonian/inference/cpu/sghmc_multicore.py:86-94); BASELINE config 4 asks for
the cross-chain R̂/ESS gather.  Standard definitions (Gelman et al., BDA3 §11.4-11.5):
split-R̂ over chain halves, ESS with Geyer's initial monotone sequence.

Two implementations of the same definitions: `device_diagnostics` runs them on the GPU where the RCCL
all-gather leaves the chain summaries (libhmcx hmcx_chain_diagnostics, csrc/hmcx_diag.hip, one thread
per parameter); the NumPy functions below are the host version used by CPU-only (gloo) runs and as the
reference the device kernel is tested against (tests/test_gpu_diagnostics.py).
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
    """Autocovariance of x along axis 1 ([m, n, P]; FFT), biased estimator."""
    n = x.shape[1]
    xc = x - x.mean(axis=1, keepdims=True)
    nfft = 1 << (2 * n - 1).bit_length()
    f = np.fft.rfft(xc, n=nfft, axis=1)
    ac = np.fft.irfft(f * np.conj(f), n=nfft, axis=1)[:, :n]
    return ac / n


def ess(chains):
    """chains: [C, T, ...] → bulk effective sample size per trailing index (split chains).
    Vectorised over the trailing indices: one FFT per chain half for all parameters, then Geyer's
    initial positive / monotone sequence advanced lag pair by lag pair for every parameter at once."""
    x = _split(chains)
    m, n = x.shape[:2]
    flat = x.reshape(m, n, -1)
    acov = _autocov(flat)                                  # [m, n, P]
    chain_var = acov[:, 0, :] * n / (n - 1)
    W = chain_var.mean(axis=0)
    B_over_n = flat.mean(axis=1).var(axis=0, ddof=1) if m > 1 else np.zeros(flat.shape[2])
    var_plus = W * (n - 1) / n + B_over_n
    ok = var_plus > 0
    with np.errstate(divide='ignore', invalid='ignore'):
        rho = 1.0 - (W[None, :] - acov.mean(axis=0)) / var_plus[None, :]   # [n, P]
    rho[0] = 1.0
    s = np.zeros(flat.shape[2])
    prev = np.full(flat.shape[2], np.inf)
    live = ok.copy()
    for t in range(0, n - 1, 2):
        pair = rho[t] + rho[t + 1]
        live &= pair >= 0
        if not live.any():
            break
        pair = np.minimum(pair, prev)
        s = np.where(live, s + pair, s)
        prev = np.where(live, pair, prev)
    tau = -1.0 + 2.0 * s
    out = m * n / np.maximum(tau, 1.0 / np.log10(m * n + 10))
    out = np.where(ok, out, np.nan)
    shape = x.shape[2:]
    return out.reshape(shape) if shape else out[0]


def device_diagnostics(trace, means=None, M2=None, n=0, device=None):
    """R̂ from per-chain moments, split-R̂ and ESS per parameter on the device (hmcx_chain_diagnostics).
    trace: [C, T, P] (a device float64 tensor, e.g. the RCCL all-gather's output, or an array copied to
    `device`); means / M2: [C, P] over n draws (optional).  Returns numpy arrays (rhat, split_rhat, ess),
    each [P] (rhat NaN without moments)."""
    import torch
    from . import _native as nat
    dev = trace.device if isinstance(trace, torch.Tensor) else torch.device(device or "cuda")
    t = torch.as_tensor(trace, dtype=torch.float64, device=dev).contiguous()
    C, T, P = t.shape
    mu = m2 = None
    if means is not None:
        mu = torch.as_tensor(means, dtype=torch.float64, device=dev).contiguous()
        m2 = torch.as_tensor(M2, dtype=torch.float64, device=dev).contiguous()
    out = torch.empty(3 * P, dtype=torch.float64, device=dev)
    ctx = nat.context(dev)
    ctx.check(ctx.lib.hmcx_chain_diagnostics(ctx.h, C, T, P, nat.ptr(t), nat.ptr(mu), nat.ptr(m2), int(n),
                                             nat.ptr(out)), "hmcx_chain_diagnostics")
    o = out.cpu().numpy().reshape(3, P)
    return o[0], o[1], o[2]
