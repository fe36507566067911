"""On-device convergence diagnostics (csrc/hmcx_diag.hip, include/hmcx.h hmcx_chain_diagnostics)
against the host definitions of diagnostics.py (split-R̂, ESS with Geyer's initial monotone sequence)
and parallel.rhat_from_moments, on AR(1) chains of known autocorrelation.  The FFT (host) and direct
(device) autocovariances round differently, so the comparison is to rtol 1e-9; a parameter whose
Geyer truncation lag sits exactly on a sign change could differ by a lag pair — the data are chosen
away from that."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from dropout_hamiltonian_montecarlo_amd import diagnostics, parallel  # noqa: E402


def _ar1(C, T, P, phi, seed):
    rs = np.random.RandomState(seed)
    x = np.empty((C, T, P))
    x[:, 0] = rs.normal(size=(C, P))
    for t in range(1, T):
        x[:, t] = phi * x[:, t - 1] + np.sqrt(1 - phi ** 2) * rs.normal(size=(C, P))
    return x + rs.normal(0, 0.3, size=(C, 1, P))              # chain offsets: R̂ > 1 on some parameters


@pytest.mark.parametrize("C,T,P,phi", [(1, 60, 7850, 0.5), (4, 60, 1000, 0.8), (8, 240, 300, 0.95), (3, 9, 50, 0.2)])
def test_device_diagnostics_match_host(C, T, P, phi):
    x = _ar1(C, T, P, phi, seed=C * 100 + T)
    x[:, :, 0] = 1.5                                          # a constant parameter: W = 0 → NaN
    wf = parallel.Welford((C, P)).update(x)
    r, sr, es = diagnostics.device_diagnostics(torch.from_numpy(x).to("cuda:0"), wf.mean, wf.M2, wf.n)
    r_h = parallel.rhat_from_moments(wf.n, wf.mean, wf.M2)
    sr_h = diagnostics.split_rhat(x)
    es_h = diagnostics.ess(x)
    for got, want in ((r, r_h), (sr, sr_h), (es, es_h)):
        assert np.array_equal(np.isnan(got), np.isnan(want))
        ok = ~np.isnan(want)
        np.testing.assert_allclose(got[ok], want[ok], rtol=1e-9)
    assert np.isnan(sr[0]) and np.isnan(es[0])


def test_device_summary_of_gathered_chains():
    """summary_diagnostics_device (what bench.py reports) equals summary_diagnostics on the same data."""
    C, T, P = 4, 60, 500
    x = _ar1(C, T, P, 0.7, seed=3)
    wf = parallel.Welford((C, P)).update(x)
    dev = torch.device("cuda:0")
    d = parallel.summary_diagnostics_device(wf.n, torch.from_numpy(wf.mean).to(dev), torch.from_numpy(wf.M2).to(dev),
                                            torch.from_numpy(x).to(dev))
    h = parallel.summary_diagnostics(wf.n, wf.mean, wf.M2, x)
    for k in ("rhat", "split_rhat", "ess"):
        for q in ("min", "median", "max"):
            assert d[k][q] == pytest.approx(h[k][q], rel=1e-9)
    assert d["computed_on"].startswith("device")
