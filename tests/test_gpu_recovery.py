"""In-process recovery of the persistent single-chain SGHMC kernel (csrc/hmcx_persist2.hip).

A launch whose workgroups time out in a hand-off writes nothing to W/b and raises the context's
sticky abort word, so every launch queued behind it returns untouched too (include/hmcx.h
hmcx_clear_abort).  sghmc._collect sees the call's own abort flag, lowers the word and re-runs that
call and every later in-flight one on the kernel-per-phase path.  The sampled trajectory must still
match the NumPy oracle exactly as an undisturbed run does: bit-exact path lengths and accept flags
(reference cpu/sghmc.py:25,36), float64 state within rel 1e-9, identical printed log lines."""
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.allow_recovery]

torch = pytest.importorskip("torch")

from oracle import inputs as gi  # noqa: E402

from test_gpu_samplers import _run_gpu, _run_oracle  # noqa: E402


def _check_vs_oracle(c, got):
    post_r, logp_r, tr_r, log_r = _run_oracle(c)
    post_g, logp_g, tr_g, log_g = got
    assert [t["L"] for t in tr_g] == [t["L"] for t in tr_r]
    assert [t["accepted"] for t in tr_g] == [t["accepted"] for t in tr_r]
    for v in ("weights", "bias"):
        np.testing.assert_allclose(post_g[v], post_r[v], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(logp_g, logp_r, rtol=1e-11)
    assert [l for l in log_g.splitlines() if "loss" in l] == [l for l in log_r.splitlines() if "loss" in l]


def _restore_path():
    from dropout_hamiltonian_montecarlo_amd import _native as nat
    nat.context(torch.device("cuda:0")).set_sghmc_path(0)


@pytest.mark.parametrize("name,path", [("sghmc_small", 2), ("sghmc_mnist", 2)])
def test_forced_abort_is_recovered_in_process(name, path, monkeypatch, capfd):
    """HMCX_P2_FORCE_ABORT=1: in every persistent launch the last workgroup gives up at step 1
    (the other workgroups then abort in their polls) — the first epoch's call and the one already
    queued behind it (sample() pipelines epoch calls) are both re-run."""
    from dropout_hamiltonian_montecarlo_amd import _native as nat
    c = gi.TRAJ_CONFIGS[name]
    before = nat.recoveries_all()["persistent_sghmc"]
    monkeypatch.setenv("HMCX_P2_FORCE_ABORT", "1")
    try:
        got = _run_gpu(c, path=path)
    finally:
        _restore_path()
    err = capfd.readouterr().err
    assert "hand-off timed out" in err
    # every re-run call counted once (hmcx_get_recoveries): the calls each recovery announces
    import re
    rerun = sum(int(n) for n in re.findall(r"re-running (\d+) call", err))
    assert rerun >= 1
    assert nat.recoveries_all()["persistent_sghmc"] == before + rerun
    _check_vs_oracle(c, got)


def test_misplaced_xcd_map_is_recovered_in_process(monkeypatch, capfd):
    """HMCX_P2_XMAP=2 keeps the row-team rounds in one XCD's L2 while the identity map spreads every
    row team over all 8 XCDs: members elsewhere never see those rounds, the launch spins to its 4 s
    bound and aborts.  (If a line is written back early the round simply completes; either way the
    result must be the oracle's.)"""
    c = gi.TRAJ_CONFIGS["sghmc_small"]
    monkeypatch.setenv("HMCX_P2_XMAP", "2")
    try:
        got = _run_gpu(c, path=2)
    finally:
        _restore_path()
    print("recovered" if "hand-off timed out" in capfd.readouterr().err else "no timeout occurred")
    _check_vs_oracle(c, got)


def test_abort_word_reported_through_c_abi(monkeypatch):
    """Without out_abort (plain C-ABI callers) the timeout is reported by hmcx_synchronize and W/b
    are left as they were; hmcx_clear_abort re-arms the persistent path."""
    from dropout_hamiltonian_montecarlo_amd import _native as nat
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.softmax import softmax
    from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sghmc import sghmc
    c = gi.TRAJ_CONFIGS["sghmc_mnist"]
    X, Y = gi.dataset(c["data_seed"], c["N"], c["D"], c["K"])
    m = softmax({"alpha": c["alpha"]}, dtype=torch.float64, device="cuda:0")
    m.ctx.set_sghmc_path(2)
    try:
        s = sghmc(m, {"weights": np.full((c["D"], c["K"]), 0.01), "bias": np.zeros(c["K"])},
                  path_length=c["path_length"], step_size=c["step_size"], noise="philox", seed=3)
        data = s._upload_data(X, Y)
        st = s._init_state()
        W0 = st["weights"].clone()
        n_iter, u, _, noff = s._schedule(3, [c["step_size"]] * 3, None, 7850)
        rows = np.zeros(3, dtype=np.int64)
        eps = np.full(3, c["step_size"])
        n_iter, u = np.ascontiguousarray(n_iter.reshape(-1)), np.ascontiguousarray(u.reshape(-1))
        out = torch.zeros(64, dtype=torch.float64, device="cuda:0")
        acc = torch.zeros(8, dtype=torch.int32, device="cuda:0")
        a = nat.SamplerArgs()
        a.dtype, a.B, a.D, a.K, a.C, a.n_steps = m.code, c["B"], c["D"], c["K"], 1, 3
        a.alpha, a.log_prior = m.alpha, s._log_prior()
        a.X, a.Y = nat.ptr(data[0]), nat.ptr(data[1])
        a.row0 = nat.addr(rows)
        a.eps = nat.addr(eps)
        a.n_iter = nat.addr(n_iter)
        a.u_accept = nat.addr(u)
        a.noise_mode = nat.NOISE_PHILOX
        a.noise_off = nat.addr(noff.reshape(-1))
        a.seed, a.chain0, a.step_base = 3, 0, 0
        a.W, a.b = nat.ptr(st["weights"]), nat.ptr(st["bias"])
        a.out_A, a.out_ll, a.out_E = out.data_ptr(), out.data_ptr() + 64, out.data_ptr() + 128
        a.out_accepted = acc.data_ptr()
        monkeypatch.setenv("HMCX_P2_FORCE_ABORT", "0")
        assert m.ctx.lib.hmcx_sghmc_run(m.ctx.h, a) == 0
        assert m.ctx.lib.hmcx_synchronize(m.ctx.h) != 0
        assert b"timed out" in m.ctx.lib.hmcx_last_error(m.ctx.h)
        torch.testing.assert_close(st["weights"], W0, rtol=0, atol=0)      # untouched
        # the persistent word is still raised: a fused wide-SGLD call on the same context polls its own
        # word (hmcx_internal.h wide_abort_dev), so it neither fails nor re-runs, and matches the oracle
        wide = dict(kind="sgld", N=1000, B=500, D=2048, K=38, alpha=0.01, step_size=1e-4, path_length=1.0,
                    burnin=1, epochs=1, data_seed=41, np_seed=2, rng_seed=3)
        monkeypatch.setenv("HMCX_SGLD_WIDE", "1")
        monkeypatch.setenv("HMCX_WIDE_FUSE", "1")
        rec0 = m.ctx.recoveries()
        post_g, logp_g, _, _ = _run_gpu(wide)
        assert m.ctx.recoveries() == rec0
        post_r, logp_r, _, _ = _run_oracle(wide)
        np.testing.assert_allclose(post_g["weights"], post_r["weights"], rtol=1e-9, atol=1e-12)
        m.ctx.clear_abort()
        monkeypatch.delenv("HMCX_P2_FORCE_ABORT")
        assert m.ctx.lib.hmcx_sghmc_run(m.ctx.h, a) == 0
        assert m.ctx.lib.hmcx_synchronize(m.ctx.h) == 0
        assert not torch.equal(st["weights"], W0) or not acc[:3].any()
    finally:
        _restore_path()
