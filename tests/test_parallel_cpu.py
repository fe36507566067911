"""Multi-process (gloo, world_size 2) tests of the chain-sharding + gather layer, and the
R̂ / ESS diagnostics on known-answer inputs."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rhat_ess_known_answers():
    from dropout_hamiltonian_montecarlo_amd import diagnostics as dg
    rs = np.random.RandomState(0)
    iid = rs.normal(size=(4, 2000))
    assert abs(dg.split_rhat(iid) - 1.0) < 0.01
    assert 0.8 * 8000 < dg.ess(iid) < 1.2 * 8000
    # AR(1) with phi: ESS ≈ N (1-phi)/(1+phi)
    phi = 0.9
    x = np.zeros((4, 4000))
    e = rs.normal(size=x.shape)
    for t in range(1, x.shape[1]):
        x[:, t] = phi * x[:, t - 1] + e[:, t]
    expect = 16000 * (1 - phi) / (1 + phi)
    assert 0.6 * expect < dg.ess(x) < 1.4 * expect
    # chains stuck at different means → R̂ >> 1
    shifted = iid + np.arange(4)[:, None] * 3.0
    assert dg.split_rhat(shifted) > 1.5
    # vector quantities
    v = rs.normal(size=(3, 500, 5))
    assert dg.split_rhat(v).shape == (5,) and dg.ess(v).shape == (5,)


def test_chain_sharding():
    from dropout_hamiltonian_montecarlo_amd.parallel import chain_block, chains_of_rank
    assert chains_of_rank(8, 0, 8) == [0]
    assert chains_of_rank(8, 1, 2) == [4, 5, 6, 7]
    assert sorted(sum((chains_of_rank(10, r, 4) for r in range(4)), [])) == list(range(10))
    # contiguous blocks: sampler(chain=chain0, chains=c) keys chain0 + c — disjoint across ranks
    assert [chain_block(10, r, 4) for r in range(4)] == [(0, 3), (3, 3), (6, 2), (8, 2)]
    for r in range(4):
        c0, c = chain_block(10, r, 4)
        assert chains_of_rank(10, r, 4) == list(range(c0, c0 + c))


def test_welford_matches_two_pass():
    from dropout_hamiltonian_montecarlo_amd.parallel import Welford, rhat_from_moments
    from dropout_hamiltonian_montecarlo_amd import diagnostics as dg
    rs = np.random.RandomState(3)
    x = rs.normal(size=(3, 301, 7)) * np.arange(1, 8) + np.arange(3)[:, None, None]
    w = Welford((3, 7))
    for a, b in ((0, 1), (1, 50), (50, 51), (51, 301)):      # uneven batches, single draws
        w.update(x[:, a] if b - a == 1 else x[:, a:b])
    assert w.n == 301
    np.testing.assert_allclose(w.mean, x.mean(axis=1), rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(w.M2, ((x - x.mean(axis=1, keepdims=True)) ** 2).sum(axis=1), rtol=1e-12)
    # classic R̂ from the moments = the direct computation on the draws
    means, var = x.mean(axis=1), x.var(axis=1, ddof=1)
    n = x.shape[1]
    direct = np.sqrt(((n - 1) / n * var.mean(axis=0) + means.var(axis=0, ddof=1)) / var.mean(axis=0))
    np.testing.assert_allclose(rhat_from_moments(n, w.mean, w.M2), direct, rtol=1e-12)
    assert np.all(rhat_from_moments(n, w.mean, w.M2) > 1.0)
    assert dg.split_rhat(x).shape == (7,)


WORKER = r'''
import os, sys
sys.path.insert(0, os.environ["REPO"])
import numpy as np
from dropout_hamiltonian_montecarlo_amd import parallel
rank, world, local = parallel.init("gloo")
rs = np.random.RandomState(100 + rank)
local_tr = rs.normal(size=(2, 64, 3)) + rank        # 2 chains per rank, 64 draws, 3 params
allt = parallel.gather_traces(local_tr)
assert allt.shape == (2 * world, 64, 3)
for r in range(world):
    ref = np.random.RandomState(100 + r).normal(size=(2, 64, 3)) + r
    np.testing.assert_array_equal(allt[2 * r:2 * r + 2], ref)
assert parallel.allreduce_sum(rank + 1) == world * (world + 1) / 2
assert parallel.allreduce_max(rank) == world - 1
d = parallel.chain_diagnostics(allt)
assert d["rhat"].shape == (3,) and np.all(d["rhat"] > 1.0)
# per-parameter summaries: Welford over the local draws + a thinned trace, one all-gather
w = parallel.Welford((2, 3)).update(local_tr)
n, means, M2, tr = parallel.gather_summaries(w, local_tr[:, ::4], device=None)
assert n == 64 and means.shape == (2 * world, 3) and tr.shape == (2 * world, 16, 3)
np.testing.assert_allclose(means, allt.mean(axis=1), rtol=1e-13)
np.testing.assert_allclose(parallel.rhat_from_moments(n, means, M2),
                           np.sqrt(((n - 1) / n * allt.var(axis=1, ddof=1).mean(axis=0)
                                    + allt.mean(axis=1).var(axis=0, ddof=1)) / allt.var(axis=1, ddof=1).mean(axis=0)),
                           rtol=1e-12)
np.testing.assert_allclose(parallel.diagnostics.split_rhat(tr), parallel.diagnostics.split_rhat(allt[:, ::4]))
s = parallel.summary_diagnostics(n, means, M2, tr)
assert s["chains"] == 2 * world and s["params"] == 3 and s["rhat"]["min"] > 1.0
# uneven blocks (chain_block(5, r, 2) = 3 + 2 chains): padded for the gather, padding dropped
c0, c = parallel.chain_block(5, rank, world)
mine = np.stack([np.full((4, 3), float(i)) for i in range(c0, c0 + c)])
allu = parallel.gather_traces(mine)
assert allu.shape == (5, 4, 3), allu.shape
np.testing.assert_array_equal(allu[:, 0, 0], np.arange(5.0))
wu = parallel.Welford((c, 3)).update(mine)
n, means, M2, tr = parallel.gather_summaries(wu, mine[:, ::2])
assert means.shape == (5, 3) and tr.shape == (5, 2, 3)
np.testing.assert_array_equal(means[:, 0], np.arange(5.0))
assert parallel.gather_objects(rank) == list(range(world))
# the N-GPU bench line's aggregation (bench.aggregate_ranks) over the gathered per-rank numbers: rank r
# did 100·(r+1) + 7 leapfrogs in 1.5·(r+1) ms; makespan Σ lf / max t, chain throughput Σ lf_r / t_r
import bench
per = parallel.gather_objects({"leapfrogs": 100.0 * (rank + 1) + 7, "seconds": 1.5e-3 * (rank + 1)})
agg = bench.aggregate_ranks(per, P_dim=1)
lf = [100.0 * (r + 1) + 7 for r in range(world)]
ts = [1.5e-3 * (r + 1) for r in range(world)]
assert agg["per_rank_leapfrogs"] == lf
assert abs(agg["value_makespan"] - sum(lf) / max(ts)) < 1e-6 * agg["value_makespan"]
assert abs(agg["value_chain_throughput"] - sum(l / t for l, t in zip(lf, ts))) < 1e-6 * agg["value_chain_throughput"]
assert world != 2 or abs(agg["value_makespan"] - 314.0 / 3e-3) < 1e-3      # hand-computed: (107 + 207) / 3 ms
assert world != 2 or abs(agg["value_chain_throughput"] - (107.0 / 1.5e-3 + 207.0 / 3e-3)) < 1e-3
parallel.barrier()
parallel.finalize()
print("ok", rank)
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_gather():
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, REPO=REPO, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
        assert "ok" in o.split()


WORKER8 = r"""
import os, sys
sys.path.insert(0, os.environ["REPO"])
import numpy as np
from dropout_hamiltonian_montecarlo_amd import parallel
rank, world, local = parallel.init("gloo")
assert world == 8
P, T, THIN = 7850, 240, 4                 # the bench's sizes: config 2 (P = 7,850), 240 diagnostics draws, every 4th kept
def draws(r):                             # rank r's one chain (BASELINE config 4: one chain per GPU)
    rs = np.random.RandomState(500 + r)
    return (np.cumsum(rs.normal(size=(1, T, P)), axis=1) * 0.05 + 0.01 * r)
mine = draws(rank)
c0, c = parallel.chain_block(8, rank, world)
assert (c0, c) == (rank, 1)
w = parallel.Welford((1, P)).update(mine)
n, means, M2, tr = parallel.gather_summaries(w, mine[:, ::THIN], device=None)
assert n == T and means.shape == (8, P) and M2.shape == (8, P) and tr.shape == (8, T // THIN, P)
if rank == 0:
    allx = np.concatenate([draws(r) for r in range(world)])            # [8, T, P], rank order
    np.testing.assert_allclose(means, allx.mean(axis=1), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(M2, ((allx - allx.mean(axis=1, keepdims=True)) ** 2).sum(axis=1), rtol=1e-10)
    np.testing.assert_array_equal(tr, allx[:, ::THIN])
    s = parallel.summary_diagnostics(n, means, M2, tr)
    assert s["chains"] == 8 and s["params"] == P and s["trace_draws_per_chain"] == 60 and s["draws_per_chain"] == T
    ref_sr = parallel.diagnostics.split_rhat(allx[:, ::THIN])
    assert abs(s["split_rhat"]["median"] - float(np.median(ref_sr))) < 1e-12
    assert s["rhat"]["min"] > 1.0 and s["ess"]["min"] > 0
# the N = 8 line: both aggregates over the gathered per-rank numbers (bench.aggregate_ranks)
import bench
lf = 182.0 + 7 * rank
per = parallel.gather_objects({"leapfrogs": lf, "seconds": 1.7e-3 * lf / 182.0})
agg = bench.aggregate_ranks(per, P_dim=P)
tot = sum(182.0 + 7 * r for r in range(world))
assert abs(agg["value_makespan"] - tot / (1.7e-3 * (182.0 + 49) / 182.0) * P) < 1e-6 * agg["value_makespan"]
assert abs(agg["value_chain_throughput"] - world * 182.0 / 1.7e-3 * P) < 1e-6 * agg["value_chain_throughput"]
parallel.barrier()
parallel.finalize()
print("ok", rank)
"""


def test_gloo_world8_gather_at_bench_sizes():
    """World-8 rehearsal of the driver's 8-GPU run (configs 4 and 5: one chain per rank, reference
    sghmc_multicore.py:81-99 concatenates the workers' posteriors): the per-chain summaries at the
    bench's real sizes (P = 7,850, 240 draws, 60 thinned) in one all-gather over gloo, R̂ / split-R̂ /
    ESS on rank 0 against the same statistics of the concatenated draws, and both aggregates of the
    N = 8 line."""
    port = _free_port()
    procs = []
    for r in range(8):
        env = dict(os.environ, REPO=REPO, RANK=str(r), WORLD_SIZE="8", LOCAL_RANK=str(r), OMP_NUM_THREADS="1",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER8], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=400) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
        assert "ok" in o.split()
