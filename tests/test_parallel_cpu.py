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
    from dropout_hamiltonian_montecarlo_amd.parallel import chains_of_rank
    assert chains_of_rank(8, 0, 8) == [0]
    assert chains_of_rank(8, 1, 2) == [1, 3, 5, 7]
    assert sorted(sum((chains_of_rank(10, r, 4) for r in range(4)), [])) == list(range(10))


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
parallel.barrier()
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
