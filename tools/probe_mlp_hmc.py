#!/usr/bin/env python3
"""Full-batch HMC on the config-3 MLP (784-256-256-10, B = 500): seconds per leapfrog iteration of
hmc.step with the trajectory in one hmcx_mlp_hmc_leapfrog call vs the host loop it replaces
(HMCX_HMC_HOST_LOOP=1: model.grad + hmcx_axpy per variable from Python).
    python tools/probe_mlp_hmc.py [f32|f64] [steps] [device]   (device: skip the host loop)"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dropout_hamiltonian_montecarlo_amd.hamiltonian.models.gpu.mlp import mlp  # noqa: E402
from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.hmc import hmc  # noqa: E402
from dropout_hamiltonian_montecarlo_amd.hamiltonian.inference.gpu.sghmc import _n_iter  # noqa: E402


def run(host, dt, steps):
    os.environ["HMCX_HMC_HOST_LOOP"] = "1" if host else "0"
    rs = np.random.RandomState(0)
    X = torch.as_tensor(rs.rand(500, 784), dtype=dt, device="cuda:0")
    y = torch.as_tensor(rs.randint(0, 10, 500), dtype=torch.int32, device="cuda:0")
    m = mlp({"alpha": 0.01}, 784, 256, 10, dtype=dt, device="cuda:0")
    s = hmc(m, m.init_params(1), path_length=0.25, step_size=0.005)
    q = {k: torch.as_tensor(v, dtype=dt, device="cuda:0") for k, v in s.start.items()}
    rng = np.random.RandomState(2)
    np.random.seed(1)
    s.step(q, None, rng, X_train=X, y_train=y)              # warm-up
    torch.cuda.synchronize()
    np.random.seed(1)
    s.trace = []
    t0 = time.perf_counter()
    for _ in range(steps):
        s.step(q, None, rng, X_train=X, y_train=y)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0), sum(_n_iter(t["L"]) for t in s.trace)


if __name__ == "__main__":
    dt = torch.float64 if (len(sys.argv) > 1 and sys.argv[1] == "f64") else torch.float32
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    modes = (False,) if "device" in sys.argv else (True, False)
    for rep in range(2):
        for host in modes:
            t, n = run(host, dt, steps)
            print("%s %s: %d steps, %.3f s, %d leapfrogs, %.1f us per leapfrog"
                  % ("host-loop" if host else "device   ", str(dt), steps, t, n, 1e6 * t / max(n, 1)), flush=True)
