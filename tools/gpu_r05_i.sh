#!/bin/bash
# MLP full-batch HMC trajectory in one call: parity against the host loop, and its speed.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mlp.py -k "hmc" > gpurun_out/pytest_r05i.log 2>&1 &&
timeout -k 10 300 python -u tools/probe_mlp_hmc.py f32 6 > gpurun_out/probe_mlp_hmc_r05.log 2>&1 &&
timeout -k 10 300 python -u tools/probe_mlp_hmc.py f64 6 >> gpurun_out/probe_mlp_hmc_r05.log 2>&1
