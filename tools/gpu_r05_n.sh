#!/bin/bash
# MLP: deep-ring GEMM kernels (default) vs the 3-chunk ring (HMCX_MLP_DEEP=0), after the MLP parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mlp.py tests/test_gpu_statistics.py > gpurun_out/pytest_r05n.log 2>&1 || { tail -30 gpurun_out/pytest_r05n.log; exit 1; }
tail -1 gpurun_out/pytest_r05n.log
for rep in 1 2 3; do for v in 0 1; do
  HMCX_MLP_DEEP=$v timeout -k 10 200 python -u tools/probe_mlp.py > gpurun_out/pm_$v.txt 2>&1 || { tail gpurun_out/pm_$v.txt; exit 1; }
  echo "DEEP=$v: $(grep -v amdgpu.ids gpurun_out/pm_$v.txt | tail -3 | tr '\n' ' ')"
done; done
