#!/bin/bash
# Chain-batched: 128-row k_bfwd tiles (default) vs 64-row (HMCX_BFWD128=0), after the chain-batched parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chains.py tests/test_gpu_samplers.py > gpurun_out/pytest_r05m.log 2>&1 || { tail -30 gpurun_out/pytest_r05m.log; exit 1; }
tail -1 gpurun_out/pytest_r05m.log
for rep in 1 2; do for v in 0 1; do
  HMCX_BFWD128=$v timeout -k 10 300 python -u tools/probe_batch.py 2048 8192 > gpurun_out/pb_$v.txt 2>&1 || { tail gpurun_out/pb_$v.txt; exit 1; }
  echo "BFWD128=$v: $(grep -v amdgpu.ids gpurun_out/pb_$v.txt | tail -2 | tr '\n' ' ')"
done; done
