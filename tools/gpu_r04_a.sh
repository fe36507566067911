#!/bin/bash
# Round 4: commit decision word, lazy RCCL, 4-rank shared-GPU bench, fused wide SGLD (A/B + parity).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for cfg in "1 1" "1 0" "0 0"; do
    set -- $cfg
    HMCX_WIDE_FUSE=$1 HMCX_WIDE_GTEAM=$2 timeout -k 10 60 python tools/probe_sgld.py 400 > gpurun_out/sgld_f$1$2.$i.txt 2>&1 || { echo "probe $cfg failed"; tail -5 gpurun_out/sgld_f$1$2.$i.txt; exit 1; }
    echo "fuse=$1 gteam=$2 $(tail -1 gpurun_out/sgld_f$1$2.$i.txt)"
  done
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_recovery.py tests/test_gpu_rccl.py tests/test_gpu_nan.py tests/test_gpu_statistics.py tests/test_gpu_chains.py -m gpu -x -v --timeout 450 --timeout-method thread > gpurun_out/pytest_a.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_a.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_a.log
