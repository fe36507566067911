#!/bin/bash
# Wide SGLD variants: probe A/B (persistent / fused two-launch / three-launch), then the wide parity tests.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
for i in 1 2; do
  for cfg in "1 1" "1 0" "0 0"; do
    set -- $cfg
    echo "fuse=$1 persist=$2 $(HMCX_WIDE_FUSE=$1 HMCX_WIDE_PERSIST=$2 timeout -k 10 60 python tools/probe_sgld.py 400 2>&1 | tail -1)"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_chains.py -k "sgld" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_b.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_b.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_b.log
