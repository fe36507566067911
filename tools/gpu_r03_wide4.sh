#!/bin/bash
# Full GPU suite after removing the row-space / persistent-SGLD variants and adding multi-chain wide
# SGLD; then config-5 probes at 1 and 8 chains per GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_gpu.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for C in 1 8; do
  echo "C=$C $(timeout -k 10 120 python tools/probe_sgld.py 400 $C 2>&1 | grep -v amdgpu.ids)"
done
echo "C=8 kernel-per-phase $(HMCX_SGLD_WIDE=0 timeout -k 10 120 python tools/probe_sgld.py 200 8 2>&1 | grep -v amdgpu.ids)"
