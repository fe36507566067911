#!/bin/bash
# Round 5 box 3: config-5 SGLD with class-pair gradient loads (wide tests, probe), headline default check.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_chains.py tests/test_gpu_multicore.py -m gpu -x -q -k "wide or sgld" --timeout 200 --timeout-method thread > gpurun_out/pytest_r05c.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_r05c.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r05c.log
for rep in 1 2 3; do
  timeout -k 10 120 python tools/probe_sgld.py 400 2>&1 | grep SGLD
done
timeout -k 10 120 python tools/probe_sgld.py 400 8 2>&1 | grep SGLD
