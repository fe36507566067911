#!/bin/bash
# GPU test suite (optionally a subset: tools/gpu_tests.sh tests/test_x.py ...), then the default bench line.
set -o pipefail
mkdir -p gpurun_out
T=${@:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_gpu.log | tail -40; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
grep -E "ens_mean" gpurun_out/pytest_gpu.log | head; true
