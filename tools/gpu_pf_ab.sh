#!/bin/bash
# GPU tests, then an A/B of the persistent SGHMC probe: AB_A / AB_B environment settings, AB_REPS pairs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu_ab.sh "${AB_A:-HMCX_P2_ACC1=1}" "${AB_B:-HMCX_P2_ACC1=0}"
