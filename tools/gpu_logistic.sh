#!/bin/bash
# Logistic model + momentum SGD parity on the GPU (tests/test_gpu_logistic_sgd.py) and the full sampler suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_logistic_sgd.py tests/test_gpu_softmax.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_logistic.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_logistic.log; exit 1; }
tail -2 gpurun_out/pytest_logistic.log
