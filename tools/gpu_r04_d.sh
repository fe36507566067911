#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_recovery.py tests/test_gpu_nan.py -m gpu -x -q --durations=6 --timeout 200 --timeout-method thread 2>&1 | tail -12
