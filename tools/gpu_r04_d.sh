#!/bin/bash
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_multicore.py tests/test_gpu_samplers.py tests/test_gpu_chains.py tests/test_gpu_statistics.py -k "sgld or multicore or wide" -m gpu -x -q --durations=5 --timeout 300 --timeout-method thread 2>&1 | tail -12
echo "fused $(timeout -k 10 60 python tools/probe_sgld.py 400 2>&1 | tail -1)"
