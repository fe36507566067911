#!/bin/bash
# Trace rows stored in-call on every sampler path (SGLD kernel-per-phase added): multicore / HDF5
# backend, samplers, chains and recovery tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_multicore.py tests/test_gpu_samplers.py tests/test_gpu_chains.py tests/test_gpu_recovery.py tests/test_gpu_nan.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_tr2.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_tr2.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_tr2.log
