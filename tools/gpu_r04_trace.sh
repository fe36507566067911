#!/bin/bash
# In-call trace rows of the chain-batched / kernel-per-phase SGHMC paths, the multicore (HDF5 backend)
# tests that trace through them, and the chain-batched parity tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multicore.py tests/test_gpu_chains.py tests/test_gpu_recovery.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_tr.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_tr.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_tr.log
