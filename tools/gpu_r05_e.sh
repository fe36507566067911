#!/bin/bash
# Round 5 box 5: chain-batched GEMM loops software-pipelined (k_bfwd, k_bgradw) — parity tests, then
# same-box A/B against the round-start library at 2048 / 8192 chains.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_diagnostics.py tests/test_gpu_chains.py tests/test_gpu_nan.py tests/test_gpu_samplers.py tests/test_gpu_statistics.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r05e.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_r05e.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r05e.log
for rep in 1 2 3; do
  for lib in libhmcx.so libhmcx_base.so; do
    HMCX_LIB=$lib timeout -k 10 200 python tools/probe_batch.py 2048 8192 2>&1 | grep "C=" | sed "s/^/$lib /"
  done
done
