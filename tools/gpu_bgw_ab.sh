#!/bin/bash
# k_bgradw<T,8> (128-feature tiles, HMCX_BGRAD_WIDE=1, default) vs the 64-feature tiles (=0): chain-batched
# parity tests, then the 2048-chain probe, 3 alternating pairs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chains.py tests/test_gpu_statistics.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_bgw.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_bgw.log | tail -20; exit 1; }
tail -1 gpurun_out/pytest_bgw.log
for rep in 1 2 3; do for w in 1 0; do
  HMCX_BGRAD_WIDE=$w timeout -k 10 120 python tools/probe_batch.py ${CS:-2048} > gpurun_out/bgw.log 2>&1 || { tail gpurun_out/bgw.log; exit 1; }
  echo "[WIDE=$w] $(tail -1 gpurun_out/bgw.log)"
done; done
