#!/bin/bash
# Round B as an all-reduce by redundant reads (HMCX_P2_BAR=1, default) against the RS + AG rounds
# (HMCX_P2_BAR=0): persistent-path parity tests with each, then µs per leapfrog, 4 alternating pairs.
set -o pipefail
mkdir -p gpurun_out
for bar in 1 0; do
  HMCX_P2_BAR=$bar timeout -k 10 300 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_edges.py tests/test_gpu_multicore.py tests/test_gpu_recovery.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bar$bar.log 2>&1 || { echo "pytest BAR=$bar failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_bar$bar.log | tail -20; exit 1; }
  echo "BAR=$bar $(tail -1 gpurun_out/pytest_bar$bar.log)"
done
for rep in 1 2 3 4; do for bar in 1 0; do
  HMCX_P2_BAR=$bar timeout -k 10 60 python tools/probe_sghmc.py reps=9 > gpurun_out/ab.log 2>&1 || { tail gpurun_out/ab.log; exit 1; }
  echo "[BAR=$bar] $(tail -1 gpurun_out/ab.log | grep -o 'us/lf [0-9.]*')"
done; done
