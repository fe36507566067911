#!/bin/bash
# k_bgradw partial-tile skip + tail-last dispatch (HMCX_BGW_TAIL=1, default) vs off (=0): chain-batched
# parity tests, then the 2048-chain probe, 3 alternating pairs; then a rocprofv3 kernel-stats run of the probe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chains.py tests/test_gpu_statistics.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_bgw.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_bgw.log | tail -20; exit 1; }
tail -1 gpurun_out/pytest_bgw.log
for rep in 1 2 3; do for w in 1 0; do
  HMCX_BGW_TAIL=$w timeout -k 10 120 python tools/probe_batch.py ${CS:-2048} > gpurun_out/bgw.log 2>&1 || { tail gpurun_out/bgw.log; exit 1; }
  echo "[TAIL=$w] $(tail -1 gpurun_out/bgw.log)"
done; done
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bgw -o run --output-format csv -- python3 $R/tools/probe_batch.py ${CS:-2048} > $R/gpurun_out/bgw_prof.log 2>&1 || { echo prof failed; tail $R/gpurun_out/bgw_prof.log; exit 1; }
find $R/gpurun_out/prof_bgw -name "*stats*"
