#!/bin/bash
# Chain-batched compaction-tail forwards on 32-row tiles (HMCX_BTAIL32, default 1) vs the 8-wave 64-row
# kernel: parity, then same-box A/B of tools/probe_batch.py at 2048 and 8192 chains.  (The round-4 run
# also A/B'd a double-buffered gradient variant, since removed: DESIGN §5.2.)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chains.py tests/test_gpu_multicore.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_tail.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_tail.log | tail -20; exit 1; }
tail -1 gpurun_out/pytest_tail.log
for rep in 1 2; do
  for t in 1 0; do
    HMCX_BTAIL32=$t timeout -k 10 120 python tools/probe_batch.py 2048 8192 > gpurun_out/tail.log 2>&1 || { tail gpurun_out/tail.log; exit 1; }
    grep "C=" gpurun_out/tail.log | sed "s/^/[tail32=$t] /"
  done
done
