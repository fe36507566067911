#!/bin/bash
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
for xm in 1 0; do
  out=gpurun_out/wide_prof_x$xm.bin; rm -f $out
  HMCX_WIDE_XMAP=$xm HMCX_WIDE_PROF=$R/$out timeout -k 10 60 python tools/probe_sgld.py 64 > gpurun_out/wide_probe.txt 2>&1 || { tail gpurun_out/wide_probe.txt; exit 1; }
  echo "== xmap=$xm"; python3 tools/wide_prof_summary.py $out fused
done
for i in 1 2; do
echo "fused xmap $(timeout -k 10 60 python tools/probe_sgld.py 400 2>&1 | tail -1)"
echo "fused      $(HMCX_WIDE_XMAP=0 timeout -k 10 60 python tools/probe_sgld.py 400 2>&1 | tail -1)"
echo "3-launch   $(HMCX_WIDE_FUSE=0 timeout -k 10 60 python tools/probe_sgld.py 400 2>&1 | tail -1)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_chains.py -k "sgld" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_b.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_b.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_b.log
