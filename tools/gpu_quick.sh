#!/bin/bash
# Quick GPU iteration: GPU tests, then the SGHMC probe over several team grids.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
for g in ${GRIDS:-auto 4x4 8x4 4x8 8x8 16x8 8x16}; do
  if [ $g = auto ]; then unset HMCX_P2_GRID; else export HMCX_P2_GRID=$g; fi
  HMCX_PERSIST_PROF=${PROF:-0} timeout -k 10 60 python tools/probe_sghmc.py > gpurun_out/probe_$g.log 2>&1 || { tail gpurun_out/probe_$g.log; exit 1; }
  echo "$g $(tail -1 gpurun_out/probe_$g.log)"; grep "prof\]" gpurun_out/probe_$g.log | tail -1
done
unset HMCX_P2_GRID
timeout -k 10 60 python tools/probe_sghmc.py f32 2>&1 | tail -1
