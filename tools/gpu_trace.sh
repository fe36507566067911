#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for g in ${GRIDS:-8x16 16x8 8x8}; do
  HMCX_P2_GRID=$g HMCX_P2_TRACE=1 timeout -k 10 60 python tools/probe_sghmc.py > gpurun_out/trace_$g.log 2>&1 || { tail gpurun_out/trace_$g.log; exit 1; }
  echo "== $g"; grep "trace\]" gpurun_out/trace_$g.log | tail -5
done
