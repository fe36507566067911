#!/bin/bash
# Probe timing with and without the in-kernel profiler for a few team grids.
set -o pipefail
mkdir -p gpurun_out
for g in ${GRIDS:-8x8 16x8}; do
  for pr in 0 1; do
    HMCX_P2_GRID=$g HMCX_PERSIST_PROF=$pr timeout -k 10 60 python tools/probe_sghmc.py > gpurun_out/cmp_${g}_$pr.log 2>&1 || { tail gpurun_out/cmp_${g}_$pr.log; exit 1; }
    echo "$g prof=$pr $(tail -1 gpurun_out/cmp_${g}_$pr.log | grep -o 'us/lf [0-9.]*')"; grep "prof\]" gpurun_out/cmp_${g}_$pr.log | tail -1
  done
done
