#!/bin/bash
# Persistent SGHMC grid shapes (HMCX_P2_GRID=GrxGf) on the MNIST probe, 3 rounds.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for g in ${GRIDS:-8x16 16x8 8x8 16x16 4x16}; do
  HMCX_P2_GRID=$g timeout -k 10 60 python tools/probe_sghmc.py > gpurun_out/ab.log 2>&1 || { tail gpurun_out/ab.log; exit 1; }
  echo "[grid=$g] $(tail -1 gpurun_out/ab.log | grep -o 'us/lf [0-9.]*')"
done; done
