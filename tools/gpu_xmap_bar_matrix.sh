#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for cfg in "1 0" "0 0" "0 1" "1 1"; do set -- $cfg
  HMCX_P2_BAR=$1 HMCX_P2_XMAP=$2 timeout -k 10 60 python tools/probe_sghmc.py reps=9 > gpurun_out/ab.log 2>&1 || { tail gpurun_out/ab.log; exit 1; }
  echo "[BAR=$1 XMAP=$2] $(tail -1 gpurun_out/ab.log | grep -o 'us/lf [0-9.]*')"
done; done
HMCX_P2_TRACE=1 timeout -k 10 60 python tools/probe_sghmc.py reps=3 > gpurun_out/trace.log 2>&1 || { tail gpurun_out/trace.log; exit 1; }
grep -i "p2 trace\|round\|A-RS\|B-AR" gpurun_out/trace.log | head -20
