#!/bin/bash
# A/B timing of the persistent SGHMC probe under two environment settings: gpu_ab.sh "A=1" "A=0"
set -o pipefail
mkdir -p gpurun_out
for rep in $(seq ${AB_REPS:-3}); do
for cfg in "$@"; do
  env $cfg timeout -k 10 60 python tools/probe_sghmc.py > gpurun_out/ab.log 2>&1 || { tail gpurun_out/ab.log; exit 1; }
  echo "[$cfg] $(tail -1 gpurun_out/ab.log | grep -o 'us/lf [0-9.]*')"
done
done
env $1 HMCX_P2_TRACE=1 timeout -k 10 60 python tools/probe_sghmc.py 2>&1 | grep trace
