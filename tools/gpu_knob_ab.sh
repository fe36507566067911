#!/bin/bash
# Persistent SGHMC transport knobs against the defaults on the MNIST probe, 3 rounds.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for k in HMCX_P2_DEFAULT=1 HMCX_P2_PAD=0 HMCX_P2_ZOFF=0 HMCX_P2_FL2=0 HMCX_P2_PREFETCH=0; do
  env $k timeout -k 10 60 python tools/probe_sghmc.py > gpurun_out/ab.log 2>&1 || { tail gpurun_out/ab.log; exit 1; }
  echo "[$k] $(tail -1 gpurun_out/ab.log | grep -o 'us/lf [0-9.]*')"
done; done
