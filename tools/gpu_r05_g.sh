#!/bin/bash
# Round 5: which chain-batched change costs time — one library per change (tools/: variant builds of
# hmcx_batch.h), 2048 chains, two alternating passes.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in libhmcx_base.so libhmcx_vF.so libhmcx_vG.so libhmcx_vS.so libhmcx_vGS.so libhmcx_vB.so libhmcx.so; do
    HMCX_LIB=$lib timeout -k 10 200 python tools/probe_batch.py 2048 2>&1 | grep "C=" | sed "s/^/$lib /" | awk '{print $1, $2, $10, $11, $12}'
  done
done
