#!/bin/bash
# Round 5: per-kernel totals of the 2048-chain call, pipelined build vs the round-start build.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for lib in libhmcx.so libhmcx_base.so; do
  HMCX_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/bk_$lib -o run -- python3 $R/tools/probe_batch.py 2048 > $R/gpurun_out/bk_$lib.log 2>&1 || { tail -5 $R/gpurun_out/bk_$lib.log; exit 1; }
  KT=$(find $R/gpurun_out/bk_$lib -name "*kernel_trace.csv" | head -1)
  echo "== $lib"; python3 $R/tools/batch_launch_profile.py $KT | grep "total"
done
