#!/bin/bash
# rocprofv3 kernel stats of the chain-batched SGHMC probe.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profb -o run --output-format csv -- python3 $R/tools/probe_batch.py ${CS:-1024} > $R/gpurun_out/profb.log 2>&1 || { tail -5 $R/gpurun_out/profb.log; exit 1; }
tail -2 $R/gpurun_out/profb.log
cut -c1-160 $R/gpurun_out/profb/run_kernel_stats.csv
