#!/bin/bash
# Config-5 SGLD probe (D=2048, K=38) and its kernel profile.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
for a in "200" "f32 200" "200 8"; do
  timeout -k 10 120 python tools/probe_sgld.py $a > gpurun_out/probe_sgld.log 2>&1 || { tail gpurun_out/probe_sgld.log; exit 1; }
  tail -1 gpurun_out/probe_sgld.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sgld -o run --output-format csv -- python3 $R/tools/probe_sgld.py 200 > $R/gpurun_out/prof_sgld.log 2>&1 || { tail -5 $R/gpurun_out/prof_sgld.log; exit 1; }
cut -d, -f1-4 $R/gpurun_out/prof_sgld/run_kernel_stats.csv | head -8
