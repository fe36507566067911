#!/bin/bash
# Bench + rocprofv3 kernel-trace stats of the default bench, plus the in-kernel phase profile.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo bench failed; tail gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
HMCX_PERSIST_PROF=1 timeout -k 10 120 python tools/probe_sghmc.py > gpurun_out/probe_prof.log 2>&1 || { echo probe failed; tail gpurun_out/probe_prof.log; exit 1; }
tail -4 gpurun_out/probe_prof.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/prof.err || { echo prof failed; grep -v "^    @" $R/gpurun_out/prof.err | tail -5; exit 1; }
cat $R/gpurun_out/bench_prof.json
cat $R/gpurun_out/prof/run_kernel_stats.csv
