#!/bin/bash
# One GPU session: tests, bench (both SGHMC paths), rocprofv3 kernel stats of the default bench.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo bench failed; tail gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 200 python bench.py --path kernels --cpu-seconds 0 > gpurun_out/bench_kernels.json 2> gpurun_out/bench_kernels.err || { echo bench2 failed; tail gpurun_out/bench_kernels.err; exit 1; }
cat gpurun_out/bench_kernels.json
timeout -k 10 200 python bench.py --dtype f32 --cpu-seconds 0 > gpurun_out/bench_f32.json 2> gpurun_out/bench_f32.err || { echo bench3 failed; exit 1; }
cat gpurun_out/bench_f32.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/prof.err || { echo prof failed; tail $R/gpurun_out/prof.err; exit 1; }
cat $R/gpurun_out/bench_prof.json
find $R/gpurun_out/prof -name "*stats*"
