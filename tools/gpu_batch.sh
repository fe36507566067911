#!/bin/bash
# Chain-batched path: GPU chain tests, then the batched probe and its kernel profile.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_chains.py -x -q > gpurun_out/pytest_chains.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_chains.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/pytest_chains.log | head -20; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profb -o run --output-format csv -- python3 $R/tools/probe_batch.py ${CS:-1024} > $R/gpurun_out/profb.log 2>&1 || { tail -5 $R/gpurun_out/profb.log; exit 1; }
grep "C=" $R/gpurun_out/profb.log
cut -c1-160 $R/gpurun_out/profb/run_kernel_stats.csv | head -6
