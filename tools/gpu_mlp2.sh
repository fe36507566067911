#!/bin/bash
# MLP iteration: parity tests, config-3 probe, kernel stats.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_mlp.log; exit 1; }
tail -2 gpurun_out/pytest_mlp.log
timeout -k 10 120 python tools/probe_mlp.py 20 > gpurun_out/probe_mlp_f32.log 2>&1 || { tail gpurun_out/probe_mlp_f32.log; exit 1; }
tail -1 gpurun_out/probe_mlp_f32.log
timeout -k 10 120 python tools/probe_mlp.py f64 20 > gpurun_out/probe_mlp_f64.log 2>&1 || { tail gpurun_out/probe_mlp_f64.log; exit 1; }
tail -1 gpurun_out/probe_mlp_f64.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mlp -o run --output-format csv -- python3 $R/tools/probe_mlp.py 20 > $R/gpurun_out/prof_mlp.log 2>&1 || { tail -5 $R/gpurun_out/prof_mlp.log; exit 1; }
echo prof done
