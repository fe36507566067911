#!/bin/bash
# MLP (config 3) GPU iteration: MLP parity tests, then the config-3 SGHMC probe (f32, f64) and a
# kernel-stats profile of the f32 probe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_mlp.py -x -q > gpurun_out/pytest_mlp.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_mlp.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert|Assert" gpurun_out/pytest_mlp.log | head -30; exit $rc; }
timeout -k 10 120 python tools/probe_mlp.py 20 > gpurun_out/probe_mlp_f32.log 2>&1 || { tail gpurun_out/probe_mlp_f32.log; exit 1; }
tail -1 gpurun_out/probe_mlp_f32.log
timeout -k 10 120 python tools/probe_mlp.py f64 20 > gpurun_out/probe_mlp_f64.log 2>&1 || { tail gpurun_out/probe_mlp_f64.log; exit 1; }
tail -1 gpurun_out/probe_mlp_f64.log
timeout -k 10 120 python tools/probe_mlp.py 20 graph > gpurun_out/probe_mlp_graph.log 2>&1 || { tail gpurun_out/probe_mlp_graph.log; exit 1; }
tail -1 gpurun_out/probe_mlp_graph.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp -o run --output-format csv -- python3 tools/probe_mlp.py 20 > gpurun_out/prof_mlp.log 2>&1 || { tail gpurun_out/prof_mlp.log; exit 1; }
f=$(find gpurun_out/prof_mlp -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -20
