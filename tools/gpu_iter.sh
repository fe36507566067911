#!/bin/bash
# One GPU iteration: sampler + MLP parity tests, config-5 SGLD probes (wide path vs kernel-per-phase
# path), the config-3 MLP probe, and rocprofv3 kernel stats of both probes.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
for w in 1 0; do
  for a in "200" "f32 200"; do
    HMCX_SGLD_WIDE=$w timeout -k 10 120 python tools/probe_sgld.py $a > gpurun_out/probe_sgld.log 2>&1 || { tail gpurun_out/probe_sgld.log; exit 1; }
    echo "wide=$w $(tail -1 gpurun_out/probe_sgld.log)"
  done
done
timeout -k 10 120 python tools/probe_mlp.py 20 > gpurun_out/probe_mlp_f32.log 2>&1 || { tail gpurun_out/probe_mlp_f32.log; exit 1; }
tail -1 gpurun_out/probe_mlp_f32.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_wide -o run --output-format csv -- python3 $R/tools/probe_sgld.py 200 > $R/gpurun_out/prof_wide.log 2>&1 || { tail -5 $R/gpurun_out/prof_wide.log; exit 1; }
cut -d, -f1-4 $R/gpurun_out/prof_wide/run_kernel_stats.csv
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mlp -o run --output-format csv -- python3 $R/tools/probe_mlp.py 20 > $R/gpurun_out/prof_mlp.log 2>&1 || { tail -5 $R/gpurun_out/prof_mlp.log; exit 1; }
cut -d, -f1-4 $R/gpurun_out/prof_mlp/run_kernel_stats.csv
