#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the persistent kernel with HMCX_P2_PAD=0 (separate passes).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
export HMCX_P2_PAD=0
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmcf_pad0 -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > $R/gpurun_out/bench_pmcf_pad0.json 2> $R/gpurun_out/pmcf_pad0.err || { tail -5 $R/gpurun_out/pmcf_pad0.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmcw_pad0 -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > $R/gpurun_out/bench_pmcw_pad0.json 2> $R/gpurun_out/pmcw_pad0.err || { tail -5 $R/gpurun_out/pmcw_pad0.err; exit 1; }
cd $R && python3 tools/pmc_summary.py gpurun_out/pmcf_pad0 gpurun_out/pmcw_pad0 "k_sghmc_p2<double, 10>" gpurun_out/pmc_pad0.json
