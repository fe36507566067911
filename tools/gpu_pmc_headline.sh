#!/bin/bash
# PMC traffic of the headline kernel at the driver's call shape (bench.py --steps 20 --warmup 5):
# FETCH_SIZE and WRITE_SIZE in separate passes (TCC slot limits), summarised per leapfrog.
set -o pipefail
R=$(pwd)
TAG=${TAG:-r03}
STEPS=${STEPS:-20}
WARM=${WARM:-5}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
ARGS="--steps $STEPS --warmup $WARM --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmcf_$TAG -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/bench_pmcf_$TAG.json 2> $R/gpurun_out/pmcf_$TAG.err || { tail -5 $R/gpurun_out/pmcf_$TAG.err; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmcw_$TAG -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/bench_pmcw_$TAG.json 2> $R/gpurun_out/pmcw_$TAG.err || { tail -5 $R/gpurun_out/pmcw_$TAG.err; exit 1; }
cd $R && python3 tools/pmc_summary.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG "k_sghmc_p2<double, 10" gpurun_out/bench_pmcf_$TAG.json gpurun_out/pmc_${TAG}_f64_persistent.json
