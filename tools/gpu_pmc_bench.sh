#!/bin/bash
# Round profile session: GPU tests, default bench, rocprofv3 kernel-trace stats of the bench, and
# the two PMC passes (FETCH_SIZE, WRITE_SIZE: separate passes, TCC slot limits) for HBM traffic.
set -o pipefail
R=$(pwd)
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 > $R/gpurun_out/bench_prof_$TAG.json 2> $R/gpurun_out/prof_$TAG.err || { tail -5 $R/gpurun_out/prof_$TAG.err; exit 1; }
cat $R/gpurun_out/bench_prof_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmcf_$TAG -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > $R/gpurun_out/bench_pmcf_$TAG.json 2> $R/gpurun_out/pmcf_$TAG.err || { tail -5 $R/gpurun_out/pmcf_$TAG.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmcw_$TAG -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > $R/gpurun_out/bench_pmcw_$TAG.json 2> $R/gpurun_out/pmcw_$TAG.err || { tail -5 $R/gpurun_out/pmcw_$TAG.err; exit 1; }
cd $R && python3 tools/pmc_summary.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG "k_sghmc_p2<double, 10>" gpurun_out/pmc_${TAG}_f64_persistent.json
echo done
