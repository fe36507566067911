#!/bin/bash
# Round-2 closing measurement on the final build: full GPU test suite, the driver-shape bench line
# (all legs), the 600-step headline, rocprofv3 kernel stats of the driver shape, PMC traffic of the
# headline kernel (FETCH_SIZE / WRITE_SIZE passes), and the SQ counters of the 2048-chain batched probe.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_gpu.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.json 2> gpurun_out/bench_s20.err || { echo bench failed; tail gpurun_out/bench_s20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s20.json')); print('s20', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['chain_batched']['roofline']['frac'])"
timeout -k 10 300 python bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/bench_s600.json 2> gpurun_out/bench_s600.err || { echo bench2 failed; tail gpurun_out/bench_s600.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s600.json')); print('s600', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_s20 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/prof.err || { echo prof failed; tail $R/gpurun_out/prof.err; exit 1; }
cd $R && TAG=r02f bash tools/gpu_pmc_headline.sh || exit 1
CS=2048 bash tools/gpu_pmc_batch.sh || exit 1
python3 tools/pmc_batch_summary.py gpurun_out/pmcb "python3 tools/probe_batch.py 2048" gpurun_out/pmc_r02_batched_sq.json
