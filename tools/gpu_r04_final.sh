#!/bin/bash
# Round-4 closing run on the final build: full GPU suite, smoke, the default bench line and the driver's
# shape (--steps 20 --warmup 5), the rocprofv3 kernel-trace summary of the default command, and the PMC
# fabric traffic of the headline kernel at the driver's shape (profiles/).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_gpu.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo bench failed; tail gpurun_out/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['chain_batched']['roofline']['frac'], d['chain_batched']['sweep'], d['mlp']['roofline']['frac'], d['plantvillage_sgld']['us_per_step'])"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.json 2> gpurun_out/bench_s20.err || { echo bench s20 failed; tail gpurun_out/bench_s20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s20.json')); print('s20', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r04 -o run --output-format csv -- python3 $R/bench.py > $R/gpurun_out/bench_prof_r04.json 2> $R/gpurun_out/prof_r04.err || { tail -5 $R/gpurun_out/prof_r04.err; exit 1; }
echo prof done
cd $R && TAG=r04 bash tools/gpu_pmc_headline.sh
