#!/bin/bash
# Round-3 closing run: full GPU suite, smoke, the default bench line (what the driver runs), and the
# rocprofv3 kernel-trace summary of the same command (profiles/).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_gpu.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo bench failed; tail gpurun_out/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['chain_batched']['roofline']['frac'], d['mlp']['roofline']['frac'], d['plantvillage_sgld']['us_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r03 -o run --output-format csv -- python3 $R/bench.py > $R/gpurun_out/bench_prof_r03.json 2> $R/gpurun_out/prof_r03.err || { tail -5 $R/gpurun_out/prof_r03.err; exit 1; }
echo prof done
