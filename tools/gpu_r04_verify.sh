#!/bin/bash
# Final-build check: full GPU suite, smoke, default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_final.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo bench failed; tail gpurun_out/bench_final.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_final.json')); print('default', d['value'], d['roofline']['frac'], d['roofline']['traffic_source'][-60:], d['chain_batched']['roofline']['frac'], d['mlp']['roofline']['frac'], d['plantvillage_sgld']['us_per_step'])"
