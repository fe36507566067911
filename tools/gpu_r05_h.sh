#!/bin/bash
# Round 5 milestone check: full GPU suite (recovery guard, device diagnostics), smoke, default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r05h.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_r05h.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r05h.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 400 python bench.py > gpurun_out/bench_r05h.json 2> gpurun_out/bench_r05h.err || { echo bench failed; tail gpurun_out/bench_r05h.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r05h.json')); print('default', d['value'], d['roofline']['frac'], d['recoveries'], d['diagnostics']['per_parameter'], d['chain_batched']['sweep'], d['mlp']['roofline']['frac'], d['plantvillage_sgld']['us_per_step'])"
