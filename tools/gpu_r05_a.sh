#!/bin/bash
# Round 5, first box: row-space iteration probe, then the GPU suite with the recovery guard, smoke, and
# the driver-shape bench line (per-rank aggregates, recoveries).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/microbench_rowspace > gpurun_out/mb_rowspace.txt 2>&1; echo "microbench rc $?"; cat gpurun_out/mb_rowspace.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r05a.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_r05a.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r05a.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r05a_s20.json 2> gpurun_out/bench_r05a_s20.err || { echo bench failed; tail gpurun_out/bench_r05a_s20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r05a_s20.json')); print('s20', d['value'], d['roofline']['frac'], d['recoveries'], d['ranks']['predicted']['8'])"
