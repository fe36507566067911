#!/bin/bash
# Full GPU suite (incl. the 4-rank shared-GPU bench), smoke, driver-shape bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=12 --timeout 450 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_gpu.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
grep -E "slowest|^[0-9.]+s (call|setup)" gpurun_out/pytest_gpu.log | head -12
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.json 2> gpurun_out/bench_s20.err || { echo bench failed; tail gpurun_out/bench_s20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s20.json')); print('s20', d['value'], d['ms_per_step'], d['mlp']['roofline']['frac'], d['mlp']['leapfrogs_per_s'], d['chain_batched']['roofline']['frac'], d['plantvillage_sgld']['us_per_step'], d['cpu_baseline']['calibration_ratio'])"
