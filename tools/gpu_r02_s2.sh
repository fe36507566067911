#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/probe_overhead.py steps=20 reps=50 > gpurun_out/probe_s20.txt 2>&1 || { tail gpurun_out/probe_s20.txt; exit 1; }
cat gpurun_out/probe_s20.txt
timeout -k 10 120 python -m cProfile -s tottime tools/probe_overhead.py steps=20 reps=300 > gpurun_out/probe_cprof.txt 2>&1 || { tail gpurun_out/probe_cprof.txt; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/bench_s20.json 2> gpurun_out/bench_s20.err || { echo bench failed; tail gpurun_out/bench_s20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s20.json')); print('s20', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['traffic'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_gpu.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
