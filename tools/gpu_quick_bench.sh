#!/bin/bash
# Sampler parity tests + default bench (headline line only printed).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { tail gpurun_out/bench_q.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_q.json')); print(d['value'], d['leapfrogs_per_s'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
