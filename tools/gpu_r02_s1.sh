#!/bin/bash
# Round-2 session: recovery + sampler GPU tests, host-overhead probe, bench at the driver shape and
# at 600 steps, PMC traffic at the driver shape.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_recovery.py tests/test_gpu_samplers.py tests/test_gpu_multicore.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_s1.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error|recovered|no timeout" gpurun_out/pytest_s1.log | tail -40; exit 1; }
grep -E "passed|failed|recovered|no timeout" gpurun_out/pytest_s1.log | tail -5
timeout -k 10 120 python tools/probe_overhead.py steps=20 reps=50 > gpurun_out/probe_s20.txt 2>&1 || { tail gpurun_out/probe_s20.txt; exit 1; }
cat gpurun_out/probe_s20.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.json 2> gpurun_out/bench_s20.err || { echo bench failed; tail gpurun_out/bench_s20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s20.json')); print('s20', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
timeout -k 10 300 python bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/bench_s600.json 2> gpurun_out/bench_s600.err || { echo bench2 failed; tail gpurun_out/bench_s600.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s600.json')); print('s600', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
bash tools/gpu_r02_pmc.sh
