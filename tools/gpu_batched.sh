#!/bin/bash
# Chain-batched path: parity tests and the bench's 2048-chain leg (MFMA roofline fraction).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chains.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_chains.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_chains.log; exit 1; }
tail -1 gpurun_out/pytest_chains.log
timeout -k 10 300 python bench.py --steps 120 --cpu-seconds 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { tail gpurun_out/bench_b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_b.json'))['chain_batched']; print('batched', d['leapfrogs_per_s'], d['roofline']['frac'], d['roofline']['device_ms'])"
