#!/bin/bash
# Host overhead at the driver's call shape: bench.py --steps 20 --warmup 5 (headline leg only) with and
# without the per-step trace dicts, alternating, then the 600-step reference line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_recovery.py tests/test_gpu_samplers.py tests/test_gpu_nan.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_p2.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_p2.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_p2.log
for rep in 1 2 3 4; do for tr in 1 0; do
  HMCX_BENCH_TRACE=$tr HMCX_BENCH_DEBUG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/h.json 2> gpurun_out/h.err || { tail gpurun_out/h.err; exit 1; }
  echo "[trace=$tr] $(python3 -c "import json; d=json.load(open('gpurun_out/h.json')); print('%.4g' % d['value'], 'wall_ms %.4f' % (d['ms_per_step']*20), 'launch_ms %.4f' % d['roofline']['launch_ms'])") | $(grep 'timed region' gpurun_out/h.err)"
done; done
timeout -k 10 300 python bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/s600.json 2> gpurun_out/s600.err || { tail gpurun_out/s600.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s600.json')); print('s600 %.4g' % d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
