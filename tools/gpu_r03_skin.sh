#!/bin/bash
# Headline kernel with the row-team accept round (slice kinetics, ll(q0) through the iteration-0
# headers): SGHMC parity tests, then same-box A/B against the previous library (HMCX_LIB=libhmcx_p0.so)
# at the driver's shape and at 600 steps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_recovery.py tests/test_gpu_nan.py tests/test_gpu_edges.py tests/test_gpu_multicore.py tests/test_gpu_statistics.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not mlp and not sgld" > gpurun_out/pytest_skin.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_skin.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_skin.log
HMCX_PERSIST_PROF=1 timeout -k 10 120 python tools/probe_sghmc.py 2>&1 | grep "p2 prof" | tail -1
for rep in 1 2 3; do
  for L in p0 new; do
    if [ $L = new ]; then unset HMCX_LIB; else export HMCX_LIB=libhmcx_$L.so; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/h.json 2> gpurun_out/h.err || { tail gpurun_out/h.err; exit 1; }
    echo "$L s20 $(python3 -c "import json; d=json.load(open('gpurun_out/h.json')); print('%.4g' % d['value'], 'launch_ms %.4f' % d['roofline']['launch_ms'], 'lf', d['leapfrogs'])")"
    timeout -k 10 300 python bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/s600.json 2> gpurun_out/s600.err || { tail gpurun_out/s600.err; exit 1; }
    echo "$L s600 $(python3 -c "import json; d=json.load(open('gpurun_out/s600.json')); print('%.4g' % d['value'], 'launch_ms %.4f' % d['roofline']['launch_ms'])")"
  done
done
unset HMCX_LIB
