#!/bin/bash
# A/B of two library builds on the bench's headline line at the driver's call shape
# (HMCX_LIB=<A> vs <B>, alternating, N pairs), after the persistent-path parity tests on build B.
# Usage: A=libhmcx_base.so B=libhmcx.so N=4 [TESTS="tests/..."] bash tools/gpu_lib_ab.sh
set -o pipefail
mkdir -p gpurun_out
A=${A:-libhmcx_base.so}; B=${B:-libhmcx.so}; N=${N:-4}
T=${TESTS:-tests/test_gpu_samplers.py tests/test_gpu_recovery.py tests/test_gpu_nan.py tests/test_gpu_mlp.py}
HMCX_LIB=$B timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_ab.log | tail -30; exit 1; }
echo "tests ($B): $(tail -1 gpurun_out/pytest_ab.log)"
for rep in $(seq $N); do for lib in $A $B; do
  HMCX_LIB=$lib HMCX_BENCH_DEBUG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  echo "[$lib] $(python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('%.4g' % d['value'], 'wall_ms %.4f' % (d['ms_per_step']*20), 'launch_ms %.4f' % d['roofline']['launch_ms'])") | $(grep 'timed region' gpurun_out/ab.err)"
done; done
