#!/bin/bash
# Chain-batched gradient-kernel epilogue A/B: library A (HMCX_LIB=libhmcx_base.so) vs B (libhmcx.so)
# on the 2048-chain probe, 3 alternating pairs, after the chain-batched parity / statistics / NaN
# tests on build B; then rocprofv3 kernel stats of the probe on build B.
set -o pipefail
mkdir -p gpurun_out
A=${A:-libhmcx_base.so}; B=${B:-libhmcx.so}
HMCX_LIB=$B timeout -k 10 400 python -u -m pytest tests/test_gpu_chains.py tests/test_gpu_statistics.py tests/test_gpu_nan.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_bepi.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_bepi.log | tail -20; exit 1; }
tail -1 gpurun_out/pytest_bepi.log
for rep in 1 2 3; do for lib in $A $B; do
  HMCX_LIB=$lib timeout -k 10 120 python tools/probe_batch.py ${CS:-2048} > gpurun_out/bepi.log 2>&1 || { tail gpurun_out/bepi.log; exit 1; }
  echo "[$lib] $(tail -1 gpurun_out/bepi.log)"
done; done
R=$(pwd); cd /tmp && export TMPDIR=/tmp
HMCX_LIB=$B timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bepi -o run --output-format csv -- python3 $R/tools/probe_batch.py ${CS:-2048} > $R/gpurun_out/bepi_prof.log 2>&1 || { echo prof failed; tail $R/gpurun_out/bepi_prof.log; exit 1; }
find $R/gpurun_out/prof_bepi -name "*stats*"
