#!/bin/bash
# Batched MLP iterations: MLP GPU tests, then the config-3 probe (f32, f64) on the round-start library
# ($A), the current one, and the current one with the 3-per-CU fused forward (HMCX_MLP_L23W=6), N
# alternating rounds; kernel stats of the current library under rocprofv3.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
A=${A:-libhmcx_base.so}; N=${N:-2}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_statistics.py -k "mlp or MLP or grad or masks or predict or sghmc or batched" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_mlp.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_mlp.log
fi
for rep in $(seq $N); do
  for dt in f32 f64; do
    echo "[$A $dt] $(HMCX_LIB=$A timeout -k 10 120 python tools/probe_mlp.py $dt 40 2>&1 | tail -1)"
    echo "[new $dt] $(timeout -k 10 120 python tools/probe_mlp.py $dt 40 2>&1 | tail -1)"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in 4; do
  HMCX_MLP_L23W=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mlpb_$v -o run --output-format csv -- python3 $R/tools/probe_mlp.py 40 > $R/gpurun_out/probe_mlpb_prof.txt 2>&1 || { tail -5 $R/gpurun_out/probe_mlpb_prof.txt; exit 1; }
  echo "== L23W=$v"
  python3 -c "
import csv
rows = list(csv.DictReader(open('$R/gpurun_out/prof_mlpb_$v/run_kernel_stats.csv')))
tot = sum(float(r['TotalDurationNs']) for r in rows if 'hmcx' in r['Name'])
print('hmcx kernels total %.2f ms' % (tot / 1e6))
for r in rows[:14]:
    print('  ', r['Name'][:70], r['Calls'], '%.1f' % (float(r['AverageNs'])/1e3))
"
done
