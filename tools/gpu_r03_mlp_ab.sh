#!/bin/bash
# Same-box A/B of the config-3 MLP probe: HMCX_LIB=$A vs $B alternating (N pairs), then kernel stats
# of both under rocprofv3.  Usage: A=libhmcx_r02.so B=libhmcx.so N=3 bash tools/gpu_r03_mlp_ab.sh
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
A=${A:-libhmcx_r02.so}; B=${B:-libhmcx.so}; N=${N:-3}
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_statistics.py -k "mlp or MLP or grad or masks or predict or sghmc" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_mlp.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_mlp.log
for rep in $(seq $N); do for lib in $A $B; do
  echo "[$lib] $(HMCX_LIB=$lib timeout -k 10 120 python tools/probe_mlp.py 40 2>&1 | tail -1)"
done; done
cd /tmp && export TMPDIR=/tmp
for lib in $A $B; do
  HMCX_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mlp_$lib -o run --output-format csv -- python3 $R/tools/probe_mlp.py 40 > $R/gpurun_out/probe_mlp_prof.txt 2>&1 || { tail -5 $R/gpurun_out/probe_mlp_prof.txt; exit 1; }
  echo "== $lib"
  python3 -c "
import csv
rows = list(csv.DictReader(open('$R/gpurun_out/prof_mlp_$lib/run_kernel_stats.csv')))
tot = sum(float(r['TotalDurationNs']) for r in rows if 'hmcx' in r['Name'])
print('hmcx kernels total %.2f ms' % (tot / 1e6))
for r in rows[:12]:
    print('  ', r['Name'][:64], r['Calls'], '%.1f' % (float(r['AverageNs'])/1e3))
"
done
