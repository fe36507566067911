#!/bin/bash
# Same-box A/B of MLP sampler variants selected by environment (one library):
# r02 library, then this build with HMCX_MLP_MASKS=keep / philox and HMCX_MLP_H1=0 / 1; N rounds.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
N=${N:-2}
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_mlp.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_mlp.log
for rep in $(seq $N); do
  echo "[r02] $(HMCX_LIB=libhmcx_r02.so timeout -k 10 120 python tools/probe_mlp.py 40 2>&1 | tail -1)"
  for m in keep philox; do for h in 0 1; do
    echo "[masks=$m h1=$h] $(HMCX_MLP_MASKS=$m HMCX_MLP_H1=$h timeout -k 10 120 python tools/probe_mlp.py 40 2>&1 | tail -1)"
  done; done
done
rm -f gpurun_out/mlp_prof.bin
HMCX_MLP_PROF=$R/gpurun_out/mlp_prof.bin timeout -k 10 120 python tools/probe_mlp.py 40 2>&1 | tail -1
python tools/mlp_prof_summary.py gpurun_out/mlp_prof.bin
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mlp -o run --output-format csv -- python3 $R/tools/probe_mlp.py 40 > $R/gpurun_out/probe_mlp_prof.txt 2>&1 || { tail -5 $R/gpurun_out/probe_mlp_prof.txt; exit 1; }
python3 -c "
import csv
rows = list(csv.DictReader(open('$R/gpurun_out/prof_mlp/run_kernel_stats.csv')))
tot = sum(float(r['TotalDurationNs']) for r in rows if 'hmcx' in r['Name'])
print('hmcx kernels total %.2f ms' % (tot / 1e6))
for r in rows[:12]:
    print('  ', r['Name'][:64], r['Calls'], '%.1f' % (float(r['AverageNs'])/1e3))
"
