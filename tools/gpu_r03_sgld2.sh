#!/bin/bash
# Config 5 SGLD: parity tests, then same-box A/B of the gradient (split vs k_wgrad) and kernel stats.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_statistics.py -k "sgld" -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/pytest_sgld.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_sgld.log | tail -40; exit 1; }
tail -1 gpurun_out/pytest_sgld.log
for rep in 1 2; do for sp in 0 1; do
  echo "[split=$sp] $(HMCX_WGRAD_SPLIT=$sp timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 400 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin)['plantvillage_sgld']; print('us/step %.2f' % d['us_per_step'], 'frac %.4f' % d['roofline']['frac'])")"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sgld -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 400 > $R/gpurun_out/sgld_prof.json 2> $R/gpurun_out/sgld_prof.err || { tail -5 $R/gpurun_out/sgld_prof.err; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$R/gpurun_out/prof_sgld/run_kernel_stats.csv')))[:9]:
    print('  ', r['Name'][:64], r['Calls'], '%.1f' % (float(r['AverageNs'])/1e3))
"
