#!/bin/bash
# MLP (config 3): GPU tests of the MLP + recovery, probe timing, in-kernel L23 phase profile, and
# rocprofv3 kernel stats of the probe.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_mlp.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_mlp.log
timeout -k 10 120 python tools/probe_mlp.py 40 2>&1 | tail -2
rm -f gpurun_out/mlp_prof.bin
HMCX_MLP_PROF=$R/gpurun_out/mlp_prof.bin timeout -k 10 120 python tools/probe_mlp.py 40 2>&1 | tail -1
python tools/mlp_prof_summary.py gpurun_out/mlp_prof.bin
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mlp -o run --output-format csv -- python3 $R/tools/probe_mlp.py 40 > $R/gpurun_out/probe_mlp_prof.txt 2>&1 || { tail -5 $R/gpurun_out/probe_mlp_prof.txt; exit 1; }
cd $R && python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_mlp/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], '%.1f' % (float(r['AverageNs'])/1e3))
" | head -16
