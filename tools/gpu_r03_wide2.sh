#!/bin/bash
# Wide SGLD kernels v2 (k_wfwd2 / k_wgrad2): parity tests, phase stamps, A/B against v1 (same box).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_statistics.py -m gpu -x -q --timeout 200 --timeout-method thread -k "sgld or wide" > gpurun_out/pytest_wide2.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_wide2.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_wide2.log
rm -f gpurun_out/wide_prof2.bin
HMCX_WIDE_PROF=$R/gpurun_out/wide_prof2.bin timeout -k 10 120 python tools/probe_sgld.py 64 > gpurun_out/wide_probe2.txt 2>&1 || { tail gpurun_out/wide_probe2.txt; exit 1; }
python3 tools/wide_prof_summary.py gpurun_out/wide_prof2.bin
for rep in 1 2 3; do
  for v in 1 2 2wt; do
    if [ $v = 2wt ]; then export HMCX_WIDE_WT=1; V=2; else unset HMCX_WIDE_WT; V=$v; fi
    echo "v$v $(HMCX_WIDE_V=$V timeout -k 10 120 python tools/probe_sgld.py 400 2>&1 | grep -v amdgpu.ids)"
  done
done
unset HMCX_WIDE_WT
echo "f32 v2 $(timeout -k 10 120 python tools/probe_sgld.py f32 400 2>&1 | grep -v amdgpu.ids)"
