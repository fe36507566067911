#!/bin/bash
# Wide SGLD: parity tests, phase stamps (write-through default), A/B plain vs write-through vs v1.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_statistics.py -m gpu -x -q --timeout 200 --timeout-method thread -k "sgld or wide" > gpurun_out/pytest_wide2.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_wide2.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_wide2.log
rm -f gpurun_out/wide_prof3.bin
HMCX_WIDE_PROF=$R/gpurun_out/wide_prof3.bin timeout -k 10 120 python tools/probe_sgld.py 64 > gpurun_out/wide_probe3.txt 2>&1 || { tail gpurun_out/wide_probe3.txt; exit 1; }
python3 tools/wide_prof_summary.py gpurun_out/wide_prof3.bin
for rep in 1 2 3; do
  echo "v1   $(HMCX_WIDE_V=1 timeout -k 10 120 python tools/probe_sgld.py 400 2>&1 | grep -v amdgpu.ids)"
  echo "v2   $(HMCX_WIDE_WT=0 timeout -k 10 120 python tools/probe_sgld.py 400 2>&1 | grep -v amdgpu.ids)"
  echo "v2wt $(timeout -k 10 120 python tools/probe_sgld.py 400 2>&1 | grep -v amdgpu.ids)"
done
echo "f32 v2wt $(timeout -k 10 120 python tools/probe_sgld.py f32 400 2>&1 | grep -v amdgpu.ids)"
