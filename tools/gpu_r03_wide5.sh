#!/bin/bash
# Wide SGLD, class-group gradient (256 workgroups, bias from the tile-0 blocks): parity tests, phase
# stamps, same-box A/B against the previous library (HMCX_LIB=libhmcx_w1.so).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_statistics.py tests/test_gpu_chains.py -m gpu -x -q --timeout 200 --timeout-method thread -k "sgld or wide" > gpurun_out/pytest_wide5.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_wide5.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_wide5.log
rm -f gpurun_out/wide_prof5.bin
HMCX_WIDE_PROF=$R/gpurun_out/wide_prof5.bin timeout -k 10 120 python tools/probe_sgld.py 64 > gpurun_out/wide_probe5.txt 2>&1 || { tail gpurun_out/wide_probe5.txt; exit 1; }
python3 tools/wide_prof_summary.py gpurun_out/wide_prof5.bin
for rep in 1; do
  echo "old $(HMCX_LIB=libhmcx_w1.so timeout -k 10 120 python tools/probe_sgld.py 400 2>&1 | grep -v amdgpu.ids)"
  echo "new $(timeout -k 10 120 python tools/probe_sgld.py 400 2>&1 | grep -v amdgpu.ids)"
done
echo "f32 new $(timeout -k 10 120 python tools/probe_sgld.py f32 400 2>&1 | grep -v amdgpu.ids)"
echo "C=8 new $(timeout -k 10 120 python tools/probe_sgld.py 400 8 2>&1 | grep -v amdgpu.ids)"
