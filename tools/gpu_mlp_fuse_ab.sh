#!/bin/bash
# Fused layer 2 + layer 3 (HMCX_MLP_FUSE=1, default) vs separate launches (=0): MLP parity tests with
# each, then the config-3 probe, 3 alternating pairs.
set -o pipefail
mkdir -p gpurun_out
for f in 1 0; do
  HMCX_MLP_FUSE=$f timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_hmc.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_fuse$f.log 2>&1 || { echo "pytest FUSE=$f failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_fuse$f.log | tail -20; exit 1; }
  echo "FUSE=$f $(tail -1 gpurun_out/pytest_fuse$f.log)"
done
for rep in 1 2 3; do for f in 1 0; do
  HMCX_MLP_FUSE=$f timeout -k 10 120 python tools/probe_mlp.py 40 > gpurun_out/fab.log 2>&1 || { tail gpurun_out/fab.log; exit 1; }
  echo "[FUSE=$f] $(tail -1 gpurun_out/fab.log)"
done; done
