#!/bin/bash
# Config-5 SGLD with diff stored class-group-major (libhmcx.so) vs [B][KP] rows (libhmcx_base.so):
# the SGLD GPU tests on the new build, then probe_sgld alternating (3 pairs); then the chain-batched
# switch-point sweep (tools/gpu_r05_w.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_chains.py tests/test_gpu_edges.py tests/test_gpu_multicore.py tests/test_gpu_recovery.py tests/test_gpu_statistics.py -m gpu -k "sgld or wide" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_x.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_x.log | tail -30; exit 1; }
echo "tests: $(tail -1 gpurun_out/pytest_x.log)"
for rep in 1 2 3; do for lib in libhmcx_base.so libhmcx.so; do
  echo "[$lib] $(HMCX_LIB=$lib timeout -k 10 120 python tools/probe_sgld.py 400 2>&1 | grep -o 'kern.*us/step [0-9.]*')" || exit 1
done; done
bash tools/gpu_r05_w.sh
