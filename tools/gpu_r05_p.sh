#!/bin/bash
# MLP: W1 gradient from the transposed ga1 and minibatch (16-byte k loads on both operands; libhmcx.so)
# vs the committed build (libhmcx_base.so), after the MLP parity tests on the new build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mlp.py tests/test_gpu_statistics.py > gpurun_out/pytest_r05p.log 2>&1 || { tail -30 gpurun_out/pytest_r05p.log; exit 1; }
tail -1 gpurun_out/pytest_r05p.log
for rep in 1 2 3; do for lib in libhmcx_base.so libhmcx.so; do
  HMCX_LIB=$lib timeout -k 10 200 python -u tools/probe_mlp.py > gpurun_out/pm_$lib.txt 2>&1 || { tail gpurun_out/pm_$lib.txt; exit 1; }
  echo "$lib: $(grep -v amdgpu.ids gpurun_out/pm_$lib.txt | tail -1)"
done; done
for lib in libhmcx_base.so libhmcx.so; do
  HMCX_LIB=$lib timeout -k 10 200 python -u tools/probe_mlp.py f64 > gpurun_out/pm64_$lib.txt 2>&1 || { tail gpurun_out/pm64_$lib.txt; exit 1; }
  echo "$lib f64: $(grep -v amdgpu.ids gpurun_out/pm64_$lib.txt | tail -1)"
done
