#!/bin/bash
# Merged step-start round (HMCX_P2_MERGE=1, libhmcx.so) vs the two-round form (libhmcx_base.so):
# persistent-path parity on the merged build, then the driver-shape headline alternating.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
A=libhmcx_base.so B=libhmcx.so N=3 TESTS="tests/test_gpu_samplers.py tests/test_gpu_recovery.py tests/test_gpu_nan.py tests/test_gpu_statistics.py tests/test_gpu_multicore.py" bash tools/gpu_lib_ab.sh
