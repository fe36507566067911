#!/bin/bash
# f64 / f32 16x16x4 MFMA cycles per instruction with 1-8 independent accumulator chains (one wave per SIMD).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 60 ./tools/microbench_mfma
