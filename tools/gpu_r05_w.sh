#!/bin/bash
# Chain-batched tile switch points: HMCX_BTAIL_WG (64-row forward workgroups at or below which the
# forward runs 32-row tiles; default = CUs) and HMCX_BGW_MIN (workgroups from which the gradient runs
# 64-feature tiles; default = 2 x CUs), 2048 and 8192 chains, two alternating passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "256 512" "384 512" "512 512" "768 512" "1024 512" "256 384" "256 768" "256 1024"; do
    set -- $cfg
    echo "tail_wg=$1 bgw_min=$2 $(HMCX_BTAIL_WG=$1 HMCX_BGW_MIN=$2 timeout -k 10 120 python tools/probe_batch.py 2048 8192 2>&1 | grep -o 'C=.*kern [0-9.]* s' | tr '\n' ' ')" || exit 1
  done
done
