#!/bin/bash
set -o pipefail
bash tools/gpu_r04_wideprof.sh | head -24 || exit 1
for i in 1 2; do
echo "fused $(timeout -k 10 60 python tools/probe_sgld.py 400 2>&1 | tail -1)"
echo "3-launch $(HMCX_WIDE_FUSE=0 timeout -k 10 60 python tools/probe_sgld.py 400 2>&1 | tail -1)"
done
