#!/bin/bash
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
rm -f gpurun_out/sgld_prof.txt
HMCX_SGLD_WIDE=2 HMCX_SGLD_PROF=$R/gpurun_out/sgld_prof.txt timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 400 > /dev/null 2>&1 || { echo failed; exit 1; }
cat gpurun_out/sgld_prof.txt | tail -10
