#!/bin/bash
# Launch fixed-cost probe, then the round-3 PMC traffic passes of the headline kernel.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/probe_launch_fixed.py > gpurun_out/launch_fixed.txt 2>&1 || { tail gpurun_out/launch_fixed.txt; exit 1; }
cat gpurun_out/launch_fixed.txt | grep -v amdgpu.ids
TAG=r03 bash tools/gpu_pmc_headline.sh
