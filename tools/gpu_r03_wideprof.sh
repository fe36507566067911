#!/bin/bash
# Config-5 wide SGLD: in-kernel phase stamps of k_wfwd / k_wsoft / k_wgrad (HMCX_WIDE_PROF), f64.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
rm -f gpurun_out/wide_prof.bin
HMCX_WIDE_PROF=$R/gpurun_out/wide_prof.bin timeout -k 10 120 python tools/probe_sgld.py 64 > gpurun_out/wide_probe.txt 2>&1 || { tail gpurun_out/wide_probe.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/wide_probe.txt
python3 tools/wide_prof_summary.py gpurun_out/wide_prof.bin
timeout -k 10 120 python tools/probe_sgld.py 400 2>&1 | grep -v amdgpu.ids
