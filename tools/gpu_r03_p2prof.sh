#!/bin/bash
# Headline kernel: in-kernel segment profile (HMCX_PERSIST_PROF) and round trace (HMCX_P2_TRACE).
set -o pipefail
mkdir -p gpurun_out
HMCX_PERSIST_PROF=1 timeout -k 10 120 python tools/probe_sghmc.py > gpurun_out/p2prof.txt 2>&1 || { tail gpurun_out/p2prof.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/p2prof.txt | tail -4
HMCX_P2_TRACE=1 HMCX_P2_SPEC=0 timeout -k 10 120 python tools/probe_sghmc.py > gpurun_out/p2trace.txt 2>&1 || { tail gpurun_out/p2trace.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/p2trace.txt | tail -8
