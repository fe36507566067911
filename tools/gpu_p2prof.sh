#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for g in 4x4 8x8; do HMCX_P2_GRID=$g HMCX_PERSIST_PROF=1 timeout -k 10 60 python tools/probe_sghmc.py > gpurun_out/p2prof_$g.log 2>&1 || { tail gpurun_out/p2prof_$g.log; exit 1; }; grep "p2 prof" gpurun_out/p2prof_$g.log | tail -1; tail -1 gpurun_out/p2prof_$g.log; done
