#!/bin/bash
# In-kernel segment profile (HMCX_PERSIST_PROF) and round-latency trace (HMCX_P2_TRACE) of the
# persistent kernel at the default grid.
set -o pipefail
mkdir -p gpurun_out
HMCX_PERSIST_PROF=1 timeout -k 10 60 python tools/probe_sghmc.py > gpurun_out/p2prof.log 2>&1 || { tail gpurun_out/p2prof.log; exit 1; }
grep "p2 prof" gpurun_out/p2prof.log | tail -1; tail -1 gpurun_out/p2prof.log
HMCX_P2_TRACE=1 timeout -k 10 60 python tools/probe_sghmc.py > gpurun_out/p2trace.log 2>&1 || { tail gpurun_out/p2trace.log; exit 1; }
grep "trace\]" gpurun_out/p2trace.log | tail -5
