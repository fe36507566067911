#!/bin/bash
# Per-dispatch kernel trace of the chain-batched path (2048 chains, 24 steps): grid sizes give the
# active chain tiles of each launch, so each GEMM kernel's rate can be read per dispatch.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/btrace -o run --output-format csv -- python3 $R/tools/probe_batch.py 2048 > $R/gpurun_out/btrace.log 2>&1 || { tail -5 $R/gpurun_out/btrace.log; exit 1; }
tail -2 $R/gpurun_out/btrace.log
