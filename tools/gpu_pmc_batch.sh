#!/bin/bash
# SQ counters (wave state breakdown, MFMA busy, LDS) of the chain-batched probe, per kernel.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $R/gpurun_out/pmcb -o run --output-format csv -- python3 $R/tools/probe_batch.py ${CS:-1024} > $R/gpurun_out/pmcb.log 2>&1 || { tail -5 $R/gpurun_out/pmcb.log; exit 1; }
grep "C=" $R/gpurun_out/pmcb.log
ls $R/gpurun_out/pmcb
