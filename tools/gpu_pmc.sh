#!/bin/bash
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
grep -i -E "ICACHE|SQ_INSTS_VALU\b|SQ_WAIT_INST_ANY|SQ_INSTS_SALU|SQ_IFETCH|SQ_WAVE_CYCLES|SQ_BUSY_CYCLES|SQ_INST_CYCLES" $R/gpurun_out/counters.txt | head -40
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES SQ_INSTS_VALU -d $R/gpurun_out/pmc1 -o run --output-format csv -- python3 $R/tools/probe_sghmc.py > $R/gpurun_out/pmc1.log 2>&1 || { tail -5 $R/gpurun_out/pmc1.log; exit 1; }
find $R/gpurun_out/pmc1 -name "*counter_collection*" | head
