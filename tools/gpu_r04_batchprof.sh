#!/bin/bash
# Chain-batched path at 2048 chains: per-dispatch kernel trace (launch sizes over the compaction schedule)
# and the SQ-counter pass (MFMA busy, wave states, LDS) -> profiles/pmc_r04_batched_sq.json.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/bkt -o run -- python3 $R/tools/probe_batch.py 2048 > $R/gpurun_out/bkt.log 2>&1 || { tail -5 $R/gpurun_out/bkt.log; exit 1; }
grep "C=" $R/gpurun_out/bkt.log
KT=$(find $R/gpurun_out/bkt -name "*kernel_trace.csv" | head -1)
python3 $R/tools/batch_launch_profile.py $KT > $R/gpurun_out/batch_launch_profile.txt && tail -12 $R/gpurun_out/batch_launch_profile.txt
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $R/gpurun_out/pmcb -o run --output-format csv -- python3 $R/tools/probe_batch.py 2048 > $R/gpurun_out/pmcb.log 2>&1 || { tail -5 $R/gpurun_out/pmcb.log; exit 1; }
cd $R && python3 tools/pmc_batch_summary.py gpurun_out/pmcb "python3 tools/probe_batch.py 2048" gpurun_out/pmc_r04_batched_sq.json
