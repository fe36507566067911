#!/bin/bash
# SQ counters of the 2048-chain batched path on the current build (profiles/pmc_r05_batched_sq.json).
set -o pipefail
R=$(cd "$GRAFT_REPO_ROOT" 2>/dev/null && pwd || echo /root/repo)
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $R/gpurun_out/pmcb_r05b -o run --output-format csv -- python3 $R/tools/probe_batch.py 2048 > $R/gpurun_out/pmcb_r05b.log 2>&1 || { tail -5 $R/gpurun_out/pmcb_r05b.log; exit 1; }
cd $R && python3 tools/pmc_batch_summary.py gpurun_out/pmcb_r05b "python3 tools/probe_batch.py 2048" gpurun_out/pmc_r05_batched_sq.json && echo batched pmc done
