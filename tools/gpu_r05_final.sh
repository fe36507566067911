#!/bin/bash
# Round-5 closing set on the final build: default bench line and the driver's shape, the rocprofv3
# kernel-trace summary of the default command, the PMC fabric traffic of the headline kernel at the
# driver's shape, and the SQ counters of the 2048-chain batched path (profiles/).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default_r05.json 2> gpurun_out/bench_default_r05.err || { echo bench failed; tail gpurun_out/bench_default_r05.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default_r05.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['chain_batched']['sweep'], d['mlp']['roofline']['frac'], d['plantvillage_sgld']['us_per_step'], d['recoveries'])"
for rep in 1 2 3; do
  HMCX_BENCH_DEBUG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20_r05_$rep.json 2> gpurun_out/bench_s20_r05_$rep.err || { echo bench s20 failed; tail gpurun_out/bench_s20_r05_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_s20_r05_$rep.json')); print('s20', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
  grep "timed region" gpurun_out/bench_s20_r05_$rep.err || true
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05 -o run --output-format csv -- python3 $R/bench.py > $R/gpurun_out/bench_prof_r05.json 2> $R/gpurun_out/prof_r05.err || { tail -5 $R/gpurun_out/prof_r05.err; exit 1; }
echo prof done
cd $R && TAG=r05 bash tools/gpu_pmc_headline.sh
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $R/gpurun_out/pmcb_r05 -o run --output-format csv -- python3 $R/tools/probe_batch.py 2048 > $R/gpurun_out/pmcb_r05.log 2>&1 || { tail -5 $R/gpurun_out/pmcb_r05.log; exit 1; }
cd $R && python3 tools/pmc_batch_summary.py gpurun_out/pmcb_r05 "python3 tools/probe_batch.py 2048" gpurun_out/pmc_r05_batched_sq.json && echo batched pmc done
