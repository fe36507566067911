#!/bin/bash
# Round-5 closing set on the final build (the single-chain kernel changed after gpu_r05_close2.sh):
# the whole GPU suite, smoke(), the default bench line, the driver's shape three times, the rocprofv3
# kernel-trace summary of the default command and the PMC fabric traffic of the headline kernel.
set -o pipefail
R=$(cd "$GRAFT_REPO_ROOT" 2>/dev/null && pwd || echo /root/repo)
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r05c.log 2>&1 || { echo pytest failed; grep -E "FAIL|Error|error" gpurun_out/pytest_r05c.log | tail -20; exit 1; }
tail -1 gpurun_out/pytest_r05c.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r05c.log 2>&1 || { tail gpurun_out/smoke_r05c.log; exit 1; }
tail -1 gpurun_out/smoke_r05c.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default_r05c.json 2> gpurun_out/bench_default_r05c.err || { echo bench failed; tail gpurun_out/bench_default_r05c.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default_r05c.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['chain_batched']['sweep'], d['mlp']['roofline']['frac'], d['plantvillage_sgld']['us_per_step'], d['recoveries'])"
for rep in 1 2 3; do
  HMCX_BENCH_DEBUG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20_r05c_$rep.json 2> gpurun_out/bench_s20_r05c_$rep.err || { echo bench s20 failed; tail gpurun_out/bench_s20_r05c_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_s20_r05c_$rep.json')); print('s20', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r05c -o run --output-format csv -- python3 $R/bench.py > $R/gpurun_out/bench_prof_r05c.json 2> $R/gpurun_out/prof_r05c.err || { tail -5 $R/gpurun_out/prof_r05c.err; exit 1; }
echo prof done
cd $R && TAG=r05c bash tools/gpu_pmc_headline.sh && echo pmc done
