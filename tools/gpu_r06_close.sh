#!/bin/bash
# Round-6 closing set on the current build: the whole GPU suite, smoke(), the default bench line, the
# driver's shape three times, the rocprofv3 kernel-trace summary of the default command, the PMC fabric
# traffic of the headline kernel, the chain-batched SQ counters and the MLP TA / TCP counters.
set -o pipefail
R=$(cd "$GRAFT_REPO_ROOT" 2>/dev/null && pwd || echo /root/repo)
T=${TAG:-r06}
O=$R/gpurun_out/close_$T
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; grep -E "FAIL|Error|error" $O/pytest.log | tail -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; tail $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: v['frac'] for k, v in d['chain_batched']['sweep'].items()}, d['mlp']['roofline']['frac'], d['mlp']['leapfrogs_per_s'], d['plantvillage_sgld']['us_per_step'], d['recoveries'])"
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_s20_$rep.json 2> $O/bench_s20_$rep.err || { echo bench s20 failed; tail $O/bench_s20_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_s20_$rep.json')); print('s20', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py > $O/bench_prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
echo prof done
cd $R && TAG=$T bash tools/gpu_pmc_headline.sh && echo pmc done
cd $R && CS=2048 bash tools/gpu_pmc_batch.sh && python3 tools/pmc_batch_summary.py gpurun_out/pmcb "python3 tools/probe_batch.py 2048" $O/pmc_batched_sq.json > $O/pmc_batched_sq.txt 2>&1; echo batched pmc rc $?
cd $R && bash tools/gpu_r06_mlp_tatd.sh > $O/mlp_tatd.txt 2>&1; echo tatd rc $?
