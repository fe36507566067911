#!/bin/bash
# Round-5 re-check on the final build: the whole GPU suite, smoke(), the default bench line and the
# driver's shape (twice).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r05z.log 2>&1 || { echo pytest failed; grep -E "FAIL|Error|error" gpurun_out/pytest_r05z.log | tail -20; exit 1; }
tail -1 gpurun_out/pytest_r05z.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r05z.log 2>&1 || { tail gpurun_out/smoke_r05z.log; exit 1; }
tail -1 gpurun_out/smoke_r05z.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default_r05z.json 2> gpurun_out/bench_default_r05z.err || { echo bench failed; tail gpurun_out/bench_default_r05z.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default_r05z.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['roofline']['traffic_source'][:60], d['chain_batched']['sweep'], d['mlp']['roofline']['frac'], d['plantvillage_sgld']['us_per_step'], d['recoveries'])"
for rep in 1 2; do
  HMCX_BENCH_DEBUG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20_r05z_$rep.json 2> gpurun_out/bench_s20_r05z_$rep.err || { echo bench s20 failed; tail gpurun_out/bench_s20_r05z_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_s20_r05z_$rep.json')); print('s20', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
done
