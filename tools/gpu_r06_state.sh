# Round 6 (re-entry): current build — the default bench line, the MLP probe and the Philox microbenchmark.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_state
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: v['frac'] for k, v in d['chain_batched']['sweep'].items()}, d['mlp']['roofline']['frac'], d['mlp']['leapfrogs_per_s'], d['plantvillage_sgld']['us_per_step'], d['recoveries'])"
for r in 1 2; do timeout -k 10 120 python tools/probe_mlp.py 40 lam=2e-2 reps=3 2>&1 | grep MLP | tail -1 || exit 1; done
hipcc -O3 --offload-arch=gfx950 tools/microbench_philox.hip -o $O/mb_philox && timeout -k 10 60 $O/mb_philox | tee $O/mb_philox.txt
