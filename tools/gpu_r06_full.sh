# Round 6 checkpoint: the whole GPU suite, then the default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_full
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'frac', d['roofline']['frac'])
print('mlp', d['mlp']['leapfrogs_per_s'], d['mlp']['roofline']['frac'], 'mean_L', d['mlp'].get('mean_L'))
print('sgld', d.get('plantvillage_sgld', {}).get('us_per_step'))
print('batched', {k: v.get('frac') for k, v in d.get('chain_batched', {}).get('sweep', {}).items()})
"
