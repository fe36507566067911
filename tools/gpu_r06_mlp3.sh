# Round 6: config-3 probe + k_fwdr stamps (A/B of one k_fwdr change: run after each build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_mlp3
mkdir -p $O
for r in 1 2 3; do timeout -k 10 120 python tools/probe_mlp.py 40 lam=2e-2 reps=3 >> $O/probe.txt 2>&1 || exit 1; done
grep MLP $O/probe.txt | tail -3
rm -f $O/fwdr.prof
HMCX_FWDR_PROF=$O/fwdr.prof timeout -k 10 120 python tools/probe_mlp.py 12 lam=2e-2 > /dev/null 2>&1 || exit 1
python tools/fwdr_prof_summary.py $O/fwdr.prof
