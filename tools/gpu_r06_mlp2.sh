# Round 6: k_fwdr phase stamps (HMCX_FWDR_PROF) at config 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_mlp2
mkdir -p $O
rm -f $O/fwdr.prof
HMCX_FWDR_PROF=$O/fwdr.prof timeout -k 10 120 python tools/probe_mlp.py 12 lam=2e-2 > $O/probe.txt 2>&1 || exit 1
python tools/fwdr_prof_summary.py $O/fwdr.prof | tee $O/summary.txt
