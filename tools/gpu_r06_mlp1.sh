# Round 6: k_fwdr (all forwards of an MLP iteration in one launch) — MLP tests, then the config-3 probe
# with k_fwdr on and off (same box, alternating).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_mlp1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for r in 1 2; do
  for f in 1 0; do HMCX_MLP_FWDR=$f timeout -k 10 120 python tools/probe_mlp.py 40 lam=2e-2 reps=3 >> $O/probe_fwdr$f.txt 2>&1 || exit 1; done
done
grep -h MLP $O/probe_fwdr1.txt $O/probe_fwdr0.txt
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python tools/probe_mlp.py 12 lam=2e-2 > $O/trace.log 2>&1 || exit 1
f=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python tools/kernel_timeline.py $f hmcx 150 30 > $O/timeline.txt 2>&1
tail -14 $O/timeline.txt
rm -f $O/fwdr.prof
HMCX_FWDR_PROF=$O/fwdr.prof timeout -k 10 120 python tools/probe_mlp.py 12 lam=2e-2 > $O/probe_prof.txt 2>&1 || exit 1
python tools/fwdr_prof_summary.py $O/fwdr.prof | tee $O/stamps.txt
