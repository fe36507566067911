set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_mlp0
mkdir -p $O
for lam in 5e-3 2e-2 3e-2; do timeout -k 10 120 python tools/probe_mlp.py 40 lam=$lam reps=3 >> $O/probe.txt 2>&1 || exit 1; done
timeout -k 10 120 python tools/probe_mlp.py 40 lam=2e-2 reps=3 >> $O/probe.txt 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python tools/probe_mlp.py 12 lam=2e-2 > $O/trace.log 2>&1 || exit 1
f=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python tools/kernel_timeline.py $f hmcx 150 60 > $O/timeline.txt 2>&1
cat $O/probe.txt
