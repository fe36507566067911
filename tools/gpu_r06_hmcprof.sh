set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_hmcprof
mkdir -p $O
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/t -o run -- python3 $GRAFT_REPO_ROOT/tools/probe_mlp_hmc.py f32 6 device > $GRAFT_REPO_ROOT/$O/probe.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && f=$(find $O/t -name '*kernel_stats.csv' | head -1) && cut -d, -f1-4 $f | cut -c1-140 | head -30
