# Round 6: grouped keep flags (16 per Philox block) — MLP tests, then the config-3 probe against the
# previous build (HMCX_LIB=libhmcx_base.so), alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06_keep}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_statistics.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do
  for L in libhmcx_base.so libhmcx.so; do
    echo "== $L $(HMCX_LIB=$L timeout -k 10 120 python tools/probe_mlp.py 40 lam=2e-2 reps=3 2>&1 | grep MLP | tail -1)" || exit 1
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python tools/probe_mlp.py 12 lam=2e-2 > $O/trace.log 2>&1 || exit 1
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
grep -E "k_mlp_start|k_fwdr|accept|sumsq|k_pending" $f | cut -c1-200
