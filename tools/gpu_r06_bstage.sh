# Round 6: branch-free staging loads in the chain-batched kernels (selects deferred to the stash) — the
# chain-batched tests, then probe_batch.py 2048 / 8192 against the previous build (HMCX_LIB=libhmcx_base.so),
# alternating, and a kernel-stats trace of the 2048-chain probe.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06_bstage}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_chains.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do
  for L in libhmcx_base.so libhmcx.so; do
    echo "== $L $(HMCX_LIB=$L timeout -k 10 180 python tools/probe_batch.py 2048 8192 2>&1 | grep 'C=' | tr '\n' ' ')" || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python tools/probe_batch.py 2048 > $O/trace.log 2>&1 || exit 1
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
grep -E "k_bgradw|k_bfwd|k_bgrad" $f | cut -d, -f1-4
