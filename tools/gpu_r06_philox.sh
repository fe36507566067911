# Round 6: Philox-4x32-10 with one 64-bit product per multiplier (v_mad_u64_u32) — GPU tests on the new
# build, then alternating probes of the previous build (HMCX_LIB=libhmcx_base.so) and the new one.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_philox
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for L in libhmcx_base.so libhmcx.so; do
    echo "== $L"
    HMCX_LIB=$L timeout -k 10 120 python tools/probe_mlp.py 40 lam=2e-2 reps=3 2>&1 | grep MLP | tail -1 || exit 1
    HMCX_LIB=$L timeout -k 10 120 python tools/probe_sgld.py 400 2>&1 | tail -1 || exit 1
    HMCX_LIB=$L timeout -k 10 120 python tools/probe_sghmc.py 2>&1 | tail -1 || exit 1
    HMCX_LIB=$L timeout -k 10 180 python tools/probe_batch.py 2048 2>&1 | tail -1 || exit 1
  done
done
