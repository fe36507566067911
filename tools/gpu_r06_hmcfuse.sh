# Round 6: full-batch HMC on the MLP with the kicks / drift / masks of two gradient calls in one launch and
# one pending launch per call — the MLP tests (device leapfrog = host loop, bit for bit), then the probe
# against the previous build (HMCX_LIB=libhmcx_base.so), alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06_hmcfuse}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_hmc.py tests/test_gpu_logistic_sgd.py tests/test_gpu_softmax.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for L in libhmcx_base.so libhmcx.so; do
    for d in f32 f64; do
      echo "== $L $(HMCX_LIB=$L timeout -k 10 200 python tools/probe_mlp_hmc.py $d 6 2>&1 | grep device | tail -1)" || exit 1
    done
  done
done
