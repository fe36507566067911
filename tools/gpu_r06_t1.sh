# Round 6: MLP + SGLD + recovery tests after the async SGLD verdict; MLP / SGLD probes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_t1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_samplers.py tests/test_gpu_recovery.py tests/test_capi.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 120 python tools/probe_mlp.py 40 lam=2e-2 reps=3 > $O/probe_mlp.txt 2>&1 || exit 1
timeout -k 10 120 python tools/probe_sgld.py 400 > $O/probe_sgld.txt 2>&1 || exit 1
grep -h "MLP\|step" $O/probe_mlp.txt $O/probe_sgld.txt | tail -5
