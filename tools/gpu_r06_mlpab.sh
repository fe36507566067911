# Round 6: config-3 MLP probe, the current build against HMCX_LIB=libhmcx_base.so, alternating (no tests).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2 3 4; do
  for L in libhmcx_base.so libhmcx.so; do
    echo "== $L $(HMCX_LIB=$L timeout -k 10 120 python tools/probe_mlp.py 40 lam=2e-2 reps=3 2>&1 | grep MLP | tail -1)" || exit 1
  done
done
