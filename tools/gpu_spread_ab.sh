set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for m in 2 0 3 6 10; do
  HMCX_P2_SPREAD=$m timeout -k 10 60 python tools/probe_sghmc.py > gpurun_out/ab.log 2>&1 || { tail gpurun_out/ab.log; exit 1; }
  echo "[spread=$m] $(tail -1 gpurun_out/ab.log | grep -o 'us/lf [0-9.]*')"
done; done
