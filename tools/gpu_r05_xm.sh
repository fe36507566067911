#!/bin/bash
# MLP plain GEMM launches with XCD-contiguous tile chunks (default) vs dispatch order (HMCX_MLP_XMAP=0):
# MLP GPU tests, the L2 hit rate of both, then probe_mlp alternating (f32 4 pairs, f64 2 pairs).
set -o pipefail
R=$(cd "$GRAFT_REPO_ROOT" 2>/dev/null && pwd || echo /root/repo)
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_xm.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_xm.log | tail -30; exit 1; }
echo "tests: $(tail -1 gpurun_out/pytest_xm.log)"
cd /tmp && export TMPDIR=/tmp
for xm in 0 1; do
  HMCX_MLP_XMAP=$xm timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/l2xm$xm -o run --output-format csv -- python3 $R/tools/probe_mlp.py 10 > $R/gpurun_out/l2xm$xm.log 2>&1 || { tail -5 $R/gpurun_out/l2xm$xm.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
for xm in (0, 1):
    f = glob.glob("gpurun_out/l2xm%d/**/*counter_collection.csv" % xm, recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hmcx::", "")[:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        if k.startswith("k_mm"):
            h, m = v["TCC_HIT_sum"], v["TCC_MISS_sum"]
            print("xmap=%d %-45s hit %.1f%% misses %.3g" % (xm, k, 100 * h / max(1, h + m), m))
PY
for rep in 1 2 3 4; do for xm in 0 1; do
  echo "[xmap=$xm] $(HMCX_MLP_XMAP=$xm timeout -k 10 120 python tools/probe_mlp.py 20 2>&1 | grep -o 'kern.*lf/s [0-9.]*')" || exit 1
done; done
for rep in 1 2; do for xm in 0 1; do
  echo "[f64 xmap=$xm] $(HMCX_MLP_XMAP=$xm timeout -k 10 120 python tools/probe_mlp.py f64 20 2>&1 | grep -o 'kern.*lf/s [0-9.]*')" || exit 1
done; done
