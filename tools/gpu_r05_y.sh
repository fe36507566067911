#!/bin/bash
# k_wgrad's cross-wave reduction in conflict-free slots (libhmcx.so) vs class-ordered columns
# (libhmcx_base.so): SGLD GPU tests on the new build, LDS conflict counters of both, probe_sgld
# alternating (4 pairs).
set -o pipefail
R=$(cd "$GRAFT_REPO_ROOT" 2>/dev/null && pwd || echo /root/repo)
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_chains.py tests/test_gpu_edges.py tests/test_gpu_multicore.py tests/test_gpu_recovery.py tests/test_gpu_statistics.py -m gpu -k "sgld or wide" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_y.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error|assert" gpurun_out/pytest_y.log | tail -30; exit 1; }
echo "tests: $(tail -1 gpurun_out/pytest_y.log)"
cd /tmp && export TMPDIR=/tmp
for lib in libhmcx_base.so libhmcx.so; do
  HMCX_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES -d $R/gpurun_out/ldsy_$lib -o run --output-format csv -- python3 $R/tools/probe_sgld.py 200 > $R/gpurun_out/ldsy_$lib.log 2>&1 || { tail -5 $R/gpurun_out/ldsy_$lib.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
for lib in ("libhmcx_base.so", "libhmcx.so"):
    f = glob.glob("gpurun_out/ldsy_%s/**/*counter_collection.csv" % lib, recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hmcx::", "")[:50]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        if "k_wgrad" in k:
            print(lib, k, "insts %.3g conf %.3g" % (v["SQ_INSTS_LDS"], v["SQ_LDS_BANK_CONFLICT"]))
PY
for rep in 1 2 3 4; do for lib in libhmcx_base.so libhmcx.so; do
  echo "[$lib] $(HMCX_LIB=$lib timeout -k 10 120 python tools/probe_sgld.py 400 2>&1 | grep -o 'kern.*us/step [0-9.]*')" || exit 1
done; done
