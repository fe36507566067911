#!/bin/bash
# Headline kernel LDS pitch change (BFP 66 → 65, B-gemm k values Br/4 rows apart per lane group):
# bank-conflict counters of both builds, then the persistent-path parity tests and the driver-shape A/B.
set -o pipefail
R=$(cd "$GRAFT_REPO_ROOT" 2>/dev/null && pwd || echo /root/repo)
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for lib in libhmcx_base.so libhmcx.so; do
  HMCX_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES -d $R/gpurun_out/ldsv_$lib -o run --output-format csv -- python3 $R/tools/probe_sghmc.py > $R/gpurun_out/ldsv_$lib.log 2>&1 || { tail -5 $R/gpurun_out/ldsv_$lib.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
for lib in ("libhmcx_base.so", "libhmcx.so"):
    f = glob.glob("gpurun_out/ldsv_%s/**/*counter_collection.csv" % lib, recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hmcx::", "")[:70]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]["SQ_LDS_BANK_CONFLICT"])[:3]:
        if v["SQ_INSTS_LDS"] == 0: continue
        print(lib, "%-50s insts %.3g conf %.3g active %.3g wave_cycles %.3g" % (k, v["SQ_INSTS_LDS"], v["SQ_LDS_BANK_CONFLICT"], v["SQ_LDS_IDX_ACTIVE"], v["SQ_WAVE_CYCLES"]))
PY
A=libhmcx_base.so B=libhmcx.so N=3 TESTS="tests/test_gpu_samplers.py tests/test_gpu_recovery.py tests/test_gpu_nan.py tests/test_gpu_statistics.py tests/test_gpu_multicore.py" bash tools/gpu_lib_ab.sh
