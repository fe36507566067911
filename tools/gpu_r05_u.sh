#!/bin/bash
# LDS bank-conflict census of the single-chain, MLP and wide-SGLD paths (one rocprofv3 pass each).
set -o pipefail
R=$(cd "$GRAFT_REPO_ROOT" 2>/dev/null && pwd || echo /root/repo)
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for cmd in "tools/probe_sghmc.py" "tools/probe_mlp.py 10" "tools/probe_mlp.py f64 10" "tools/probe_sgld.py 200"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES -d $R/gpurun_out/ldsc$i -o run --output-format csv -- python3 $R/$cmd > $R/gpurun_out/ldsc$i.log 2>&1 || { tail -5 $R/gpurun_out/ldsc$i.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
for i in range(1, 5):
    f = glob.glob("gpurun_out/ldsc%d/**/*counter_collection.csv" % i, recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hmcx::", "")[:70]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]["SQ_LDS_BANK_CONFLICT"]):
        if v["SQ_INSTS_LDS"] == 0: continue
        print(i, "%-70s insts %.3g conf %.3g (%.2f%% insts, %.2f%% active)" % (k, v["SQ_INSTS_LDS"], v["SQ_LDS_BANK_CONFLICT"],
              100 * v["SQ_LDS_BANK_CONFLICT"] / v["SQ_INSTS_LDS"], 100 * v["SQ_LDS_BANK_CONFLICT"] / max(1, v["SQ_LDS_IDX_ACTIVE"])))
PY
