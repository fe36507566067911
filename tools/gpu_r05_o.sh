#!/bin/bash
# Config-5 SGLD (tools/probe_mlp.py 10): TA / TD / TCP / UTCL1 counters of the fused forward and the
# gradient, one counter group per pass (per-block limits: 2 TA, 2 TD, 4 TCP, 2 GRBM).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pmc -d $R/gpurun_out/mtatd$i -o run --output-format csv -- python3 $R/tools/probe_mlp.py 10 > $R/gpurun_out/mtatd$i.log 2>&1 || { tail -5 $R/gpurun_out/mtatd$i.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
dur = collections.defaultdict(list)
for i in range(1, 6):
    f = glob.glob("gpurun_out/mtatd%d/**/*counter_collection.csv" % i, recursive=True)[0]
    seen = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hmcx::", "")
        if "k_mm" not in k: continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); seen[k].add(r["Dispatch_Id"])
    for k, v in seen.items(): acc[k]["_disp%d" % i] = len(v)
for k, v in acc.items():
    out = {}
    for c, x in v.items():
        if c.startswith("_"): continue
        p = [i for i in range(1, 6) if ("_disp%d" % i) in v]
        d = next(v["_disp%d" % i] for i in p)
        out[c] = round(x / d, 1)
    print(k, out)
PY
