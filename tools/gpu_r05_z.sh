#!/bin/bash
# L2 hit rate of the MLP config-3 launches (f32), one PMC pass: which share of each GEMM's L2 requests
# the XCD's L2 already holds.
set -o pipefail
R=$(cd "$GRAFT_REPO_ROOT" 2>/dev/null && pwd || echo /root/repo)
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $R/gpurun_out/l2z -o run --output-format csv -- python3 $R/tools/probe_mlp.py 10 > $R/gpurun_out/l2z.log 2>&1 || { tail -5 $R/gpurun_out/l2z.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/l2z/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hmcx::", "")[:70]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "TCC_HIT_sum": n[k] += 1
for k, v in sorted(acc.items(), key=lambda kv: -(kv[1]["TCC_HIT_sum"] + kv[1]["TCC_MISS_sum"])):
    h, m = v["TCC_HIT_sum"], v["TCC_MISS_sum"]
    if h + m == 0: continue
    print("%-70s dispatches %4d  L2 req/dispatch %9.0f  hit %.1f%%  EA rdreq/dispatch %.0f" % (k, n[k], (h + m) / n[k], 100 * h / (h + m), v["TCC_EA0_RDREQ_sum"] / n[k]))
PY
