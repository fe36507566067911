#!/bin/bash
# Config-5 SGLD (tools/probe_sgld.py 400): fabric bytes (FETCH_SIZE, WRITE_SIZE) and L2 hit/miss of the
# fused forward and the gradient kernel, in separate counter passes.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/spf -o run --output-format csv -- python3 $R/tools/probe_sgld.py 400 > $R/gpurun_out/spf.log 2>&1 || { tail -5 $R/gpurun_out/spf.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/spw -o run --output-format csv -- python3 $R/tools/probe_sgld.py 400 > $R/gpurun_out/spw.log 2>&1 || { tail -5 $R/gpurun_out/spw.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/sph -o run --output-format csv -- python3 $R/tools/probe_sgld.py 400 > $R/gpurun_out/sph.log 2>&1 || { tail -5 $R/gpurun_out/sph.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob, collections
for d in ("spf", "spw", "sph"):
    f = glob.glob("gpurun_out/%s/**/*counter_collection.csv" % d, recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hmcx::", "")
        if "k_w" not in k: continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    for k, v in acc.items():
        print(d, k, len(n[k]), {c: round(x / len(n[k]), 1) for c, x in v.items()})
PY
