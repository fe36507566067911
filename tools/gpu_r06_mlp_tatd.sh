#!/bin/bash
# Config-3 MLP (tools/probe_mlp.py 12 lam=2e-2): L2 read requests per CU and their latency, per launch,
# with k_fwdr (HMCX_MLP_FWDR=1, the round-6 path) and with the k_mm fused forwards (=0, round 5's),
# one counter group per pass.  Output: per kernel and mode, mean per dispatch.
set -o pipefail
R=$(cd "$GRAFT_REPO_ROOT" 2>/dev/null && pwd || echo /root/repo)
O=$R/gpurun_out/r06_tatd
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for f in 1 0; do
  i=0
  for pmc in "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum" \
             "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
    i=$((i+1))
    HMCX_MLP_FWDR=$f timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pmc -d $O/f${f}_$i -o run --output-format csv -- python3 $R/tools/probe_mlp.py 12 lam=2e-2 > $O/f${f}_$i.log 2>&1 || { tail -5 $O/f${f}_$i.log; exit 1; }
  done
done
cd $R && python3 - "$O" <<'PY'
import csv, glob, collections, sys
O = sys.argv[1]
for f in ("1", "0"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
    for i in (1, 2):
        path = glob.glob("%s/f%s_%d/**/*counter_collection.csv" % (O, f, i), recursive=True)[0]
        seen = collections.defaultdict(set)
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hmcx::", "")[:48]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); seen[k].add(r["Dispatch_Id"])
        for k, v in seen.items(): acc[k]["_n%d" % i] = len(v)
    print("HMCX_MLP_FWDR=%s (per dispatch; L2 requests per CU = TCP_TCC_READ_REQ / 256)" % f)
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1].get("TCP_TCC_READ_REQ_sum", 0)):
        n1, n2 = v.get("_n1", 1), v.get("_n2", 1)
        req = v.get("TCP_TCC_READ_REQ_sum", 0) / n1
        lat = v.get("TCP_TCC_READ_REQ_LATENCY_sum", 0) / max(1.0, v.get("TCP_TCC_READ_REQ_sum", 1))
        print("  %-48s n %4d  L2 req/CU %8.0f  cycles/req %6.0f  pending-stall/CU %8.0f  TA busy/CU %8.0f" % (
            k, n1, req / 256, lat, v.get("TCP_PENDING_STALL_CYCLES_sum", 0) / n1 / 256,
            v.get("TA_TA_BUSY_sum", 0) / n2 / 256))
PY
