# Round 6: rocBLAS DGEMM ceiling at the chain-batched shapes beside k_bgradw's
# per-dispatch durations at 2048 chains (kernel trace of the batched probe).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_dgemm
mkdir -p $O
timeout -k 10 120 python tools/probe_dgemm.py 2048 > $O/dgemm.txt 2>&1 || exit 1
timeout -k 10 120 python tools/probe_dgemm.py 8192 >> $O/dgemm.txt 2>&1 || exit 1
cat $O/dgemm.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python tools/probe_batch.py 2048 > $O/batch.log 2>&1 || exit 1
grep "C=" $O/batch.log
f=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "k_bgradw" in n or "Cijk" in n or "k_bfwd" in n:
        g = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1)) * int(r.get("Grid_Size_Z", 1)) // max(1, int(r["Workgroup_Size_X"]))
        by[(n.split("(")[0][:60], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, g), v in sorted(by.items(), key=lambda kv: (kv[0][0], -kv[0][1]))[:30]:
    v.sort()
    print("%-60s WGs %5d  n %4d  median %8.1f us" % (n, g, len(v), v[len(v) // 2]))
PY
