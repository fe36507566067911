"""Chain-batched call, launch by launch: from a rocprofv3 --kernel-trace CSV of tools/probe_batch.py, group the
dispatches of each kernel by their workgroup count and print count, median duration (µs) and total time (ms),
so the share of time spent in launches that do not fill the chip (the compaction tail) is visible.
Usage: python tools/batch_launch_profile.py <kernel_trace.csv> [num_cus]"""
import csv
import sys
from collections import defaultdict

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "hmcx" in r["Kernel_Name"]]
cus = int(sys.argv[2]) if len(sys.argv) > 2 else 256
g = defaultdict(list)
tot = 0.0
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hmcx::", "")
    wg = int(r.get("Grid_Size", r.get("Grid_Size_X", 0))) // max(1, int(r.get("Workgroup_Size", r.get("Workgroup_Size_X", 1))))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    g[(name, wg)].append(d)
    tot += d
print("total device time %.2f ms over %d dispatches" % (tot / 1e3, len(rows)))
by_k = defaultdict(float)
under = defaultdict(float)
for (name, wg), v in sorted(g.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
    s = sum(v)
    by_k[name] += s
    if wg < 2 * cus:
        under[name] += s
    print("%-40s wg %6d  n %4d  median %8.2f us  total %8.2f ms" % (name[:40], wg, len(v), np.median(v), s / 1e3))
for k in by_k:
    print("%-40s total %8.2f ms, in launches of < 2 workgroups per CU %8.2f ms" % (k[:40], by_k[k] / 1e3, under[k] / 1e3))
