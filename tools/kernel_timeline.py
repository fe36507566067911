"""Per-dispatch timeline from a rocprofv3 --kernel-trace CSV: for dispatches [first, first + n) of the
kernels whose name contains `match`, print duration and the gap since the previous dispatch's end (µs),
then per kernel name the median duration and median preceding gap over the whole trace.
Usage: python tools/kernel_timeline.py <run_kernel_trace.csv> [match] [first] [n]"""
import csv
import sys
from collections import defaultdict

import numpy as np

path = sys.argv[1]
match = sys.argv[2] if len(sys.argv) > 2 else "hmcx"
first = int(sys.argv[3]) if len(sys.argv) > 3 else 200
n = int(sys.argv[4]) if len(sys.argv) > 4 else 40
rows = [r for r in csv.DictReader(open(path)) if match in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = np.array([int(r["Start_Timestamp"]) for r in rows], dtype=np.float64)
en = np.array([int(r["End_Timestamp"]) for r in rows], dtype=np.float64)
names = [r["Kernel_Name"].split("(")[0].replace("void ", "")[:60] for r in rows]
gap = np.concatenate([[0.0], st[1:] - en[:-1]]) / 1e3
dur = (en - st) / 1e3
for i in range(first, min(first + n, len(rows))):
    print("%5d  %-60s  %8.2f  gap %6.2f" % (i, names[i], dur[i], gap[i]))
agg = defaultdict(list)
for i in range(1, len(rows)):
    agg[names[i]].append((dur[i], gap[i]))
print("\nper kernel: calls, median duration, median gap before it (µs)")
for k, v in sorted(agg.items(), key=lambda kv: -sum(d for d, _ in kv[1])):
    v = np.array(v)
    print("  %-60s %5d  %7.2f  %6.2f" % (k, len(v), np.median(v[:, 0]), np.median(v[:, 1])))
