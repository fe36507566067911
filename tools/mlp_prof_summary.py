"""Summarise HMCX_MLP_PROF stamps (hmcx_mlp.hip MM_L23): per phase, the median over launches of
the median / max over workgroups of (stamp − the workgroup's first stamp), in µs (s_memrealtime,
100 MHz).  Usage: python tools/mlp_prof_summary.py <file>"""
import sys

import numpy as np

NAMES = ["start", "gemm+epilogue", "publish", "pending", "poll", "ce", "backward", "prefetch issued",
         "first mfma (loads in)", "mfma done", "reduce barrier"]
buf = open(sys.argv[1], "rb").read()
off = 0
rows = []
while off < len(buf):
    n, nlb, ns, nph = np.frombuffer(buf, dtype=np.int32, count=4, offset=off)
    off += 16
    cnt = int(n) * int(nlb) * int(ns) * int(nph)
    a = np.frombuffer(buf, dtype=np.uint64, count=cnt, offset=off).reshape(n, nlb * ns, nph).astype(np.float64)
    off += 8 * cnt
    rows.append(a)
a = np.concatenate(rows)[:, :, :len(NAMES)]
ORDER = [7, 8, 9, 10, 1, 2, 3, 4, 5, 6]
rel = (a - a[:, :, :1]) / 100.0                       # µs
start_skew = (a[:, :, 0] - a[:, :, 0].min(axis=1, keepdims=True)) / 100.0
print("launches %d, workgroups %d" % a.shape[:2])
print("dispatch skew of workgroup starts: median %.2f, max %.2f us" % (np.median(np.median(start_skew, 1)),
                                                                      np.median(start_skew.max(1))))
for i in ORDER:
    nm = NAMES[i]
    print("%-15s median %.2f us   max-over-WG %.2f us" % (nm, np.median(np.median(rel[:, :, i], 1)),
                                                         np.median(rel[:, :, i].max(1))))
end = (a[:, :, 6].max(1) - a[:, :, 0].min(1)) / 100.0
print("first start -> last end: median %.2f us" % np.median(end))
