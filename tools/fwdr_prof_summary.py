"""Summarise HMCX_FWDR_PROF stamps (hmcx_mlp.hip k_fwdr): per phase, the median over launches of the
median / max over workgroups of (stamp − the launch's first workgroup start), in µs (s_memrealtime,
100 MHz).  Usage: python tools/fwdr_prof_summary.py <file>"""
import sys

import numpy as np

NAMES = ["start", "operands issued", "h1 in LDS", "layer-2 GEMM done", "epilogue (d3)", "layer-3 partials",
         "cross-entropy", "backward done"]
buf = open(sys.argv[1], "rb").read()
off, launches = 0, []
while off < len(buf):
    npb, nrb, nph = np.frombuffer(buf, dtype=np.int32, count=3, offset=off)
    off += 12
    cnt = int(npb) * int(nrb) * int(nph)
    a = np.frombuffer(buf, dtype=np.uint64, count=cnt, offset=off).reshape(npb * nrb, nph).astype(np.float64)
    off += 8 * cnt
    launches.append(a)
print("launches %d, workgroups per launch %s" % (len(launches), sorted({a.shape[0] for a in launches})))
for i, nm in enumerate(NAMES):
    med = np.median([np.median((a[:, i] - a[:, 0].min()) / 100.0) for a in launches])
    mx = np.median([np.max((a[:, i] - a[:, 0].min()) / 100.0) for a in launches])
    print("%-20s median %6.2f us   max-over-WG %6.2f us" % (nm, med, mx))
