"""Summarise HMCX_WIDE_PROF stamps (hmcx_wide.hip): per kernel and phase, the median over steps of the
median / max over workgroups of (stamp − the kernel's earliest start), in µs (s_memrealtime, 100 MHz);
and the gaps between one kernel's last stamp and the next kernel's first start.
Usage: python tools/wide_prof_summary.py <file>"""
import sys

import numpy as np

PH = {"k_wfwd": ["start", "loads issued", "staged (LDS stores)", "barrier", "mfma done", "reduce barrier", "slab stored"],
      "k_wsoft": ["start", "slab summed", "softmax done", "end"],
      "k_wgrad": ["start", "epilogue operands + noise", "gemm done", "reduce barrier", "update done", "end (bias)"]}
buf = open(sys.argv[1], "rb").read()
off, steps = 0, []
while off < len(buf):
    n, gf, gs, gg, wph = np.frombuffer(buf, dtype=np.int32, count=5, offset=off)
    off += 20
    cnt = int(n) * int(gf + gs + gg) * int(wph)
    a = np.frombuffer(buf, dtype=np.uint64, count=cnt, offset=off).reshape(n, gf + gs + gg, wph).astype(np.float64)
    off += 8 * cnt
    for st in a[1:]:                          # the first step of a call includes the launch ramp
        steps.append((st[:gf], st[gf:gf + gs], st[gf + gs:]))
print("steps %d" % len(steps))
prev_end = []
for ki, name in enumerate(PH):
    nph = len(PH[name])
    rel = []
    for st in steps:
        k = st[ki][:, :nph]
        t0 = k[:, 0].min()
        rel.append((k - t0) / 100.0)
    rel = np.array(rel)                       # [steps, wg, ph]
    span = np.median(rel[:, :, nph - 1].max(1))
    print("%s: %d workgroups, first start -> last end %.2f us" % (name, rel.shape[1], span))
    for i, nm in enumerate(PH[name]):
        print("   %-28s median %6.2f   max-over-WG %6.2f" % (nm, np.median(np.median(rel[:, :, i], 1)),
                                                            np.median(rel[:, :, i].max(1))))
gaps = []
for st in steps:
    f, s_, g = st
    gaps.append(((s_[:, 0].min() - f[:, 6].max()) / 100.0, (g[:, 0].min() - s_[:, 3].max()) / 100.0))
gaps = np.array(gaps)
print("gap k_wfwd end -> k_wsoft start %.2f us; k_wsoft end -> k_wgrad start %.2f us" % tuple(np.median(gaps, 0)))
tot = [(st[2][:, 5].max() - st[0][:, 0].min()) / 100.0 for st in steps]
print("step (k_wfwd first start -> k_wgrad last end) median %.2f us" % np.median(tot))
