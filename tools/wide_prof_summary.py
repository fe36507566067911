"""Summarise HMCX_WIDE_PROF stamps (hmcx_wide.hip): per kernel and phase, the median over steps of the
median / max over workgroups of (stamp − the kernel's earliest start), in µs (s_memrealtime, 100 MHz);
and the gaps between one kernel's last stamp and the next kernel's first start.
Usage: python tools/wide_prof_summary.py <file> [fused] [team]
  fused: the forward is k_wfwd_sm (forward + softmax, no k_wsoft launch); team: the gradient is
  k_wgrad_team (row-slice teams) — pass what HMCX_WIDE_FUSE / HMCX_WIDE_GTEAM selected."""
import sys

import numpy as np

fused = "fused" in sys.argv[2:]
team = "team" in sys.argv[2:]
PH = {"k_wfwd": ["start", "loads in", "mfma done", "partials in LDS", "barrier", "slab stored", "end"],
      "k_wsoft": ["start", "slab summed", "softmax done", "end"],
      "k_wgrad": ["start", "epilogue operands + noise", "gemm done", "reduce barrier", "update done", "end (bias)"]}
if fused:
    PH["k_wfwd"] = ["start", "loads in", "mfma done", "partials published", "partials gathered", "softmax done",
                    "end"]
    del PH["k_wsoft"]
if team:
    PH["k_wgrad"] = ["start", "operands + noise", "gemm done", "partials published", "partials gathered",
                     "update done"]
buf = open(sys.argv[1], "rb").read()
off, steps = 0, []
while off < len(buf):
    n, gf, gs, gg, wph = np.frombuffer(buf, dtype=np.int32, count=5, offset=off)
    off += 20
    cnt = int(n) * int(gf + gs + gg) * int(wph)
    a = np.frombuffer(buf, dtype=np.uint64, count=cnt, offset=off).reshape(n, gf + gs + gg, wph).astype(np.float64)
    off += 8 * cnt
    for st in a[1:]:                          # the first step of a call includes the launch ramp
        k = {"k_wfwd": st[:gf], "k_wsoft": st[gf:gf + gs], "k_wgrad": st[gf + gs:]}
        k["k_wgrad"] = k["k_wgrad"][k["k_wgrad"][:, 0] > 0]      # padding workgroups store nothing
        steps.append(k)
print("steps %d" % len(steps))
for name in PH:
    nph = len(PH[name])
    rel = []
    for st in steps:
        k = st[name][:, :nph]
        t0 = k[:, 0].min()
        rel.append((k - t0) / 100.0)
    rel = np.array(rel)                       # [steps, wg, ph]
    span = np.median(rel[:, :, nph - 1].max(1))
    print("%s: %d workgroups, first start -> last end %.2f us" % (name, rel.shape[1], span))
    for i, nm in enumerate(PH[name]):
        if nm:
            print("   %-28s median %6.2f   max-over-WG %6.2f" % (nm, np.median(np.median(rel[:, :, i], 1)),
                                                                np.median(rel[:, :, i].max(1))))
seq = list(PH)
gaps = []
for st in steps:
    g = []
    for a_, b_ in zip(seq[:-1], seq[1:]):
        g.append((st[b_][:, 0].min() - st[a_][:, len(PH[a_]) - 1].max()) / 100.0)
    gaps.append(g)
gaps = np.median(np.array(gaps), 0)
print("; ".join("gap %s end -> %s start %.2f us" % (a_, b_, g) for a_, b_, g in zip(seq[:-1], seq[1:], gaps)))
tot = [(st[seq[-1]][:, len(PH[seq[-1]]) - 1].max() - st[seq[0]][:, 0].min()) / 100.0 for st in steps]
nxt = [(steps[i + 1][seq[0]][:, 0].min() - steps[i][seq[-1]][:, len(PH[seq[-1]]) - 1].max()) / 100.0
       for i in range(len(steps) - 1)]
print("step (first start -> last end) median %.2f us; gap to the next step's forward %.2f us"
      % (np.median(tot), np.median(nxt) if nxt else float("nan")))
