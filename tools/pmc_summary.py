"""Summarise the two rocprofv3 PMC passes of tools/gpu_pmc_headline.sh into profiles/pmc_<tag>_<dtype>_<path>.json
(read by bench.py's roofline 'traffic').

    python tools/pmc_summary.py gpurun_out/pmcf gpurun_out/pmcw "k_sghmc_p2<double, 10>" gpurun_out/bench_pmcf.json \
        profiles/pmc_r02_f64_persistent.json

HBM/fabric bytes per launch = 2·FETCH_SIZE + WRITE_SIZE (kB units; MI355X_MICROARCH.md HBM section:
FETCH_SIZE counts half the bytes of 16-byte-per-lane reads, WRITE_SIZE is exact for 16-byte stores;
both include Infinity-Cache hits).  The bench JSON of the profiled run says how many timed calls it
made (roofline.calls) and how many leapfrogs they ran: the timed launches are the `calls` dispatches
after the warm-up ones (bench.py runs warm-up, timed, then the untimed diagnostics calls), and their
bytes ÷ their leapfrogs is the per-leapfrog figure bench.py scales.
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import warmup_calls  # noqa: E402  (bench.py's warm-up protocol, the single definition)


def per_launch(d, counter, kname):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit("no counter_collection.csv under %s" % d)
    out = {}
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] != counter or kname not in r["Kernel_Name"]:
            continue
        key = int(r["Dispatch_Id"])
        out[key] = out.get(key, 0.0) + float(r["Counter_Value"])
    return [out[k] for k in sorted(out)]


def main():
    fdir, wdir, kname, bench_json, dst = sys.argv[1:6]
    fetch = per_launch(fdir, "FETCH_SIZE", kname)
    write = per_launch(wdir, "WRITE_SIZE", kname)
    with open(bench_json) as fh:
        b = json.loads(fh.read().strip().splitlines()[-1])
    calls = int(b["roofline"]["calls"])
    lf = float(b["leapfrogs"])
    steps = int(b["steps"])
    chunk = 120                                         # bench.py: one call per epoch of 60000 / 500 rows
    w0 = len(warmup_calls(int(b["warmup"]), chunk))    # warm-up dispatches before the timed ones
    fm = sum(fetch[w0:w0 + calls]) / calls
    wm = sum(write[w0:w0 + calls]) / calls
    per_launch_bytes = (2.0 * fm + wm) * 1024.0
    lf_per_launch = lf / calls
    alg = 500 * 784 * 8 * steps / calls
    doc = {
        "kernel": kname,
        "config": "python bench.py --steps %d --warmup %d (f64, B=500, D=784, K=10): %d timed launch(es), "
                  "%.0f leapfrogs" % (steps, b["warmup"], calls, lf),
        "collection": "rocprofv3 --kernel-trace --pmc FETCH_SIZE, then a separate pass with --pmc WRITE_SIZE "
                      "(tools/gpu_pmc_headline.sh); summarised by tools/pmc_summary.py",
        "fetch_size_kb_per_launch": fetch,
        "write_size_kb_per_launch": write,
        "timed_launches": calls,
        "fetch_size_kb_timed_mean": fm,
        "write_size_kb_timed_mean": wm,
        "correction": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section); both count Infinity-Cache "
                      "(MALL) hits, so this is fabric traffic, not HBM-only",
        "traffic_bytes_per_launch": per_launch_bytes,
        "leapfrogs_per_launch": lf_per_launch,
        "traffic_bytes_per_leapfrog": per_launch_bytes / lf_per_launch,
        "algorithmic_hbm_bytes_per_launch": alg,
        "traffic_over_algorithmic": per_launch_bytes / alg,
        "note": "the minibatch tiles (3.1 MB per step) are the only algorithmic HBM reads; the rest is the tagged-"
                "granule exchange (write-through stores of partial sums, diff rows, weight slices) and its polling",
    }
    with open(dst, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps({k: doc[k] for k in ("traffic_bytes_per_launch", "traffic_bytes_per_leapfrog",
                                          "traffic_over_algorithmic")}))


if __name__ == "__main__":
    main()
