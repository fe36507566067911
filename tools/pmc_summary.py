"""Summarise the two rocprofv3 PMC passes of tools/gpu_pmc_bench.sh into profiles/pmc_<tag>_<dtype>_<path>.json
(read by bench.py's roofline 'traffic').

    python tools/pmc_summary.py gpurun_out/pmcf_r01 gpurun_out/pmcw_r01 "k_sghmc_p2<double, 10>" profiles/pmc_r01_f64_persistent.json

HBM/fabric bytes per launch = 2·FETCH_SIZE + WRITE_SIZE (kB units; MI355X_MICROARCH.md HBM section:
FETCH_SIZE counts half the bytes of 16-byte-per-lane reads, WRITE_SIZE is exact for 16-byte stores;
both include Infinity-Cache hits).  The first launch of the process (cold code objects, workspace
growth) is kept in the per-launch lists but excluded from the mean.
"""
import csv
import glob
import json
import os
import sys


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
    fdir, wdir, kname, dst = sys.argv[1:5]
    fetch = per_launch(fdir, "FETCH_SIZE", kname)
    write = per_launch(wdir, "WRITE_SIZE", kname)
    fm = sum(fetch[1:]) / max(1, len(fetch) - 1) if len(fetch) > 1 else fetch[0]
    wm = sum(write[1:]) / max(1, len(write) - 1) if len(write) > 1 else write[0]
    doc = {
        "kernel": kname,
        "config": "bench.py defaults (f64, B=500, D=784, K=10, 120-step launches)",
        "collection": "rocprofv3 --kernel-trace --pmc FETCH_SIZE, then a separate pass with --pmc WRITE_SIZE "
                      "(tools/gpu_pmc_bench.sh); summarised by tools/pmc_summary.py",
        "fetch_size_kb_per_launch": fetch,
        "write_size_kb_per_launch": write,
        "fetch_size_kb_mean": fm,
        "write_size_kb_mean": wm,
        "correction": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section); both count Infinity-Cache "
                      "(MALL) hits, so this is fabric traffic, not HBM-only",
        "traffic_bytes_per_launch": (2.0 * fm + wm) * 1024.0,
        "algorithmic_hbm_bytes_per_launch": 120 * 500 * 784 * 8,
        "note": "the minibatch tiles (3.1 MB per step) are the only algorithmic HBM reads; the rest is the tagged-"
                "granule exchange (write-through stores of partial sums, diff rows, weight slices) and its polling",
    }
    with open(dst, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps({k: doc[k] for k in ("fetch_size_kb_mean", "write_size_kb_mean", "traffic_bytes_per_launch")}))


if __name__ == "__main__":
    main()
