"""Summarise the SQ-counter pass of tools/gpu_pmc_batch.sh (chain-batched probe) per kernel into a JSON file.

    python tools/pmc_batch_summary.py gpurun_out/pmcb "python3 tools/probe_batch.py 2048" profiles/pmc_r02_batched_sq.json

Per kernel: dispatches, device seconds (kernel trace of the same pass), the wave-state fractions
(SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES), MFMA busy as
SQ_VALU_MFMA_BUSY_CYCLES / (device seconds x 2.4 GHz x 1024 SIMDs), LDS instructions and LDS
bank-conflict cycles.  The profiled pass runs at its own (lower) clock, so the MFMA-busy fraction is a
lower bound on the unprofiled run's (MI355X_MICROARCH.md, DVFS).
"""
import collections
import csv
import glob
import json
import os
import sys

COUNTERS = ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
            "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_BUSY_CYCLES"]


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("hmcx::", "")
    return n


def main():
    d, cmd, dst = sys.argv[1:4]
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc:
        raise SystemExit("no counter_collection.csv under %s" % d)
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(cc[0])):
        if "hmcx" not in r["Kernel_Name"]:
            continue
        k = short(r["Kernel_Name"])
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    dur = collections.defaultdict(float)
    if kt:
        for r in csv.DictReader(open(kt[0])):
            if "hmcx" in r["Kernel_Name"]:
                dur[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for k, v in sorted(vals.items()):
        wc = v.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        ds = dur.get(k, 0.0)
        out[k] = {
            "dispatches": len(disp[k]),
            "device_s": ds,
            "wait_any_frac": v.get("SQ_WAIT_ANY", 0.0) / wc,
            "wait_inst_any_frac": v.get("SQ_WAIT_INST_ANY", 0.0) / wc,
            "active_inst_any_frac": v.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
            "mfma_busy_frac_of_1024_simds_at_2p4GHz":
                v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (ds * 2.4e9 * 1024) if ds > 0 else None,
            "lds_insts": v.get("SQ_INSTS_LDS", 0.0),
            "lds_bank_conflict_cycles": v.get("SQ_LDS_BANK_CONFLICT", 0.0),
        }
    doc = {"source": "rocprofv3 --kernel-trace --pmc " + " ".join(COUNTERS) + " -- " + cmd +
                     " (tools/gpu_pmc_batch.sh; summarised by tools/pmc_batch_summary.py)",
           "kernels": out}
    with open(dst, "w") as fh:
        json.dump(doc, fh, indent=1)
    for k, v in out.items():
        print("%-34s %5d disp %8.2f ms  mfma busy %s" % (k, v["dispatches"], v["device_s"] * 1e3,
              "%.3f" % v["mfma_busy_frac_of_1024_simds_at_2p4GHz"] if v["mfma_busy_frac_of_1024_simds_at_2p4GHz"] is not None else "-"))


if __name__ == "__main__":
    main()
