#!/bin/bash
# Chain-batched LDS pitches (noise tile 176 in f64, k_bfwd epilogue tile 163; libhmcx.so) vs the
# committed build (libhmcx_base.so): parity tests, SQ LDS counters of both at 2048 chains, then timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chains.py tests/test_gpu_samplers.py tests/test_gpu_multicore.py > gpurun_out/pytest_r05s.log 2>&1 || { tail -30 gpurun_out/pytest_r05s.log; exit 1; }
tail -1 gpurun_out/pytest_r05s.log
cd /tmp && export TMPDIR=/tmp
for lib in libhmcx_base.so libhmcx.so; do
  HMCX_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES -d $R/gpurun_out/lds_$lib -o run --output-format csv -- python3 $R/tools/probe_batch.py 2048 > $R/gpurun_out/lds_$lib.log 2>&1 || { tail -5 $R/gpurun_out/lds_$lib.log; exit 1; }
done
cd $R
python3 - <<'PY'
import csv, glob, collections
for lib in ("libhmcx_base.so", "libhmcx.so"):
    f = glob.glob("gpurun_out/lds_%s/**/*counter_collection.csv" % lib, recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hmcx::", "")
        if not k.startswith("k_b"): continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in sorted(acc.items()):
        print(lib, k, "LDS insts %.3g conflict cycles %.3g (%.2f%% of insts, %.2f%% of LDS-active cycles)" % (
            v["SQ_INSTS_LDS"], v["SQ_LDS_BANK_CONFLICT"], 100 * v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_INSTS_LDS"], 1),
            100 * v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_LDS_IDX_ACTIVE"], 1)))
PY
for rep in 1 2; do for lib in libhmcx_base.so libhmcx.so; do
  HMCX_LIB=$lib timeout -k 10 300 python -u tools/probe_batch.py 2048 8192 > gpurun_out/pbs_$lib.txt 2>&1 || { tail gpurun_out/pbs_$lib.txt; exit 1; }
  echo "$lib: $(grep -v amdgpu.ids gpurun_out/pbs_$lib.txt | tail -2 | cut -c1-140 | tr '\n' ' ')"
done; done
