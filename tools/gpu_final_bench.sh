#!/bin/bash
# Default bench line (reads profiles/pmc_r01_f64_persistent.json for the traffic field).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail gpurun_out/bench_final.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_final.json')); print(d['value'], d['roofline']['traffic'], d['roofline']['launch_ms'])"
