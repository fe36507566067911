#!/bin/bash
# A/B of the persistent kernel's spread-gather mask (HMCX_P2_SPREAD) under the XCD placement.
set -o pipefail
mkdir -p gpurun_out
for sp in 2 0 3 2 10 15 2 0; do
  HMCX_P2_SPREAD=$sp timeout -k 10 120 python bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/xm.json 2> gpurun_out/xm.err || { tail gpurun_out/xm.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/xm.json')); print(sys.argv[1], round(d['value']/1e6,1), round(d['roofline']['launch_ms'],3))" $sp
done
