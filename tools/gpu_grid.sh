#!/bin/bash
# Persistent-kernel grid sweep (HMCX_P2_GRID) with the default XCD placement.
set -o pipefail
mkdir -p gpurun_out
for g in ${GRIDS:-8x16 8x32 8x24 8x20 8x16}; do
  HMCX_P2_GRID=$g timeout -k 10 120 python bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/xm.json 2> gpurun_out/xm.err || { tail gpurun_out/xm.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/xm.json')); print(sys.argv[1], round(d['value']/1e6,1), round(d['roofline']['launch_ms'],3))" $g
done
