#!/bin/bash
# HMCX_P2_BAR A/B on the bench itself (600 timed steps, kernel ms per 120-step launch), 3 pairs.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for bar in ${BARS:-1 0}; do
  HMCX_P2_BAR=$bar HMCX_P2_XMAP=${XMAP:-1} timeout -k 10 120 python bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/bb.json 2> gpurun_out/bb.err || { tail gpurun_out/bb.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bb.json')); r=d['roofline']; print('BAR=$bar value %.4g launch_ms %.3f us/lf %.3f' % (d['value'], r['launch_ms'], r['launch_ms']*1e3/r['leapfrogs_per_launch']))"
done; done
