#!/bin/bash
# Host-overhead A/B of the driver-shape headline across source trees on one box: HEAD (.) against git
# worktrees of older commits checked out and built under the repo root (TREES="." "_old" ...).
set -o pipefail
R=$(pwd)
for rep in 1 2; do for t in ${TREES:-. _old _old2}; do
  (cd $R/$t && HMCX_BENCH_DEBUG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > $R/gpurun_out/h.json 2> $R/gpurun_out/h.err) || { tail $R/gpurun_out/h.err; exit 1; }
  echo "[$t] $(python3 -c "import json; d=json.load(open('$R/gpurun_out/h.json')); print('%.4g' % d['value'], 'wall_ms %.4f' % (d['ms_per_step']*20), 'launch_ms %.4f' % d['roofline']['launch_ms'])") | $(grep 'timed region' $R/gpurun_out/h.err)"
done; done
