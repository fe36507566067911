#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/probe_hostpath.py > gpurun_out/hostpath.txt 2>&1 || { tail gpurun_out/hostpath.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/hostpath.txt
for rep in 1 2; do
  HMCX_BENCH_DEBUG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/h.json 2> gpurun_out/h.err || { tail gpurun_out/h.err; exit 1; }
  echo "$(python3 -c "import json; d=json.load(open('gpurun_out/h.json')); print('%.4g' % d['value'], 'wall_ms %.4f' % (d['ms_per_step']*20), 'launch_ms %.4f' % d['roofline']['launch_ms'])") | $(grep 'timed region' gpurun_out/h.err)"
done
