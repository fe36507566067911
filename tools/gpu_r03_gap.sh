#!/bin/bash
# Driver-shape headline (bench.py --steps 20 --warmup 5) vs the 600-step figure, same box.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3 4; do
  HMCX_BENCH_DEBUG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/h.json 2> gpurun_out/h.err || { tail gpurun_out/h.err; exit 1; }
  echo "$(python3 -c "import json; d=json.load(open('gpurun_out/h.json')); print('%.4g' % d['value'], 'wall_ms %.4f' % (d['ms_per_step']*20), 'launch_ms %.4f' % d['roofline']['launch_ms'], 'lf', d['leapfrogs'])") | $(grep 'timed region' gpurun_out/h.err)"
done
for rep in 1 2; do
  timeout -k 10 300 python bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/s600.json 2> gpurun_out/s600.err || { tail gpurun_out/s600.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s600.json')); print('s600 %.4g' % d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
done
