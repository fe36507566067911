#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for C in 2048 4096 8192; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --batched-chains $C --mlp-steps 0 --sgld-steps 0 > gpurun_out/b$C.json 2> gpurun_out/b$C.err || { tail gpurun_out/b$C.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b$C.json'))['chain_batched']; print($C, 'frac %.4f' % d['roofline']['frac'], 'lf/s %.4g' % d['leapfrogs_per_s'], 'ms %.1f' % d['ms'])"
done
