#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  HMCX_HOST_PROF=1 HMCX_BENCH_DEBUG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/h.json 2> gpurun_out/h.err || { tail gpurun_out/h.err; exit 1; }
  grep -A1 'timed region' gpurun_out/h.err
done
