#!/bin/bash
# Cost of the float64 Box–Muller normals: the shipped library against an A/B build (built by hand with
# a define that made NormalT<double> draw the float stream; measured once, define since removed) whose f64 chains
# draw the float stream (lib/libhmcx_n32.so, -DHMCX_EXPERIMENT_F32_NOISE): headline bench (600 steps)
# and the 2048-chain batched probe, 3 alternating pairs.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for lib in libhmcx.so libhmcx_n32.so; do
  HMCX_LIB=$lib timeout -k 10 120 python bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/nab.json 2> gpurun_out/nab.err || { tail gpurun_out/nab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/nab.json')); r=d['roofline']; print('$lib headline us/lf %.3f' % (r['launch_ms']*1e3/r['leapfrogs_per_launch']))"
  HMCX_LIB=$lib timeout -k 10 120 python tools/probe_batch.py 2048 > gpurun_out/nab.log 2>&1 || { tail gpurun_out/nab.log; exit 1; }
  echo "$lib batched $(tail -1 gpurun_out/nab.log | grep -o 'kern [0-9.]* s')"
done; done
