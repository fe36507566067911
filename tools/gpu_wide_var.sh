#!/bin/bash
# Config-5 SGLD: tiling variants of hmcx_wide.hip (libraries built with -DHMCX_GNW / -DHMCX_WDZ).
set -o pipefail
mkdir -p gpurun_out
V=dropout_hamiltonian_montecarlo_amd/lib/var
for lib in default g16 z64 gz default g16 z64 gz; do
  if [ $lib = default ]; then unset HMCX_LIB; else export HMCX_LIB=var/libhmcx_$lib.so; fi
  if [ $lib != default ]; then timeout -k 10 120 python -u -m pytest tests/test_gpu_samplers.py -q -x --timeout 120 --timeout-method thread -k wide > gpurun_out/wv.log 2>&1 || { tail -20 gpurun_out/wv.log; exit 1; }; fi
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 400 > gpurun_out/wv.json 2> gpurun_out/wv.err || { tail gpurun_out/wv.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/wv.json'))['plantvillage_sgld']; print(sys.argv[1], round(d['us_per_step'],2), round(d['roofline']['frac'],4))" $lib
done
