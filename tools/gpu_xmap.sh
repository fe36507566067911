#!/bin/bash
# A/B of the persistent kernel's store flavour on cross-XCD rounds (HMCX_P2_PLAIN).
set -o pipefail
mkdir -p gpurun_out
HMCX_P2_PLAIN=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_samplers.py -x -q --timeout 120 --timeout-method thread -k "sghmc or persist" > gpurun_out/xmap_pytest.log 2>&1 || { tail -20 gpurun_out/xmap_pytest.log; exit 1; }
tail -1 gpurun_out/xmap_pytest.log
for p in 0 1 0 1 0 1; do
  HMCX_P2_PLAIN=$p timeout -k 10 120 python bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/xm.json 2> gpurun_out/xm.err || { tail gpurun_out/xm.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/xm.json')); print(sys.argv[1], round(d['value']/1e6,1), round(d['roofline']['launch_ms'],3))" $p
done
