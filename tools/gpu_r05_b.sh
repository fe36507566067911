#!/bin/bash
# Round 5 box 2: GPU suite (recovery guard), headline early-A A/B (driver shape and 600 steps,
# alternating libraries), config-5 SGLD with class-pair gradient loads.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r05b.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_r05b.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_r05b.log
H="--cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0"
for rep in 1 2 3; do
  for lib in libhmcx.so libhmcx_noearly.so; do
    HMCX_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 $H > gpurun_out/ab.json 2>/dev/null || { echo "bench failed ($lib)"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$lib s20', '%.4e' % d['value'], '%.1f' % (d['roofline']['launch_ms']*1e3), d['recoveries'])"
    HMCX_LIB=$lib timeout -k 10 120 python bench.py $H > gpurun_out/ab.json 2>/dev/null || { echo "bench failed ($lib)"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$lib s600', '%.4e' % d['value'], d['recoveries'])"
  done
done
for rep in 1 2; do
  timeout -k 10 120 python tools/probe_sgld.py 400 2>&1 | tail -2
done
