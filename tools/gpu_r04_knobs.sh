#!/bin/bash
# Persistent-kernel protocol knobs and plans re-swept on the round-4 build: 600-step headline only, two
# passes.  Every knob row runs the generic kernel (HMCX_P2_SPEC=0) against the generic default, since a
# non-default knob disables the folded config-2 instantiation; the first row is the folded default.
set -o pipefail
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 120 python bench.py --steps 600 --warmup 120 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("%.4e %.4f" % (d["value"], d["roofline"]["launch_ms"]))'
}
for pass in 1 2; do
  echo "spec-default $(run HMCX_NOP=1)" || exit 1
  for cfg in "HMCX_NOP=1" "HMCX_P2_GRID=16x8" "HMCX_P2_GRID=16x16" "HMCX_P2_GRID=8x8" "HMCX_P2_SPREAD=0" "HMCX_P2_SPREAD=3" "HMCX_P2_SPREAD=6" "HMCX_P2_SPREAD=10" "HMCX_P2_BAR=0" "HMCX_P2_FL2=0" "HMCX_P2_ACC1=0" "HMCX_P2_PREFETCH=0" "HMCX_P2_ZOFF=0"; do
    echo "$cfg $(run HMCX_P2_SPEC=0 $cfg)" || exit 1
  done
done
