#!/bin/bash
# SGLD one chain: wide path (HMCX_SGLD_WIDE=1) vs kernel-per-phase path (0), MNIST and config-5 shapes.
set -o pipefail
for shape in "mnist" ""; do for w in 1 0; do
  HMCX_SGLD_WIDE=$w timeout -k 10 120 python tools/probe_sgld.py 200 $shape > gpurun_out/probe_sgld.log 2>&1 || { tail gpurun_out/probe_sgld.log; exit 1; }
  echo "wide=$w $shape $(tail -1 gpurun_out/probe_sgld.log)"
done; done
