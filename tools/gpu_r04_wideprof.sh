#!/bin/bash
# Config-5 wide SGLD: in-kernel phase stamps (HMCX_WIDE_PROF) of the fused and three-launch paths, f64.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
for f in 1 0; do
  out=gpurun_out/wide_prof_f$f.bin
  rm -f $out
  HMCX_WIDE_FUSE=$f HMCX_WIDE_PROF=$R/$out timeout -k 10 120 python tools/probe_sgld.py 64 > gpurun_out/wide_probe.txt 2>&1 || { tail gpurun_out/wide_probe.txt; exit 1; }
  echo "== fuse=$f"
  python3 tools/wide_prof_summary.py $out $([ $f = 1 ] && echo fused)
done
