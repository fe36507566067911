#!/bin/bash
# Config-5 wide SGLD: in-kernel phase stamps (HMCX_WIDE_PROF) of the three variants, f64.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
for cfg in "1 1 fused team" "1 0 fused" "0 0"; do
  set -- $cfg
  f=gpurun_out/wide_prof_$1$2.bin
  rm -f $f
  HMCX_WIDE_FUSE=$1 HMCX_WIDE_GTEAM=$2 HMCX_WIDE_PROF=$R/$f timeout -k 10 120 python tools/probe_sgld.py 64 > gpurun_out/wide_probe.txt 2>&1 || { tail gpurun_out/wide_probe.txt; exit 1; }
  echo "== fuse=$1 gteam=$2"
  python3 tools/wide_prof_summary.py $f $3 $4
done
