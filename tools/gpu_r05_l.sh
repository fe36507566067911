#!/bin/bash
# Segment profile (HMCX_PERSIST_PROF) of the config-2 instantiation: merged step-start round vs base.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
for rep in 1 2; do for lib in libhmcx_base.so libhmcx.so; do
  HMCX_LIB=$lib HMCX_PERSIST_PROF=1 timeout -k 10 120 python tools/probe_sghmc.py > gpurun_out/p2prof_$lib.txt 2>&1 || { tail gpurun_out/p2prof_$lib.txt; exit 1; }
  echo "== $lib"; grep -v amdgpu.ids gpurun_out/p2prof_$lib.txt | tail -3
done; done
