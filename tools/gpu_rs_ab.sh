#!/bin/bash
# Row-space persistent SGHMC (HMCX_RS=1, opt-in) against the 2-D persistent kernel (HMCX_RS=0, default):
# µs per leapfrog (probe, 3 alternating pairs), the driver-shape bench line with each, and the
# kernel split of one row-space bench run (rocprofv3 --kernel-trace --stats).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
for rep in 1 2 3; do for rs in 1 0; do
  HMCX_RS=$rs timeout -k 10 60 python tools/probe_sghmc.py reps=9 > gpurun_out/ab.log 2>&1 || { tail gpurun_out/ab.log; exit 1; }
  echo "[RS=$rs] $(tail -1 gpurun_out/ab.log | grep -o 'us/lf [0-9.]*')"
done; done
for rs in 1 0; do
  HMCX_RS=$rs HMCX_BENCH_DEBUG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  echo "[bench RS=$rs] $(python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('%.4g' % d['value'], 'wall_ms %.4f' % (d['ms_per_step']*20), 'launch_ms %.4f' % d['roofline']['launch_ms'])")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rs -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > $R/gpurun_out/prof_rs.json 2> $R/gpurun_out/prof_rs.err || { tail -5 $R/gpurun_out/prof_rs.err; exit 1; }
cut -d, -f1-4 $R/gpurun_out/prof_rs/run_kernel_stats.csv | head -8
