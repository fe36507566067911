#!/bin/bash
# Round 4 profiling: wide SGLD stamps (three variants), MLP config-3 kernel timeline (f32).
set -o pipefail
R=$(pwd)
bash tools/gpu_r04_wideprof.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_mlp_tl -o run --output-format csv -- python3 $R/tools/probe_mlp.py 40 > $R/gpurun_out/probe_mlp_tl.txt 2>&1 || { tail -5 $R/gpurun_out/probe_mlp_tl.txt; exit 1; }
tail -1 $R/gpurun_out/probe_mlp_tl.txt
f=$(ls $R/gpurun_out/prof_mlp_tl/*kernel_trace.csv $R/gpurun_out/prof_mlp_tl/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 $R/tools/kernel_timeline.py $f hmcx 300 45
