#!/bin/bash
# Round 5 box 4: where config 3 (MLP f32) and the 2048-chain batched path spend their time — kernel
# traces of the probes, per-kernel medians and gaps.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/mlpkt -o run -- python3 $R/tools/probe_mlp.py 40 > $R/gpurun_out/mlpkt.log 2>&1 || { tail -5 $R/gpurun_out/mlpkt.log; exit 1; }
tail -3 $R/gpurun_out/mlpkt.log
KT=$(find $R/gpurun_out/mlpkt -name "*kernel_trace.csv" | head -1)
python3 $R/tools/kernel_timeline.py $KT hmcx 400 60 > $R/gpurun_out/mlp_timeline.txt && tail -25 $R/gpurun_out/mlp_timeline.txt
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/bkt5 -o run -- python3 $R/tools/probe_batch.py 2048 > $R/gpurun_out/bkt5.log 2>&1 || { tail -5 $R/gpurun_out/bkt5.log; exit 1; }
grep "C=" $R/gpurun_out/bkt5.log
KT=$(find $R/gpurun_out/bkt5 -name "*kernel_trace.csv" | head -1)
python3 $R/tools/batch_launch_profile.py $KT > $R/gpurun_out/batch_launch_profile5.txt && tail -14 $R/gpurun_out/batch_launch_profile5.txt
