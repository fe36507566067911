#!/bin/bash
# Round-2 measurement session: default bench line (driver shape --steps 20 --warmup 5), the
# 600-step line, rocprofv3 kernel stats of the driver shape, and PMC traffic (tools/gpu_r02_pmc.sh).
set -o pipefail
R=$(pwd)
TAG=${TAG:-r02}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_s20.json 2> gpurun_out/bench_${TAG}_s20.err || { tail gpurun_out/bench_${TAG}_s20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_s20.json')); print('s20', d['value'], d['ms_per_step']*20, d['roofline']['launch_ms'])"
timeout -k 10 300 python bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/bench_${TAG}_s600.json 2> gpurun_out/bench_${TAG}_s600.err || { tail gpurun_out/bench_${TAG}_s600.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_s600.json')); print('s600', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $R/gpurun_out/bench_prof_${TAG}.json 2> $R/gpurun_out/prof_${TAG}.err || { tail -5 $R/gpurun_out/prof_${TAG}.err; exit 1; }
cd $R && TAG=$TAG bash tools/gpu_r02_pmc.sh
