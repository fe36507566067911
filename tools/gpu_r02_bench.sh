#!/bin/bash
# Round-2 bench session: the driver's call shape (--steps 20 --warmup 5), the default shape, and a
# rocprofv3 kernel-stats run of the driver shape.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.json 2> gpurun_out/bench_s20.err || { echo bench failed; tail gpurun_out/bench_s20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s20.json')); print('s20', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
timeout -k 10 300 python bench.py --cpu-seconds 0 --batched-chains 0 --mlp-steps 0 --sgld-steps 0 > gpurun_out/bench_s600.json 2> gpurun_out/bench_s600.err || { echo bench2 failed; tail gpurun_out/bench_s600.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_s600.json')); print('s600', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_s20 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/prof.err || { echo prof failed; tail $R/gpurun_out/prof.err; exit 1; }
find $R/gpurun_out/prof_s20 -name "*stats*"
