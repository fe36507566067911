#!/bin/bash
# Rehearse the multi-rank bench path on a one-GPU box: 2 ranks share cuda:0, gloo collectives.
set -o pipefail
mkdir -p gpurun_out
HMCX_BENCH_SHARED_GPU=1 HMCX_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 240 --warmup 120 --cpu-seconds 0 --batched-chains 64 > gpurun_out/dist2.json 2> gpurun_out/dist2.err || { tail -20 gpurun_out/dist2.err; exit 1; }
cat gpurun_out/dist2.json
