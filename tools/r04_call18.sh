#!/bin/bash
# round 4, final tree: the two-rank launch paths rehearsed on one GPU (ranks folded onto it, barrier and
# max-over-ranks reduction on gloo): bench.py's own spawn path and torchrun
set -o pipefail
mkdir -p gpurun_out/r04
export PQUIC_BENCH_SHARE_GPU=1 PQUIC_BENCH_BACKEND=gloo
timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-legs --cpu-seconds 4 > gpurun_out/r04/dist2_spawn_final.log 2>&1 &&
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-legs --no-cpu > gpurun_out/r04/dist2_torchrun_final.log 2>&1
