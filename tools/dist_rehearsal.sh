#!/bin/bash
# 2-rank rehearsals of the multi-GPU bench on a 1-GPU box: both ranks share device 0 and talk over
# gloo (RCCL refuses two ranks on one device).  The driver's real runs use one GPU per rank.
#   1. torchrun launch (the driver's N > 1 command)
#   2. plain `python bench.py --gpus 2` (no WORLD_SIZE: bench.py starts the ranks itself)
set -o pipefail
OUT=gpurun_out/${1:-dist2}
shift
mkdir -p $OUT
export PQUIC_BENCH_SHARE_GPU=1 PQUIC_BENCH_BACKEND=gloo
MASTER_ADDR=127.0.0.1 timeout -k 10 400 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 5 --warmup 2 "$@" > $OUT/bench_torchrun.log 2>&1 || { tail -20 $OUT/bench_torchrun.log; exit 1; }
grep '^{' $OUT/bench_torchrun.log | cut -c1-300
timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 "$@" > $OUT/bench_spawn.log 2>&1 || { tail -20 $OUT/bench_spawn.log; exit 1; }
grep '^{' $OUT/bench_spawn.log | cut -c1-300
