#!/bin/bash
# round 4, final tree: the bench line, the same bench under a kernel trace, and the two-rank launch
# path rehearsed on one GPU (ranks folded onto it)
set -o pipefail
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r04/bench_final.log 2>&1 || { tail -20 gpurun_out/r04/bench_final.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/bench_final_prof -o bench --output-format csv -- python -u bench.py --no-cpu > gpurun_out/r04/bench_final_prof.log 2>&1 || exit 1
PQUIC_BENCH_SHARE_GPU=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-legs --cpu-seconds 4 > gpurun_out/r04/dist2_spawn_final.log 2>&1
