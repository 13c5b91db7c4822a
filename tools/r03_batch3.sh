#!/bin/bash
# One GPU call: encode pattern probe (G1 / G2 / split waves, alternating), the configs[3] / [4] bench
# lines, and a 4-rank rehearsal of bench.py --gpus 4 on one GPU (gloo, ranks sharing the device).
set -o pipefail
OUT=gpurun_out/r03h
mkdir -p $OUT
export TMPDIR=/tmp
SPLIT_ONLY=1 timeout -k 10 300 tools/microbench/layout_probe > $OUT/split2.log 2>&1 || { tail $OUT/split2.log; exit 1; }
cat $OUT/split2.log
timeout -k 10 400 python bench.py --config k32r8 --no-cpu --steps 5 --warmup 2 > $OUT/bench_k32r8.log 2>&1 || { tail $OUT/bench_k32r8.log; exit 1; }
tail -1 $OUT/bench_k32r8.log | cut -c1-300
timeout -k 10 300 python bench.py --config k64r16 --no-cpu --steps 5 --warmup 2 > $OUT/bench_k64r16.log 2>&1 || { tail $OUT/bench_k64r16.log; exit 1; }
tail -1 $OUT/bench_k64r16.log | cut -c1-300
PQUIC_BENCH_SHARE_GPU=1 PQUIC_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 4 --no-legs --steps 4 --warmup 1 > $OUT/dist4.log 2>&1 || { tail $OUT/dist4.log; exit 1; }
grep '^{' $OUT/dist4.log | cut -c1-200
grep -o '"per_rank_ms_per_step": \[[^]]*\]' $OUT/dist4.log
