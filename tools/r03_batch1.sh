#!/bin/bash
# One GPU call: headline bench (plan on its own stream), split-wave pattern probe, PMC traffic refresh.
set -o pipefail
OUT=gpurun_out/r03e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-legs --no-cpu > $OUT/bench_head.log 2>&1 || { tail $OUT/bench_head.log; exit 1; }
tail -1 $OUT/bench_head.log | cut -c1-400
SPLIT_ONLY=1 timeout -k 10 200 tools/microbench/layout_probe > $OUT/split.log 2>&1 || { tail $OUT/split.log; exit 1; }
cat $OUT/split.log
DEC_ONLY=1 timeout -k 10 200 tools/microbench/layout_probe > $OUT/dec.log 2>&1 || { tail $OUT/dec.log; exit 1; }
cat $OUT/dec.log
bash tools/pmc_refresh.sh r03_pmc
