#!/bin/bash
# round 4, final tree: configs[3] (k32 r8, 2^24 blocks in passes) and configs[4] (k64 r16 L9000) as bench lines
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 500 python -u bench.py --config k32r8 --no-cpu > gpurun_out/r04/bench_final_k32r8.log 2>&1 &&
timeout -k 10 500 python -u bench.py --config k64r16 --no-cpu > gpurun_out/r04/bench_final_k64r16.log 2>&1
