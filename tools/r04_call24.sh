#!/bin/bash
# round 4, final tree: the default bench line twice more (box / thermal spread of the headline)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/r04/bench_final_b.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu --no-legs > gpurun_out/r04/bench_final_c.log 2>&1
