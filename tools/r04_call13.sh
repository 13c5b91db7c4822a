#!/bin/bash
# round 4: the bench line on the current tree, then the same bench under a kernel trace
set -o pipefail
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r04/bench_nt.log 2>&1 || { tail -20 gpurun_out/r04/bench_nt.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/bench_nt_prof -o bench --output-format csv -- python -u bench.py --no-cpu > gpurun_out/r04/bench_nt_prof.log 2>&1
