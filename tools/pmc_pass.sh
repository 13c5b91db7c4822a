#!/bin/bash
# PMC HBM-traffic passes (separate rocprofv3 runs per counter group, kernel trace only).
# usage: bash tools/pmc_pass.sh TAG [bench args]
set -o pipefail
TAG=${1:-pmc}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d $OUT/$C -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --no-legs "$@" > $OUT/$C.log 2>&1 || { tail -5 $OUT/$C.log; exit 1; }
done
ls -R $OUT | head -20
