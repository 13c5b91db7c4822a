#!/bin/bash
# Final-build GPU pass: tests, smoke, bench with its legs, kernel trace of the headline, k16 PMC passes.
set -o pipefail
OUT=gpurun_out/r03k
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_check.sh r03k_check || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_k16/$C -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --no-legs > $OUT/pmc_k16_$C.log 2>&1 || { tail -5 $OUT/pmc_k16_$C.log; exit 1; }
done
echo pmc done
