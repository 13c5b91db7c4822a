#!/bin/bash
# One GPU call: apply A/B (packed vs slots, group caps), the routine check (tests, smoke, bench, kernel
# trace), and the k16 PMC passes on the bench as it now runs (packed decode output).
set -o pipefail
OUT=gpurun_out/r03g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/apply_ab.py --cycles=5 > $OUT/apply_ab.log 2>&1 || { tail $OUT/apply_ab.log; exit 1; }
cat $OUT/apply_ab.log
bash tools/gpu_check.sh r03g_check || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_k16/$C -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --no-legs > $OUT/pmc_k16_$C.log 2>&1 || { tail -5 $OUT/pmc_k16_$C.log; exit 1; }
done
echo pmc done
