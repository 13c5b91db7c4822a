#!/bin/bash
# Encode occupancy / prefetch A/B (4-repair tiles at 2 waves with 19 rows in flight; 8-repair tiles on
# the wide map at 2 waves with 15) against the current build, then the final-build pass.
set -o pipefail
OUT=gpurun_out/r03l
mkdir -p $OUT
export TMPDIR=/tmp
V=pquic_amd/lib/variants
timeout -k 10 600 python tools/lib_ab.py cur=$V/cur/libpquic_fec.so e19=$V/e19/libpquic_fec.so e8w2=$V/e8w2/libpquic_fec.so --cycles=5 > $OUT/lib_ab.log 2>&1 || { tail $OUT/lib_ab.log; exit 1; }
cat $OUT/lib_ab.log
bash tools/r03_batch6.sh
