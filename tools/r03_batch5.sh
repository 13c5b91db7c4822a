#!/bin/bash
# In-process A/B of decode occupancy and prefetch depth: HEAD (2 waves, P 6), margin-0 build (3 waves, P 8)
# with and without the dec_waves = 2 cap, P 12 / P 19 builds (2 waves for 4-unknown tiles).
set -o pipefail
OUT=gpurun_out/r03j
mkdir -p $OUT
export TMPDIR=/tmp
V=pquic_amd/lib/variants
timeout -k 10 600 python tools/lib_ab.py head=$V/head/libpquic_fec.so all0=$V/all0/libpquic_fec.so "all0w2=$V/all0/libpquic_fec.so:dec_waves=2" p12=$V/p12/libpquic_fec.so p19=$V/p19/libpquic_fec.so "p12w3=$V/p12/libpquic_fec.so:dec_waves=3" --cycles=5 > $OUT/lib_ab.log 2>&1 || { tail $OUT/lib_ab.log; exit 1; }
cat $OUT/lib_ab.log
