#!/bin/bash
# round 4: 8-repair encode tiles on the wide register map (3 waves/SIMD, 4 sources in flight) with nt or
# default loads, against the compact map at 4 waves (this tree)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u tools/ab_inproc.py "compact:" "wide_nt:LIB=pquic_amd/lib/variants/enc8_wide/libpquic_fec.so" \
  "wide_default:LIB=pquic_amd/lib/variants/enc8_wide_dflt/libpquic_fec.so" --only \
  --case=enc:32:8:1048576:1200 --case=enc:32:8:2097152:1200 --case=enc:16:8:1048576:1200 --cycles=6 --reps=4 > gpurun_out/r04/ab_enc8_wide_nt.log 2>&1
