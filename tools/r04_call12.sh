#!/bin/bash
# round 4: occupancy / prefetch-depth variants of the register-prefetch bodies under nt loads
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u tools/lib_ab.py base=pquic_amd/lib/libpquic_fec.so \
  dec4_3w=pquic_amd/lib/variants/dec4_3w/libpquic_fec.so dec4_4w=pquic_amd/lib/variants/dec4_4w/libpquic_fec.so \
  enc4_2w=pquic_amd/lib/variants/enc4_2w/libpquic_fec.so enc8_3w=pquic_amd/lib/variants/enc8_3w/libpquic_fec.so \
  --cycles=5 > gpurun_out/r04/ab_occupancy_nt.log 2>&1
