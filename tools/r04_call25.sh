#!/bin/bash
# round 4: 4-repair encode tiles on the compact register map (4 waves/SIMD; 5 with a 96-VGPR budget)
# under nt loads, against the wide map at 3 waves (this tree)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u tools/lib_ab.py base=pquic_amd/lib/libpquic_fec.so \
  compact4w=pquic_amd/lib/variants/enc4_compact/libpquic_fec.so \
  compact5w=pquic_amd/lib/variants/enc4_compact5/libpquic_fec.so --cycles=6 > gpurun_out/r04/ab_enc4_compact_nt.log 2>&1
