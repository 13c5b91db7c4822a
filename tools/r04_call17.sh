#!/bin/bash
# round 4: where the k16 e4 apply loses to its access pattern (trivial-compute probe: as fast as the
# encode's) -- workspace records in LDS or not, group sizes, 3 waves/SIMD, and a timing-only build
# whose setup reads no workspace (FEC_PROBE_NOWS: wrong bytes)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u tools/lib_ab.py base=pquic_amd/lib/libpquic_fec.so \
  wslds0=pquic_amd/lib/libpquic_fec.so:ws_lds=0 g4=pquic_amd/lib/libpquic_fec.so:group=4 \
  g16=pquic_amd/lib/libpquic_fec.so:group=16 dec4_3w=pquic_amd/lib/variants/dec4_3w/libpquic_fec.so \
  nows=pquic_amd/lib/variants/nows/libpquic_fec.so --cycles=5 > gpurun_out/r04/ab_apply_nt.log 2>&1
