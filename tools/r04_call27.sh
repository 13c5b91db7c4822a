#!/bin/bash
# round 4: what the timing-only "no workspace" apply saves, split in two (wrong bytes, timing only):
# constant coefficients with the real slot map, and the real coefficients with a fixed slot map
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u tools/lib_ab.py base=pquic_amd/lib/libpquic_fec.so \
  nows=pquic_amd/lib/variants/nows/libpquic_fec.so constcoef=pquic_amd/lib/variants/constcoef/libpquic_fec.so \
  fixedslots=pquic_amd/lib/variants/fixedslots/libpquic_fec.so --cycles=6 > gpurun_out/r04/ab_apply_probe_split.log 2>&1
