#!/bin/bash
# round 4: GPU suite on the current tree; cache policy of the symbol loads (FEC_LD_POL) -- default vs
# nt / sc1 / nt sc1, in process
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu_call10.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/ab_inproc.py "base:" "nt:LIB=pquic_amd/lib/variants/ld_nt/libpquic_fec.so" \
  "sc1:LIB=pquic_amd/lib/variants/ld_sc1/libpquic_fec.so" "ntsc1:LIB=pquic_amd/lib/variants/ld_ntsc1/libpquic_fec.so" \
  --wide --cycles=5 --reps=5 > gpurun_out/r04/ab_ld_policy.log 2>&1
