#!/bin/bash
# round 4: recover tiles streaming a block's inputs in memory order (FEC_DEC_SORTED, this tree) against
# equation-slot order (variants/slotorder); decode parity first
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "decode or recover or full_size" > gpurun_out/r04/pytest_sorted.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/lib_ab.py sorted=pquic_amd/lib/libpquic_fec.so \
  slotorder=pquic_amd/lib/variants/slotorder/libpquic_fec.so --cycles=8 > gpurun_out/r04/ab_dec_sorted.log 2>&1
