#!/bin/bash
# round 4: nt symbol loads as the default -- confirm against the old default policy and against nt
# everywhere but the compact-map 8-repair encode bodies; GPU suite on the new default
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu_call11.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/ab_inproc.py "nt:" "old_default:LIB=pquic_amd/lib/variants/ld_default/libpquic_fec.so" \
  "nt_compact_default:LIB=pquic_amd/lib/variants/ld_compact_default/libpquic_fec.so" \
  --wide --cycles=6 --reps=5 > gpurun_out/r04/ab_ld_policy2.log 2>&1
