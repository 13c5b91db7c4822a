#!/bin/bash
# round 4: RT = 16 ring kernels without scratch spills -- GPU suite, in-process A/B against the
# spilling build (pquic_amd/lib/variants/spill), SQ counter passes on the r >= 8 configurations.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu_nospill.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_inproc.py "nospill:" "spill:LIB=pquic_amd/lib/variants/spill/libpquic_fec.so" \
  --only --cycles=5 --reps=5 --case=enc:64:16:65536:9000 --case=dec:64:16:65536:9000 \
  --case=enc:32:16:262144:1200 --case=dec:32:16:262144:1200 > gpurun_out/r04/ab_spill.log 2>&1 || exit 1
bash tools/sq_evidence.sh r04_sq > gpurun_out/r04/sq_evidence.log 2>&1
