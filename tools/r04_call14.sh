#!/bin/bash
# round 4: window bodies back on the default load policy (A/B against nt); HBM-traffic PMC passes on
# the nt build (tools/pmc_refresh.sh)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u tools/ab_inproc.py "sc_default:" "sc_nt:LIB=pquic_amd/lib/variants/sc_nt/libpquic_fec.so" \
  --only --case=win8:32:8:2097152:1200 --case=win1:30:4:2097152:1200 --case=win10:30:4:2097152:1200 \
  --cycles=4 --reps=3 > gpurun_out/r04/ab_sc_policy.log 2>&1 || exit 1
bash tools/pmc_refresh.sh r04_pmc > gpurun_out/r04/pmc_refresh.log 2>&1
