#!/bin/bash
# round 4: k16 r4 encode group size under nt loads (2 default; 1, 4), in process
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u tools/ab_inproc.py "g2:" "g1:group=1" "g4:group=4" --only \
  --case=enc:16:4:1048576:1200 --case=dec:16:4:1048576:1200 --cycles=8 --reps=5 > gpurun_out/r04/ab_k16_group_nt.log 2>&1
