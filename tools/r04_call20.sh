#!/bin/bash
# round 4: k32 r8 encode group size (blocks per wave's stream: 8 default, 4, 2), in process, 2^20 and
# 2^21 blocks
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u tools/ab_inproc.py "g8:" "g4:group=4" "g2:group=2" --only \
  --case=enc:32:8:1048576:1200 --case=enc:32:8:2097152:1200 --cycles=8 --reps=5 > gpurun_out/r04/ab_k32_group.log 2>&1
