# round 4: split encode group / interleave variants (in-process A/B)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u tools/ab_inproc.py "base:split=0" "sp4:split=4" "sp4g1:split=4,group=1" "sp4ilv0:split=4,interleave=0" "sp2g1:split=2,group=1" --cycles=4 --reps=5 > gpurun_out/r04/ab_split3.log 2>&1
