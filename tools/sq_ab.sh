#!/bin/bash
# SQ counter passes for one kernel configuration under an environment (A/B of knobs).
# usage (GPU box): bash tools/sq_ab.sh TAG "ENV=..." MODE K R BLOCKS [L]
set -o pipefail
TAG=$1; ENVS=$2; MODE=$3; K=$4; R=$5; NB=$6; L=${7:-1200}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
env $ENVS FEC_L=$L bash tools/pmc_sq.sh $TAG/raw $MODE $K $R $NB 2 > $OUT/pmc.txt 2>&1 || exit 1
python tools/sq_summary.py gpurun_out/$TAG/raw $NB "$TAG $MODE k$K r$R L$L $ENVS"
