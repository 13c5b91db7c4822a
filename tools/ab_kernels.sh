#!/bin/bash
# Interleaved kernel-only A/B (less noisy than whole bench runs): ROUNDS x (variants) x configs.
# A variant is LIB or LIB:VAR=VAL[,VAR=VAL] (environment for that run); LIB "main" is
# pquic_amd/lib/libpquic_fec.so, anything else pquic_amd/lib/variants/LIB/libpquic_fec.so.
# usage: bash tools/ab_kernels.sh TAG variant1 [variant2 ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for round in ${ROUNDS:-1 2 3}; do
  for spec in "$@"; do
    v=${spec%%:*}; envs=""
    [ "$spec" != "$v" ] && envs=$(echo "${spec#*:}" | tr "," " ")
    if [ "$v" = main ]; then lib=pquic_amd/lib/libpquic_fec.so; else lib=pquic_amd/lib/variants/$v/libpquic_fec.so; fi
    line="$spec r$round"
    for cfg in ${CONFIGS:-enc@16@4@1048576 dec@16@4@1048576 enc@32@8@1048576}; do
      cfg=${cfg//@/ }
      res=$(env $envs PQUIC_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/kernel_only.py $cfg ${REPS:-10} 2>&1 | tail -1) || { echo "$res"; exit 1; }
      line="$line | $(echo $res | sed 's/.*: //; s/ ms per call//')"
    done
    echo "$line" | tee -a $OUT/ab.log
  done
done
