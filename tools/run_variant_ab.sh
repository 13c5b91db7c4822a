#!/bin/bash
# One GPU pass for generator variants: parity tests (tests/test_gpu_parity.py) on each variant's
# library, then an in-process A/B against the main build.
# usage: bash tools/run_variant_ab.sh TAG "ab_inproc options" variant1 [variant2 ...]
set -o pipefail
TAG=$1; OPTS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
specs=(base)
for v in "$@"; do
  PQUIC_AMD_LIB=$PWD/pquic_amd/lib/variants/$v/libpquic_fec.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { tail -n 20 $OUT/pytest_$v.log; exit 1; }
  tail -n 1 $OUT/pytest_$v.log
  specs+=("$v:LIB=pquic_amd/lib/variants/$v/libpquic_fec.so")
done
timeout -k 10 600 python -u tools/ab_inproc.py "${specs[@]}" $OPTS > $OUT/ab.log 2>&1
rc=$?; cat $OUT/ab.log; exit $rc
