#!/bin/bash
# One GPU-box pass for a kernel change: the whole GPU test suite, then an interleaved kernel-only
# A/B (tools/ab_kernels.sh) of the given variants.
# usage: bash tools/gpu_ab.sh TAG variant1 [variant2 ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit 1
bash tools/ab_kernels.sh $TAG "$@"
