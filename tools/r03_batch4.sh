#!/bin/bash
# One GPU call: in-process A/B of library builds (session start, HEAD = regressed recover occupancy,
# one group per workgroup with decode margin 14 / 0), then the GPU suite on the current tree.
set -o pipefail
OUT=gpurun_out/r03i
mkdir -p $OUT
export TMPDIR=/tmp
V=pquic_amd/lib/variants
timeout -k 10 500 python tools/lib_ab.py start=$V/start/libpquic_fec.so head=$V/head/libpquic_fec.so m0=$V/m0/libpquic_fec.so all14=$V/all14/libpquic_fec.so all0=$V/all0/libpquic_fec.so --cycles=5 > $OUT/lib_ab.log 2>&1 || { tail $OUT/lib_ab.log; exit 1; }
cat $OUT/lib_ab.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
