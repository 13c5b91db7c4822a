#!/bin/bash
# Group-setup overhead probes (round 3): in-process A/B of the recover data pass with its plan
# records staged in LDS (ws_lds=1) or read in place (0), against timing-probe builds whose group
# setup reads no workspace (nows) or runs no TinyMT32 (constco), and the access-pattern ceilings
# (tools/microbench/layout_probe) on the same box.
# usage (GPU box, from the repo root): bash tools/probe_setup.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/probe_setup}
mkdir -p $OUT
timeout -k 10 400 python tools/ab_inproc.py base wsoff:ws_lds=0 \
  "nows:LIB=pquic_amd/lib/variants/nows/libpquic_fec.so" \
  "constco:LIB=pquic_amd/lib/variants/constco/libpquic_fec.so" --cycles=5 > $OUT/ab_probe.log 2>&1 || { tail $OUT/ab_probe.log; exit 1; }
cat $OUT/ab_probe.log
timeout -k 10 200 tools/microbench/layout_probe > $OUT/layout.log 2>&1 || { tail $OUT/layout.log; exit 1; }
head -20 $OUT/layout.log
