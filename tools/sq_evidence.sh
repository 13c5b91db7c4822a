#!/bin/bash
# SQ counter evidence for the r >= 8 data-path kernels (tools/pmc_sq.sh per configuration) and a
# kernel-trace --stats run of the full bench with its legs.  usage (GPU box): bash tools/sq_evidence.sh TAG
set -o pipefail
TAG=${1:-sq}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/pmc_sq.sh $TAG/enc_k32_r8 enc 32 8 1048576 3 > $OUT/enc_k32_r8.txt 2>&1 || exit 1
bash tools/pmc_sq.sh $TAG/dec_k32_e8 dec 32 8 1048576 3 > $OUT/dec_k32_e8.txt 2>&1 || exit 1
FEC_L=9000 bash tools/pmc_sq.sh $TAG/enc_k64_r16 enc 64 16 65536 3 > $OUT/enc_k64_r16_L9000.txt 2>&1 || exit 1
FEC_L=9000 bash tools/pmc_sq.sh $TAG/dec_k64_e16 dec 64 16 65536 3 > $OUT/dec_k64_e16_L9000.txt 2>&1 || exit 1
bash tools/pmc_sq.sh $TAG/enc_k16_r4 enc 16 4 1048576 3 > $OUT/enc_k16_r4.txt 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/bench -o bench --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu > $OUT/bench.log 2>&1 || exit 1
ls $OUT
