#!/bin/bash
# Refresh the HBM-traffic PMC passes behind profiles/pmc_traffic.json (one rocprofv3 run per
# counter, kernel trace only): the bench's k16 r4 encode + decode apply, k32 r8 encode, and
# configs[4]'s k64 r16 L9000 encode + decode apply.
# usage (GPU box): bash tools/pmc_refresh.sh TAG ; then locally:
#   python tools/pmc_summarize.py profiles/pmc_traffic.json \
#     rlc_encode_k16_r4=gpurun_out/TAG/k16:k_rlc_encode_bs<4:1048576 \
#     rlc_decode_apply_k16_e4=gpurun_out/TAG/k16:k_rlc_recover_bs<4:1048576 \
#     rlc_encode_k32_r8=gpurun_out/TAG/k32:k_rlc_encode_bs<8:1048576 \
#     rlc_encode_k64_r16_L9000=gpurun_out/TAG/k64e:k_rlc_encode_bs2<16:32768 \
#     rlc_decode_apply_k64_e16=gpurun_out/TAG/k64d:k_rlc_recover_bs2<16:32768
set -o pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/k16/$C -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu --no-legs > $OUT/k16_$C.log 2>&1 || { tail -5 $OUT/k16_$C.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/k32/$C -o run --output-format csv -- python tools/kernel_only.py enc 32 8 1048576 3 > $OUT/k32_$C.log 2>&1 || { tail -5 $OUT/k32_$C.log; exit 1; }
  FEC_L=9000 timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/k64e/$C -o run --output-format csv -- python tools/kernel_only.py enc 64 16 32768 3 > $OUT/k64e_$C.log 2>&1 || { tail -5 $OUT/k64e_$C.log; exit 1; }
  FEC_L=9000 timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/k64d/$C -o run --output-format csv -- python tools/kernel_only.py dec 64 16 32768 3 > $OUT/k64d_$C.log 2>&1 || { tail -5 $OUT/k64d_$C.log; exit 1; }
done
ls $OUT/k16/FETCH_SIZE $OUT/k32/WRITE_SIZE
