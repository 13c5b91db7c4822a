#!/bin/bash
# round 4, final kernels: SQ counter passes (one --pmc group per run) on the k16 r4 encode and k16 e4
# decode (nt symbol loads), k32 r8 encode, configs[4] encode / decode
set -o pipefail
mkdir -p gpurun_out/r04_sq_final
export TMPDIR=/tmp
bash tools/pmc_sq.sh r04_sq_final/enc_k16_r4 enc 16 4 1048576 3 > gpurun_out/r04_sq_final/enc_k16_r4.txt 2>&1 &&
bash tools/pmc_sq.sh r04_sq_final/dec_k16_e4 dec 16 4 1048576 3 > gpurun_out/r04_sq_final/dec_k16_e4.txt 2>&1 &&
bash tools/pmc_sq.sh r04_sq_final/enc_k32_r8 enc 32 8 1048576 3 > gpurun_out/r04_sq_final/enc_k32_r8.txt 2>&1 &&
FEC_L=9000 bash tools/pmc_sq.sh r04_sq_final/dec_k64_e16 dec 64 16 65536 3 > gpurun_out/r04_sq_final/dec_k64_e16_L9000.txt 2>&1
