#!/bin/bash
# round 4: GPU suite on the current tree; the decode apply's access pattern in the trivial-compute
# probe; k32 r8 encode HBM traffic with the compact-map bodies back on default loads
set -o pipefail
mkdir -p gpurun_out/r04 gpurun_out/r04_pmc2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu_call15.log 2>&1 || exit 1
timeout -k 10 120 tools/microbench/split_probe_k16 dec > gpurun_out/r04/dec_probe_k16.log 2>&1 &&
timeout -k 10 120 tools/microbench/split_probe_k32 dec > gpurun_out/r04/dec_probe_k32.log 2>&1 || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/r04_pmc2/k32/$C -o run --output-format csv -- python tools/kernel_only.py enc 32 8 1048576 3 > gpurun_out/r04_pmc2/k32_$C.log 2>&1 || exit 1
done
