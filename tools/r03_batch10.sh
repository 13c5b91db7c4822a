#!/bin/bash
# XOR recover into rows of their own (fecgpu_xor_decode_to) vs in place, then the XOR parity tests
set -o pipefail
mkdir -p gpurun_out/r03t
timeout -k 10 300 python -u tools/xor_ab.py cur=pquic_amd/lib/libpquic_fec.so --cycles=9 > gpurun_out/r03t/xor_ab.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "xor" > gpurun_out/r03t/pytest_xor.log 2>&1
rc=$?; cat gpurun_out/r03t/xor_ab.log; tail -3 gpurun_out/r03t/pytest_xor.log; exit $rc
