#!/bin/bash
# XOR decode: two pieces per thread vs the previous build (in-process A/B), then the XOR parity tests
set -o pipefail
mkdir -p gpurun_out/r03o
timeout -k 10 300 python -u tools/xor_ab.py new=pquic_amd/lib/libpquic_fec.so old=pquic_amd/lib/variants/xold/libpquic_fec.so --cycles=7 > gpurun_out/r03o/xor_ab.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "xor or XOR" > gpurun_out/r03o/pytest_xor.log 2>&1
rc=$?; cat gpurun_out/r03o/xor_ab.log; tail -3 gpurun_out/r03o/pytest_xor.log; exit $rc
