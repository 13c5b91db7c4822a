#!/bin/bash
# One GPU pass for the 64-bit-shift transpose (T64) and pack-before-shift chain tail (HH) variants:
# VALU issue probe, parity tests on each variant library, in-process A/B against the main build.
mkdir -p gpurun_out/t64
timeout -k 10 120 tools/microbench/valu_issue_probe > gpurun_out/t64/valu_issue.log 2>&1 && \
PQUIC_AMD_LIB=$PWD/pquic_amd/lib/variants/t64/libpquic_fec.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t64/pytest_t64.log 2>&1 && \
PQUIC_AMD_LIB=$PWD/pquic_amd/lib/variants/t64hh/libpquic_fec.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t64/pytest_t64hh.log 2>&1 && \
timeout -k 10 500 python -u tools/ab_inproc.py base "t64:LIB=pquic_amd/lib/variants/t64/libpquic_fec.so" "t64hh:LIB=pquic_amd/lib/variants/t64hh/libpquic_fec.so" --wide --cycles=5 > gpurun_out/t64/ab.log 2>&1
rc=$?; cat gpurun_out/t64/valu_issue.log; tail -3 gpurun_out/t64/pytest_*.log; cat gpurun_out/t64/ab.log; exit $rc
