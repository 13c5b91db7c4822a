#!/bin/bash
# batching adapter: engine-only gathered rate vs contiguous, and the saturated run's thread times
set -o pipefail
mkdir -p gpurun_out/r03m
timeout -k 10 300 python -u tools/rows_probe.py 3 > gpurun_out/r03m/rows_probe.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_batch_gpu.py > gpurun_out/r03m/pytest_batch.log 2>&1
rc=$?; tail -3 gpurun_out/r03m/pytest_batch.log; cat gpurun_out/r03m/rows_probe.log; exit $rc
