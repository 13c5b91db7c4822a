#!/bin/bash
# round 4: adjacent-block workgroups in the trivial-compute pattern probe (no reduction between waves)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 120 tools/microbench/split_probe_k32 adj > gpurun_out/r04/adj_probe_k32.log 2>&1 &&
timeout -k 10 120 tools/microbench/split_probe_k16 adj > gpurun_out/r04/adj_probe_k16.log 2>&1
