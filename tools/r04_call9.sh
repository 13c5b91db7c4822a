#!/bin/bash
# round 4: adjacent-block pattern probe; hooks under a bulk job in a bench-shaped process, with the
# block-service worker on a greatest-priority stream (this tree) and on a default one (variants/spill)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 120 tools/microbench/split_probe_k32 adj > gpurun_out/r04/adj_probe_k32.log 2>&1 &&
timeout -k 10 120 tools/microbench/split_probe_k16 adj > gpurun_out/r04/adj_probe_k16.log 2>&1 &&
timeout -k 10 240 python -u -m pytest tests/test_block_svc_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_svc.log 2>&1 &&
timeout -k 10 180 python -u tools/hook_load_probe.py > gpurun_out/r04/hook_load_prio.log 2>&1 &&
LD_LIBRARY_PATH=$PWD/pquic_amd/lib/variants/spill timeout -k 10 180 python -u tools/hook_load_probe.py pquic_amd/lib/variants/spill/libpquic_fec.so > gpurun_out/r04/hook_load_default_stream.log 2>&1
