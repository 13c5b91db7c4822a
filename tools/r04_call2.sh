set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 100 tools/microbench/split_probe_k16 > gpurun_out/r04/split_probe_k16.log 2>&1 &&
timeout -k 10 100 tools/microbench/split_probe_k32 > gpurun_out/r04/split_probe_k32.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "decode_rows" tests/test_block_svc_gpu.py tests/test_batch_gpu.py > gpurun_out/r04/pytest_new.log 2>&1 &&
(timeout -k 10 120 python bench.py --gpus 2 --no-cpu > gpurun_out/r04/bench_gpus2.log 2>&1; echo "rc=$?" >> gpurun_out/r04/bench_gpus2.log)
