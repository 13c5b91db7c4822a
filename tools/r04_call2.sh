# round 4: split-pattern probes, the GPU suite, the launcher's refusal on a 1-GPU box
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 100 tools/microbench/split_probe_k16 > gpurun_out/r04/split_probe_k16.log 2>&1 &&
timeout -k 10 100 tools/microbench/split_probe_k32 > gpurun_out/r04/split_probe_k32.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r04/pytest_gpu.log 2>&1 &&
(timeout -k 10 120 python bench.py --gpus 2 --no-cpu > gpurun_out/r04/bench_gpus2.log 2>&1; echo "rc=$?" >> gpurun_out/r04/bench_gpus2.log)
