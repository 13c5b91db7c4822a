# round 4: split encode parity, then the GPU suite, then the in-process A/B of split vs one wave per block
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "split or decode_rows" > gpurun_out/r04/pytest_split.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r04/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_inproc.py "base:split=0" "sp2:split=2" "sp4:split=4" --cycles=5 --reps=5 > gpurun_out/r04/ab_split.log 2>&1 &&
(timeout -k 10 120 python bench.py --gpus 2 --no-cpu > gpurun_out/r04/bench_gpus2.log 2>&1; echo "rc=$?" >> gpurun_out/r04/bench_gpus2.log)
