# round 4: lock-free split encode -- parity, then in-process A/B against one wave per block
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "split" > gpurun_out/r04/pytest_split2.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_inproc.py "base:split=0" "sp2:split=2" "sp4:split=4" --cycles=5 --reps=5 > gpurun_out/r04/ab_split2.log 2>&1
