#!/bin/bash
# Routine GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats.
# usage (from the repo root, through gpurun): bash tools/gpu_check.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "pytest_rc=$?" >> $OUT/pytest_gpu.log
tail -3 $OUT/pytest_gpu.log
grep -q "pytest_rc=0" $OUT/pytest_gpu.log || exit 1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python bench.py "$@" > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
# the headline workload again under rocprofv3 (kernel trace only, no side legs): its own bench line
# (bench_prof.log) and the kernel statistics come from the same process and the same launches
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-legs --no-cpu > $OUT/bench_prof.log 2>&1 || { tail $OUT/bench_prof.log; exit 1; }
grep '^{' $OUT/bench_prof.log | tail -1 | cut -c1-200
python - "$OUT/prof/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r["Percentage"]) > 0.3:
        print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>4s} avg_us={float(r["AverageNs"])/1e3:9.1f} pct={float(r["Percentage"]):5.1f}')
PY
