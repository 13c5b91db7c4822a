#!/bin/bash
# One GPU call as a chain of steps, each under its own time limit, each logging to its own file.
# The chain stops at the first failing step (a fault, abort, time limit or test failure): nothing
# after it touches the GPU.  Replaces the one-off per-call scripts of rounds 3-4.
# usage (through gpurun, from the repo root):
#   bash tools/gpu_steps.sh TAG "NAME SECONDS COMMAND..." ["NAME SECONDS COMMAND..." ...]
# e.g. bash tools/gpu_steps.sh r05a "pytest 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
#                                    "bench 300 python bench.py"
# Logs: gpurun_out/TAG/NAME.log; a step's exit status is appended to its log as "rc=N".
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  read -r name secs cmd <<<"$step"
  echo "[$(date +%T)] $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -o pipefail -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "rc=$rc" >> "$OUT/$name.log"
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then
    echo "step $name failed (rc=$rc): stopping"
    exit $rc
  fi
done
