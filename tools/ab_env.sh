#!/bin/bash
# A/B runtime knobs on one GPU box: each argument is NAME or NAME:VAR=VALUE[,VAR=VALUE] (env for that run).
# usage: bash tools/ab_env.sh TAG base tile82:FECGPU_ENC_TILE=8,2 ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for spec in "$@"; do
  name=${spec%%:*}; envs=""
  [ "$spec" != "$name" ] && envs=${spec#*:}
  ( [ -n "$envs" ] && export $(echo "$envs" | tr ";" " ") ; timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-pcie > $OUT/bench_$name.log 2>&1 ) || { tail $OUT/bench_$name.log; exit 1; }
  python - "$name" "$OUT/bench_$name.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
L = d["legs"]; c5 = L["rlc_k64_r16_L9000"]
print(f'{sys.argv[1]:10s} value={d["value"]:7.1f} enc16={L["rlc_encode_k16_r4"]["ms"]:.3f} '
      f'apply16={L["rlc_decode_k16_e4"]["apply_ms"]:.3f} enc32={L["rlc_encode_k32_r8"]["ms"]:.3f} '
      f'c5 enc={c5["encode_ms"]:.2f} plan={c5["plan_ms"]:.2f} apply={c5["apply_ms"]:.2f}')
PY
done
