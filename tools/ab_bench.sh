#!/bin/bash
# A/B the library variants built by tools/build_variants.py on one GPU box.
# usage: bash tools/ab_bench.sh TAG variant1 variant2 ...   ("main" = pquic_amd/lib/libpquic_fec.so)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in "$@"; do
  if [ "$v" = main ]; then lib=pquic_amd/lib/libpquic_fec.so; else lib=pquic_amd/lib/variants/$v/libpquic_fec.so; fi
  PQUIC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-pcie > $OUT/bench_$v.log 2>&1 || { tail $OUT/bench_$v.log; exit 1; }
  python - "$v" "$OUT/bench_$v.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
L = d["legs"]
print(f'{sys.argv[1]:10s} value={d["value"]:8.1f}  enc16={L["rlc_encode_k16_r4"]["ms"]:.3f}ms '
      f'plan={L["rlc_decode_k16_e4"]["plan_ms"]:.3f} apply={L["rlc_decode_k16_e4"]["apply_ms"]:.3f} '
      f'enc32={L["rlc_encode_k32_r8"]["ms"]:.3f}ms ({L["rlc_encode_k32_r8"]["algorithmic_GB_s"]} GB/s)')
PY
done
