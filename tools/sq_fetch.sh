#!/bin/bash
# Instruction-fetch / LDS-wait counter passes (one rocprofv3 run per group, kernel trace only)
# over tools/kernel_only.py.  usage (GPU box): bash tools/sq_fetch.sh TAG MODE K R BLOCKS [L]
set -o pipefail
TAG=$1; MODE=$2; K=$3; R=$4; NB=$5; L=${6:-1200}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS" \
         "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ" \
         "SQ_WAVES SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  FEC_L=$L timeout -k 10 240 rocprofv3 --pmc $G -d $OUT/p$i -o run --output-format csv -- python tools/kernel_only.py $MODE $K $R $NB 2 > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
python - $OUT $NB <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_rlc_encode_bs" in r["Kernel_Name"] or "k_rlc_recover_bs" in r["Kernel_Name"]:
            acc[(r["Kernel_Name"][:34], r["Counter_Name"])].append(float(r["Counter_Value"]))
nb = float(sys.argv[2])
for (k, c), v in sorted(acc.items()):
    m = sum(v) / len(v)
    print(f"{k:34s} {c:28s} {m:16.4g}  per block {m / nb:12.4g}")
PY
