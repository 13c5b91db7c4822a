"""Per-block SQ figures from tools/pmc_sq.sh passes (rocprofv3 --pmc, one counter group per run).
SQ cycle counters count in quad-cycles (one issued wave-instruction = one); ACTIVE_INST_ANY,
WAIT_INST_ANY and WAIT_ANY split a wave's lifetime (WAVE_CYCLES).  SIMD VALU utilisation assumes a
wave64 VALU instruction occupies its SIMD-32 for 2 cycles (MI355X_MICROARCH.md) over GRBM_GUI_ACTIVE
cycles (summed over the 8 XCDs) x 4 SIMDs x 32 CUs.
usage: python tools/sq_summary.py DIR BLOCKS [label]   (DIR holds p1/ p2/ p3/ run_counter_collection.csv)"""
import csv
import glob
import sys
from collections import defaultdict

d, blocks = sys.argv[1], int(sys.argv[2])
label = sys.argv[3] if len(sys.argv) > 3 else d
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(d + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_rlc" not in k:
            continue
        acc[k.split("(")[0].replace("void ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    c = {n: sum(v) / len(v) for n, v in cs.items()}
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    grbm = c.get("GRBM_GUI_ACTIVE", 0)
    simd_cycles = grbm / 8 * 1024 if grbm else 0
    print(f"{label}: {k}")
    print(f"  per block: VALU {c.get('SQ_INSTS_VALU', 0) / blocks:8.0f}  SALU {c.get('SQ_INSTS_SALU', 0) / blocks:8.0f}  "
          f"LDS {c.get('SQ_INSTS_LDS', 0) / blocks:6.1f}  VMEM rd {c.get('SQ_INSTS_VMEM_RD', 0) / blocks:6.1f}  "
          f"wr {c.get('SQ_INSTS_VMEM_WR', 0) / blocks:6.1f}   waves {c.get('SQ_WAVES', 0):.0f}")
    print(f"  wave time: issuing {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.1%}  issue-stalled (WAIT_INST_ANY) "
          f"{c.get('SQ_WAIT_INST_ANY', 0) / wc:5.1%}  waiting on counters/barriers (WAIT_ANY) {c.get('SQ_WAIT_ANY', 0) / wc:5.1%}")
    if simd_cycles:
        print(f"  SIMD VALU utilisation {2 * c.get('SQ_INSTS_VALU', 0) / simd_cycles:5.1%}   "
              f"kernel cycles per XCD {grbm / 8:.3g}")
