"""Summarise a rocprofv3 --kernel-trace CSV per (kernel, grid size): dispatches, mean / min
duration, VGPRs, LDS.  The bench mixes its big legs with thousands of one-block launches (hook
latency, batching), so per-kernel averages of --stats alone mislead; grid size separates them.
usage: python tools/trace_summary.py run_kernel_trace.csv > summary.txt"""
import csv
import re
import sys
from collections import defaultdict

rows = defaultdict(list)
meta = {}
for r in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
    key = (name, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
    rows[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    meta[key] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"])
print(f"# {sys.argv[1]}: per (kernel, grid threads, workgroup) -- durations in microseconds")
print(f"{'kernel':34s} {'grid':>10s} {'wg':>4s} {'calls':>6s} {'mean_us':>10s} {'min_us':>10s} {'vgpr':>5s} "
      f"{'agpr':>5s} {'sgpr':>5s} {'lds':>6s}")
for key in sorted(rows, key=lambda k: -sum(rows[k])):
    v = rows[key]
    m = meta[key]
    print(f"{key[0]:34s} {key[1]:10d} {key[2]:4d} {len(v):6d} {sum(v) / len(v):10.1f} {min(v):10.1f} {m[0]:>5s} "
          f"{m[1]:>5s} {m[2]:>5s} {m[3]:>6s}")
