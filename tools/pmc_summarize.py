"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM traffic.

gfx950 correction (/opt/skills/guides/MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7):
FETCH_SIZE counts 64 B per 128-B request of a wide (16 B/lane) coalesced read stream, i.e.
half the bytes, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Both are
in KiB.  usage: python tools/pmc_summarize.py OUT.json TAG=DIR:KERNEL_SUBSTR[:BLOCKS] ...
"""
import csv
import json
import os
import sys
from collections import defaultdict


def per_kernel(path):
    acc = defaultdict(list)
    for row in csv.DictReader(open(path)):
        acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return acc


def main():
    out = sys.argv[1]
    res = json.load(open(out)) if os.path.exists(out) else {}
    for spec in sys.argv[2:]:
        tag, rest = spec.split("=", 1)
        parts = rest.split(":")
        d, sub = parts[0], parts[1]
        blocks = int(parts[2]) if len(parts) > 2 else None
        f = per_kernel(os.path.join(d, "FETCH_SIZE", "run_counter_collection.csv"))
        w = per_kernel(os.path.join(d, "WRITE_SIZE", "run_counter_collection.csv"))
        names = [n for n in f if sub in n]
        if not names:
            raise SystemExit(f"no kernel matching {sub!r} in {d}")
        n = names[0]
        fk = sum(f[n]) / len(f[n])
        wk = sum(w[n]) / len(w[n]) if n in w else 0.0
        res[tag] = {"kernel": n, "launches": len(f[n]), "FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk,
                    "hbm_bytes_per_launch_raw": (fk + wk) * 1024,
                    "hbm_bytes_per_launch_corrected": (2 * fk + wk) * 1024,
                    "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE x1"}
        if blocks:
            res[tag]["blocks_per_launch"] = blocks
            res[tag]["hbm_bytes_per_block_corrected"] = (2 * fk + wk) * 1024 / blocks
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
