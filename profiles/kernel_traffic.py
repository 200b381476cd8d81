#!/usr/bin/env python3
"""Per-kernel fabric traffic of one profiles/collect.sh directory: FETCH_SIZE x 2 (read),
WRITE_SIZE (written) and the L2 hit rate TCC_HIT / (TCC_HIT + TCC_MISS), averaged over each
kernel's dispatches.  usage: kernel_traffic.py <prof dir> [name filter ...]"""
import csv
import os
import sys
from collections import defaultdict


def main(d, filt):
    acc = defaultdict(lambda: defaultdict(list))
    for f in ("pmc_fetch", "pmc_write", "pmc_hit"):
        path = os.path.join(d, f + "_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            acc[r["Kernel_Name"].split("(")[0].replace("void ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        if filt and not any(x in k for x in filt):
            continue
        avg = {c: sum(x) / len(x) for c, x in v.items()}
        rd, wr = avg.get("FETCH_SIZE", 0) * 2 * 1024 / 1e9, avg.get("WRITE_SIZE", 0) * 1024 / 1e9
        h, m = avg.get("TCC_HIT_sum", 0), avg.get("TCC_MISS_sum", 0)
        print(f"{k:50s} read {rd:9.3f} GB  written {wr:9.3f} GB  L2 hit {h / (h + m) if h + m else 0:.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
