#!/usr/bin/env python3
"""Summarize rocprofv3 CSV output: per-kernel average duration (kernel trace) and per-kernel
average PMC counter values.  Usage: summarize.py <dir with *_kernel_trace.csv / *_counter_collection.csv>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    name = name.split("(")[0]
    return name.replace("void ", "").replace("spg::", "")


def main(d):
    for f in sorted(glob.glob(os.path.join(d, "*kernel_stats.csv"))):
        print(f"== {os.path.basename(f)}")
        for r in csv.DictReader(open(f)):
            print(f"  {short(r['Name']):60s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:9.2f} "
                  f"pct={float(r['Percentage']):5.1f}")
    for f in sorted(glob.glob(os.path.join(d, "*counter_collection.csv"))):
        print(f"== {os.path.basename(f)}")
        acc = defaultdict(lambda: defaultdict(list))
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in acc.items():
            vals = "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items()))
            print(f"  {k:50s} {vals}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
