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
    # per (kernel, grid): average duration from the per-dispatch trace
    for f in sorted(glob.glob(os.path.join(d, "*kernel_trace.csv"))):
        print(f"== {os.path.basename(f)} (per kernel and grid size)")
        acc = defaultdict(list)
        for r in csv.DictReader(open(f)):
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            acc[(short(r["Kernel_Name"]), int(r["Grid_Size_X"]))].append(dur)
        for (k, g), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
            v.sort()
            print(f"  {k:55s} grid={g:>9} calls={len(v):>5} avg_us={sum(v)/len(v):8.2f} "
                  f"median_us={v[len(v)//2]:8.2f}")
    for f in sorted(glob.glob(os.path.join(d, "*kernel_stats.csv"))):
        print(f"== {os.path.basename(f)}")
        for r in csv.DictReader(open(f)):
            print(f"  {short(r['Name']):60s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:9.2f} "
                  f"pct={float(r['Percentage']):5.1f}")
    for f in sorted(glob.glob(os.path.join(d, "*counter_collection.csv"))):
        print(f"== {os.path.basename(f)}")
        acc = defaultdict(lambda: defaultdict(list))
        for r in csv.DictReader(open(f)):
            acc[(short(r["Kernel_Name"]), int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for (k, g), cs in sorted(acc.items()):
            vals = "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items()))
            print(f"  {k:50s} grid={g:>9} {vals}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
