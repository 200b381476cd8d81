#!/usr/bin/env python3
"""Folds abtest/gather_probe.sh's runs into one table: per run the useful bytes per launch (from
the probe's own JSON line), the fabric read bytes from the TCC request mix (32 x n32 + 64 x n64 +
128 x n128), FETCH_SIZE raw and x2, the L2 hit rate and WRITE_SIZE, all per launch.

usage: probe_report.py <gpurun_out/probe>
"""
import csv
import glob
import json
import os
import sys


def counters(d):
    """{counter: mean per dispatch} over the probe kernel's dispatches (k_stream / k_gather)."""
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if not ("k_gather" in r["Kernel_Name"] or "k_stream" in r["Kernel_Name"]):
                continue
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    out = sys.argv[1]
    rows = []
    for j in sorted(glob.glob(os.path.join(out, "*.json"))):
        tag = os.path.basename(j)[:-5]
        line = json.loads(open(j).read().strip().splitlines()[-1])
        c = counters(os.path.join(out, f"p_{tag}"))
        useful = line.get("bytes_per_launch") or line.get("record_bytes_per_launch")
        n32, n64, n128 = (c.get(f"TCC_EA0_RDREQ_{s}B_sum", 0.0) for s in (32, 64, 128))
        mix = 32 * n32 + 64 * n64 + 128 * n128
        fetch = c.get("FETCH_SIZE", 0.0) * 1024
        hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        rows.append({
            "tag": tag, "ms": line["best_ms"], "useful_read_GB": round(useful / 1e9, 3),
            "useful_read_GBps": round(useful / (line["best_ms"] * 1e-3) / 1e9, 1),
            "req_mix_read_GB": round(mix / 1e9, 3), "req_mix_over_useful": round(mix / useful, 3) if useful else None,
            "rdreq": c.get("TCC_EA0_RDREQ_sum"), "n32": n32, "n64": n64, "n128": n128,
            "fetch_size_GB": round(fetch / 1e9, 3), "fetch_x2_over_useful": round(2 * fetch / useful, 3) if useful else None,
            "l2_hit_rate": round(hit / (hit + miss), 4) if hit + miss else None,
            "write_GB": round(c.get("WRITE_SIZE", 0.0) * 1024 / 1e9, 3),
            "store_GB": round(line.get("store_bytes_per_launch", 0) / 1e9, 3)})
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
