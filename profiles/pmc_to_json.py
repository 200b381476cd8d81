#!/usr/bin/env python3
"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_traffic.json.

HBM-side bytes per launch of one kernel (the bench's dominant kernel), following
MI355X_MICROARCH.md "HBM [CDNA4]":
  read  = FETCH_SIZE (KiB) x 1024 x 2   (gfx950 tallies 128-B requests at 64 B)
  write = WRITE_SIZE (KiB) x 1024
FETCH_SIZE counts L2 misses to the fabric, Infinity-Cache hits included, so for inputs that
stay resident in the 256 MiB Infinity Cache it is an upper bound on HBM reads.  The x2
correction holds for the tile kernels' gathers as well (round 4 calibration,
abtest/gather_probe.sh: every fabric read request is 128 B).  A third pass adds the L2 hit rate.

Each entry is stamped with the build id of the library it was measured on
(spmm_amd._lib.build_id(): SHA-256 of libmi355_spgemm.so); bench.py reports a traffic figure
only when the stamp matches the library it runs.

usage: pmc_to_json.py <dir> <key> <kernel regex> [json path]
"""
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def per_launch(d, counter, rx):
    """Average over the matching dispatches with the LARGEST grid (the full product; ALG3's
    row chunks launch the same kernel on smaller grids)."""
    rows = []
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and rx.search(r["Kernel_Name"]):
                rows.append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    if not rows:
        return None, 0
    g = max(x[0] for x in rows)
    vals = [v for gs, v in rows if gs == g]
    return sum(vals) / len(vals), len(vals)


def main():
    from spmm_amd._lib import build_id, source_id
    d, key, pat = sys.argv[1], sys.argv[2], sys.argv[3]
    path = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(__file__), "pmc_traffic.json")
    rx = re.compile(pat)
    fetch, nf = per_launch(d, "FETCH_SIZE", rx)
    write, nw = per_launch(d, "WRITE_SIZE", rx)
    if fetch is None or write is None:
        raise SystemExit(f"no FETCH_SIZE/WRITE_SIZE rows for /{pat}/ under {d}")
    hit, _ = per_launch(d, "TCC_HIT_sum", rx)
    miss, _ = per_launch(d, "TCC_MISS_sum", rx)
    rd = fetch * 1024 * 2
    wr = write * 1024
    db = json.load(open(path)) if os.path.exists(path) else {}
    db[key] = {"kernel_regex": pat, "dispatches": [nf, nw],
               "fetch_size_kib": round(fetch, 1), "write_size_kib": round(write, 1),
               "read_bytes_per_launch": int(rd), "write_bytes_per_launch": int(wr),
               "hbm_bytes_per_launch": int(rd + wr),
               "l2_hit_rate": round(hit / (hit + miss), 4) if hit is not None and miss is not None and hit + miss else None,
               "note": ("FETCH_SIZE x2 + WRITE_SIZE; Infinity-Cache hits included.  The x2 is exact for these "
                        "gathers too: every fabric read request of the 12-/10-byte record gathers is a 128-byte "
                        "request tallied at 64 B (TCC_EA0_RDREQ_128B_sum = TCC_EA0_RDREQ_sum, "
                        "abtest/gather_probe.sh, profiles/r04_gather_probe.txt)"),
               "build_id": build_id(), "source_id": source_id()}
    json.dump(db, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps({key: db[key]}))


if __name__ == "__main__":
    main()
