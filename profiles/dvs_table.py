#!/usr/bin/env python3
"""Compact table of a dense_vs_sparseGEMM run (harness/dense_vs_sparseGEMM/run.sh output):
per (N, density) the sparse and dense times and their ratio, and per N the break-even density
(the smallest swept density where the sparse product is slower than the dense GEMM; linear in
log-density between the two sweep points that bracket ratio 1).
usage: dvs_table.py <results.txt> [older results.txt to put beside it]"""
import math
import re
import sys


def parse(path):
    out, cur = {}, None
    for ln in open(path):
        m = re.match(r"size = (\d+), density = ([\d.e-]+)", ln) or \
            re.match(r"A / B shape \(CSR\) : A=\((\d+), \d+\).*target_density=([\d.e-]+)", ln)
        if m:
            cur = (int(m.group(1)), float(m.group(2)))
            continue
        m = re.match(r"A @ B \[(sparse|dense), inputs_on_gpu\]\s+([\d.]+)\s+([\d.]+ \S+)", ln)
        if m and cur:
            out.setdefault(cur, {})[m.group(1)] = (float(m.group(2)), m.group(3))
    return out


def main():
    new = parse(sys.argv[1])
    old = parse(sys.argv[2]) if len(sys.argv) > 2 else {}
    print(f"{'N':>6} {'density':>8} {'sparse ms':>10} {'dense ms':>9} {'sparse/dense':>12} {'sparse dPeak':>13}"
          + (f" {'older sparse ms':>15}" if old else ""))
    by_n = {}
    for (n, d), r in sorted(new.items()):
        if "sparse" not in r or "dense" not in r:
            continue
        ratio = r["sparse"][0] / r["dense"][0]
        by_n.setdefault(n, []).append((d, ratio))
        o = old.get((n, d), {}).get("sparse")
        print(f"{n:6d} {d:8g} {r['sparse'][0]:10.3f} {r['dense'][0]:9.3f} {ratio:12.3f} {r['sparse'][1]:>13}"
              + (f" {o[0]:15.3f}" if o else (" " * 16 if old else "")))
    print()
    for n, pts in sorted(by_n.items()):
        be = None
        for (d0, r0), (d1, r1) in reversed(list(zip(pts, pts[1:]))):   # the last upward crossing
            if r0 < 1.0 <= r1:
                t = (0.0 - math.log(r0)) / (math.log(r1) - math.log(r0))
                be = math.exp(math.log(d0) + t * (math.log(d1) - math.log(d0)))
                break
        if be is None:
            be = "beyond the sweep (sparse faster everywhere)" if all(r < 1 for _, r in pts) else \
                 "below the sweep (dense faster everywhere)"
            print(f"N={n}: break-even density vs dense GEMM: {be}")
        else:
            print(f"N={n}: break-even density vs dense GEMM ~ {be:.3g} (log-linear between sweep points)")


if __name__ == "__main__":
    main()
