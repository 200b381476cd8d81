#!/usr/bin/env python3
"""Worst-case error vs value range [0, high] (port of numerical_error/range.py:18-61)."""
import argparse

import numpy as np

from common import errors, uniform_csr

high_values = [1, 10, 100, 500, 1000, 5000, 10000]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--density", type=float, default=0.1)
    ap.add_argument("--repeat", type=int, default=5, help="reference: 300")
    args = ap.parse_args()
    rng = np.random.default_rng(0)
    print(f"{'high':>7} {'max|alg1-alg3|':>15} {'max|alg1-fp64|':>15} {'max ulp':>8}")
    for high in high_values:
        worst = (0.0, 0.0, 0)
        for _ in range(args.repeat):
            A = uniform_csr(args.n, args.density, 0, high, rng)
            B = uniform_csr(args.n, args.density, 0, high, rng)
            e = errors(A, B, cf=0.3)
            worst = tuple(max(a, b) for a, b in zip(worst, e))
        print(f"{high:7d} {worst[0]:15.3e} {worst[1]:15.3e} {worst[2]:8d}")


if __name__ == "__main__":
    main()
