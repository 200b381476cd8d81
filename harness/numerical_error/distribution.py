#!/usr/bin/env python3
"""Distribution of element-wise differences (port of numerical_error/distribution.py:17-42):
ALG1 vs ALG3, and ALG1 (fp32) vs an fp64 reference, as histograms."""
import argparse

import numpy as np

from common import gpu, savefig, uniform_csr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--density", type=float, default=0.1)
    ap.add_argument("--low", type=float, default=0.0)
    ap.add_argument("--high", type=float, default=1.0)
    args = ap.parse_args()
    rng = np.random.default_rng(1)
    A = uniform_csr(args.n, args.density, args.low, args.high, rng)
    B = uniform_csr(args.n, args.density, args.low, args.high, rng)
    c1 = gpu(A, B, 1).toarray()
    c3 = gpu(A, B, 3, 0.3).toarray()
    ref = (A.astype(np.float64) @ B.astype(np.float64)).toarray()
    d13 = (c1 - c3).ravel()
    d64 = (c1.astype(np.float64) - ref).ravel()
    print(f"alg1-alg3: nonzero diffs {np.count_nonzero(d13)} of {d13.size}")
    hist, edges = np.histogram(np.abs(d64[d64 != 0]) if np.any(d64) else [0.0], bins=10)
    print("alg1 - fp64 |error| histogram:")
    for h, e0, e1 in zip(hist, edges[:-1], edges[1:]):
        print(f"  [{e0:.3e}, {e1:.3e}) {h}")
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        plt.hist(d64, bins=100)
        plt.title("SpGEMM fp32 error vs fp64 reference")
        savefig("spgemm_error_distribution.png")
    except Exception as e:   # noqa: BLE001
        print(f"(plot skipped: {e})")


if __name__ == "__main__":
    main()
