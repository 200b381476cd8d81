#!/usr/bin/env python3
"""Max |ALG1 - ALG3| heatmap over size x density (port of numerical_error/error.py:16-48),
plus the error against an fp64 reference and the ULP distance to scipy fp32."""
import numpy as np

from common import errors, savefig, uniform_csr

matrix_size = [256, 512, 1024]
density = [0.01, 0.1, 0.5]


def main():
    rng = np.random.default_rng(10)
    err = np.zeros((len(matrix_size), len(density)))
    print(f"{'n':>6} {'density':>8} {'|alg1-alg3|':>12} {'|alg1-fp64|':>12} {'ulp vs scipy':>12}")
    for i, n in enumerate(matrix_size):
        for j, d in enumerate(density):
            A = uniform_csr(n, d, 0, 1, rng)
            B = uniform_csr(n, d, 0, 1, rng)
            d13, e64, ulp = errors(A, B, cf=0.3)
            err[i, j] = d13
            print(f"{n:6d} {d:8g} {d13:12.3e} {e64:12.3e} {ulp:12d}")
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        plt.figure(figsize=(8, 6))
        plt.imshow(err, origin="lower", aspect="auto")
        plt.colorbar(label="Max error")
        plt.xticks(range(len(density)), density)
        plt.yticks(range(len(matrix_size)), matrix_size)
        plt.xlabel("Density"); plt.ylabel("Matrix size")
        plt.title("SpGEMM max error heatmap (alg1 vs alg3) chunk_fraction: 0.3")
        for i in range(len(matrix_size)):
            for j in range(len(density)):
                plt.text(j, i, f"{err[i, j]:.2e}", ha="center", va="center")
        savefig("spgemm_error_heapmap.png")
    except Exception as e:   # noqa: BLE001
        print(f"(plot skipped: {e})")


if __name__ == "__main__":
    main()
