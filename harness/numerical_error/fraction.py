#!/usr/bin/env python3
"""ALG3 chunk_fraction sweep: does the chunking change the result? (port of
numerical_error/fraction.py:18-38).  Deliberate fix: the reference sets density = 0.
(fraction.py:8), so its matrices are empty; here density = 0.1."""
import numpy as np

from common import gpu, uniform_csr

n, density = 1024, 0.1
fractions = [0.01, 0.05, 0.1, 0.2, 0.3, 0.5, 0.8, 1.0]


def main():
    rng = np.random.default_rng(3)
    A = uniform_csr(n, density, 0, 1, rng)
    B = uniform_csr(n, density, 0, 1, rng)
    ref = gpu(A, B, 1).toarray()
    print(f"{'chunk_fraction':>14} {'max|alg3-alg1|':>15}")
    for cf in fractions:
        d = np.abs(gpu(A, B, 3, cf).toarray() - ref).max()
        print(f"{cf:14g} {d:15.3e}")


if __name__ == "__main__":
    main()
