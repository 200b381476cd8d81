"""Shared pieces of the numerical_error ports (numerical_error/*.py).

The reference measures max |ALG1 - ALG3| of cuSPARSE results as dense arrays and plots it.
Here every algorithm accumulates in the same fixed order, so ALG1 - ALG3 is identically 0;
the scripts therefore also report the error against an fp64 scipy reference (the measure
of accuracy that stays informative), and the ULP distance to scipy's own fp32 result.
Plots are written when matplotlib is importable, text tables always.
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from spmm_amd import cusparse  # noqa: E402
from spmm_amd.sparse import csr_matrix  # noqa: E402


def uniform_csr(n, density, low, high, rng):
    M = sp.random(n, n, density=density, format="csr", dtype=np.float32, random_state=rng,
                  data_rvs=lambda k: rng.uniform(low, high, size=k).astype(np.float32))
    M.sort_indices()
    return M


def gpu(A, B, alg, cf=0.2):
    C = cusparse.spgemm(csr_matrix(A, device="cuda"), csr_matrix(B, device="cuda"), alg=alg,
                        chunk_fraction=cf)
    return C.get()


def errors(A, B, cf=0.3):
    """(max|ALG1-ALG3|, max|ALG1 - fp64 ref|, max ULP distance ALG1 vs scipy fp32)."""
    c1 = gpu(A, B, 1)
    c3 = gpu(A, B, 3, cf)
    d13 = np.abs(c1.toarray() - c3.toarray()).max() if c1.shape[0] else 0.0
    ref64 = (A.astype(np.float64) @ B.astype(np.float64)).toarray()
    e64 = np.abs(c1.toarray().astype(np.float64) - ref64).max() if c1.shape[0] else 0.0
    s32 = (A @ B).toarray()
    g32 = c1.toarray()
    ulp = np.abs(g32.view(np.int32).astype(np.int64) - s32.view(np.int32).astype(np.int64)).max() \
        if g32.size else 0
    return float(d13), float(e64), int(ulp)


def savefig(name):
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        plt.savefig(name, dpi=150, bbox_inches="tight")
        plt.close()
        print(f"Saved: {name}")
    except Exception as e:   # noqa: BLE001
        print(f"(plot skipped: {e})")
