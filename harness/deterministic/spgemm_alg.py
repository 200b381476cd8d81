#!/usr/bin/env python3
"""Dump C = A @ B for a grid of sizes and densities (port of deterministic/cupy_alg{1,2,3}.py
:18-40).  Two runs in separate processes must write identical files.

Deliberate fixes: --seed is honoured (the reference seeds once at import and ignores the
flag, cupy_alg1.py:15,21), and arrays are written in full (str(cupy_array) elides the
middle above 1000 elements, so the reference compares heads and tails only): the file holds
nnz and a SHA-256 of the raw bytes of indices, indptr and data, plus the first values.
"""
import argparse
import hashlib
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from spmm_amd import cusparse  # noqa: E402
from spmm_amd.sparse import csr_matrix  # noqa: E402

MATRIX_SIZE = [32, 64, 128, 256, 512, 1024]
DENSITY = [0.01, 0.1, 0.3, 0.5]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--seed", type=int, default=2008)
    ap.add_argument("--dtype", default="float32", choices=["float32", "float64"])
    ap.add_argument("--alg", type=int, default=1, choices=[1, 2, 3])
    args = ap.parse_args()
    dt = np.float32 if args.dtype == "float32" else np.float64
    rng = np.random.default_rng(args.seed)
    with open(args.out, "w") as f:
        for n in MATRIX_SIZE:
            for d in DENSITY:
                A = sp.random(n, n, density=d, format="csr", dtype=dt, random_state=rng)
                B = sp.random(n, n, density=d, format="csr", dtype=dt, random_state=rng)
                C = cusparse.spgemm(csr_matrix(A, device="cuda"), csr_matrix(B, device="cuda"), alg=args.alg)
                h = hashlib.sha256()
                for t in (C.indices, C.indptr, C.data):
                    h.update(t.cpu().numpy().tobytes())
                f.write(f"{n} {d} nnz={C.nnz} sha256={h.hexdigest()}\n")
                f.write(str(C.data[:8].cpu().numpy()) + "\n\n")


if __name__ == "__main__":
    main()
