#!/usr/bin/env python3
"""Compare two text CSR results bit for bit (port of cupy_cusparse/compare_csrs_txt.py:20-47):
rows and nnz, indptr, indices, and data (fp32 bitwise).  Prints EQUAL / NOT EQUAL, exit 0/1."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from spmm_amd.txtio import load_csr_txt  # noqa: E402


def main(py_prefix, cu_prefix, dtype="float32"):
    dt = np.float32 if dtype == "float32" else np.float64
    r1, n1, p1, i1, d1 = load_csr_txt(py_prefix, dt)
    r2, n2, p2, i2, d2 = load_csr_txt(cu_prefix, dt)
    ok = True
    if r1 != r2 or n1 != n2:
        print(f"rows/nnz mismatch: py=({r1},{n1}) cu=({r2},{n2})")
        ok = False
    if not np.array_equal(p1, p2):
        print("indptr mismatch")
        ok = False
    if not np.array_equal(i1, i2):
        print("indices mismatch")
        ok = False
    if d1.shape != d2.shape or not np.array_equal(d1.view(np.uint8), d2.view(np.uint8)):
        print("data mismatch")
        ok = False
    print("EQUAL" if ok else "NOT EQUAL")
    return 0 if ok else 1


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("py_prefix")
    ap.add_argument("cu_prefix")
    ap.add_argument("--dtype", default="float32", choices=["float32", "float64"])
    a = ap.parse_args()
    raise SystemExit(main(a.py_prefix, a.cu_prefix, a.dtype))
