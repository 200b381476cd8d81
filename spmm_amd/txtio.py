"""Text CSR format of the reference's parity pipeline (cupy_cusparse/).

``<prefix>_indptr.txt`` / ``_indices.txt`` / ``_data.txt``, one value per line: integers
with %d, fp32 data with %.9g (gen_and_save_alg1_txt.py:9-14; the C++ side reads data as
double then narrows to float and writes 9 significant digits, spgemm_from_txt_alg1.cu:
19-78).  fp64 data is written with %.17g (round-trip exact).
"""
from __future__ import annotations

import numpy as np


def save_csr_txt(prefix: str, indptr, indices, data) -> None:
    indptr = np.asarray(indptr).astype(np.int32, copy=False)
    indices = np.asarray(indices).astype(np.int32, copy=False)
    data = np.asarray(data)
    np.savetxt(prefix + "_indptr.txt", indptr, fmt="%d")
    np.savetxt(prefix + "_indices.txt", indices, fmt="%d")
    np.savetxt(prefix + "_data.txt", data, fmt="%.9g" if data.dtype == np.float32 else "%.17g")


def load_csr_txt(prefix: str, dtype=np.float32):
    """(rows, nnz, indptr, indices, data) as compare_csrs_txt.py:5-17 reads them."""
    indptr = np.loadtxt(prefix + "_indptr.txt", dtype=np.int32, ndmin=1)
    indices = np.loadtxt(prefix + "_indices.txt", dtype=np.int32, ndmin=1)
    data = np.loadtxt(prefix + "_data.txt", dtype=dtype, ndmin=1)
    return indptr.size - 1, indices.size, indptr, indices, data
