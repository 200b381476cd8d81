"""Loader for the committed golden vectors (plain .npz arrays, allow_pickle=False)."""
import glob
import os

import numpy as np
import scipy.sparse as sp

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def case_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


def load(name):
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)

    def mat(p):
        return sp.csr_matrix((z[p + "_data"], z[p + "_indices"], z[p + "_indptr"]),
                             shape=tuple(int(s) for s in z[p + "_shape"]))
    return mat("A"), mat("B"), mat("C"), float(z["alpha"])


SPMV_DIR = os.path.join(GOLDEN_DIR, "spmv")


def spmv_case_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(SPMV_DIR, "*.npz")))


def load_spmv(name):
    """(A csr, x, y, alpha) of an SpMV fixture: y = alpha * (A @ x) from scipy."""
    z = np.load(os.path.join(SPMV_DIR, name + ".npz"), allow_pickle=False)
    A = sp.csr_matrix((z["A_data"], z["A_indices"], z["A_indptr"]),
                      shape=tuple(int(s) for s in z["A_shape"]))
    return A, z["x"], z["y"], float(z["alpha"])
