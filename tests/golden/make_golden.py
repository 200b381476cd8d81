#!/usr/bin/env python3
"""Generate the golden SpGEMM vectors in tests/golden/ (run in the build container).

The truth is scipy.sparse 1.15.3 ``csr_matrix @ csr_matrix`` / ``.dot`` -- the CPU
comparator the reference itself times (SpGEMM_vs_SpMV/profiler.py:408) and the expectation
its upstream tests assert against (modify_src/cupy-src/tests/cupyx_tests/test_cusparse.py:
405-411; .../scipy_tests/sparse_tests/test_csr.py:631-635, 815-819).  cuSPARSE (the
reference's GPU engine) is closed-source and not present, so scipy's outputs are the
vectors the oracle is pinned to.

Each case is an ``.npz`` of plain arrays (no pickles): A_*/B_* inputs, C_* = scipy's raw
output (its own linked-list column order, zeros dropped), plus ``alpha``.  The fixture
inputs of the upstream CSR tests (test_csr.py:25-134) are reproduced as data.
"""
import json
import zlib
import os

import numpy as np
import scipy
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))


def save(name, A, B, alpha=1.0, note=""):
    A = sp.csr_matrix(A)
    B = sp.csr_matrix(B)
    C = (A @ B)
    if alpha != 1.0:
        C = C * A.dtype.type(alpha)
    C = sp.csr_matrix(C)
    np.savez_compressed(
        os.path.join(HERE, name + ".npz"),
        A_shape=np.array(A.shape, np.int64), A_indptr=A.indptr.astype(np.int64),
        A_indices=A.indices.astype(np.int32), A_data=A.data,
        B_shape=np.array(B.shape, np.int64), B_indptr=B.indptr.astype(np.int64),
        B_indices=B.indices.astype(np.int32), B_data=B.data,
        C_shape=np.array(C.shape, np.int64), C_indptr=C.indptr.astype(np.int64),
        C_indices=C.indices.astype(np.int32), C_data=C.data,
        alpha=np.array(alpha, np.float64))
    return {"name": name, "A": list(A.shape), "B": list(B.shape), "nnzA": int(A.nnz),
            "nnzB": int(B.nnz), "nnzC_scipy": int(C.nnz), "dtype": str(A.dtype),
            "alpha": alpha, "note": note}


# upstream CSR fixtures (modify_src/cupy-src/tests/cupyx_tests/scipy_tests/sparse_tests/
# test_csr.py:25-134), as data.
def fx(data, indices, indptr, shape, dt):
    return sp.csr_matrix((np.array(data, dt), np.array(indices, np.int32),
                          np.array(indptr, np.int32)), shape=shape)


FIXTURES = {
    "make": ([0, 1, 2, 3], [0, 1, 3, 2], [0, 2, 3, 4], (3, 4)),          # :25-32 (explicit 0)
    "make2": ([1, 2, 3, 4], [2, 1, 2, 2], [0, 1, 3, 4], (3, 4)),         # :47-54
    "make4": ([1, 2, 3, 4, 5, 6, 7, 8, 9], [0, 2, 3, 0, 1, 3, 0, 1, 2],
              [0, 3, 6, 9], (3, 4)),                                      # :67-74
    "make_unordered": ([1, 2, 3, 4], [1, 0, 1, 2], [0, 2, 3, 4], (3, 4)),  # :77-84
    "make_duplicate": ([0, 1, 3, 2, 4, 5], [0, 0, 0, 2, 0, 2], [0, 3, 6, 6], (3, 4)),  # :87-94
    "make_empty": ([], [], [0, 0, 0, 0], (3, 4)),                         # :97-100
    "make_shape": ([], [], [0, 0, 0, 0], (3, 4)),                         # :133-134
}
MAKE3 = ([1, 2, 3, 4, 5], [0, 2, 1, 0, 2], [0, 1, 3, 3, 5], (4, 3))        # :57-64


def rand(m, n, density, rng, dt, rvs=None):
    M = sp.random(m, n, density=density, format="csr", dtype=dt, random_state=rng,
                  data_rvs=rvs)
    M.sort_indices()
    return M


def make_spmv():
    """SpMV fixtures (csr_matrix @ dense vector, SpGEMM_vs_SpMV/profiler.py:410-411):
    A, x, y = alpha * (A @ x) from scipy, one directory of their own."""
    d = os.path.join(HERE, "spmv")
    os.makedirs(d, exist_ok=True)
    out = []
    specs = [("n1024_d0.01_f64", 1024, 1024, 0.01, np.float64, 1.0),
             ("rect_300x900_f32", 300, 900, 0.02, np.float32, -1.5),
             ("n700_d0.03_c128", 700, 700, 0.03, np.complex128, 0.5),
             ("rect_200x500_c64", 200, 500, 0.05, np.complex64, 1.0),
             ("emptyrows_64x64_f64", 64, 64, 0.05, np.float64, 1.0)]
    for name, m, n, dens, dt, alpha in specs:
        rng = np.random.default_rng(zlib.crc32(name.encode()))
        A = sp.random(m, n, density=dens, format="csr", random_state=rng, dtype=np.float64)
        A.data = rng.standard_normal(A.nnz)
        x = rng.standard_normal(n)
        if np.dtype(dt).kind == "c":
            A.data = A.data + 1j * rng.standard_normal(A.nnz)
            x = x + 1j * rng.standard_normal(n)
        if name.startswith("emptyrows"):
            A = A.tolil(); A[::3, :] = 0; A = sp.csr_matrix(A); A.eliminate_zeros()
        A = A.astype(dt); A.sort_indices()
        x = x.astype(dt)
        y = A @ x
        if alpha != 1.0:
            y = y * np.dtype(dt).type(alpha)
        np.savez_compressed(os.path.join(d, name + ".npz"), A_shape=np.array(A.shape, np.int64),
                            A_indptr=A.indptr.astype(np.int64), A_indices=A.indices.astype(np.int32),
                            A_data=A.data, x=x, y=y, alpha=np.array(alpha, np.float64))
        out.append({"name": name, "A": list(A.shape), "nnzA": int(A.nnz), "dtype": str(np.dtype(dt)),
                    "alpha": alpha})
    return out


def main():
    cases = []
    for dt in (np.float32, np.float64):
        tag = "f32" if dt == np.float32 else "f64"
        x = fx(*MAKE3, dt)
        for name, spec in FIXTURES.items():
            cases.append(save(f"fixture_{name}_{tag}", fx(*spec, dt), x,
                              note="upstream test_csr.py m.dot(_make3)"))
        # upstream TestSpgemm shapes (test_cusparse.py:372-411): density 0.5, alpha 0.5
        for (m, n, k) in [(2, 3, 4), (4, 3, 2)]:
            rng = np.random.default_rng(1000 + m)
            a = rand(m, k, 0.5, rng, dt)
            b = rand(k, n, 0.5, rng, dt)
            cases.append(save(f"testspgemm_{m}x{n}x{k}_{tag}", a, b, alpha=0.5,
                              note="upstream TestSpgemm, alpha=0.5"))

    # config 1 of BASELINE.json: scipy csr@csr 1024x1024 density 0.01 fp64, seed 42,
    # B drawn from the same rng stream after A.
    rng = np.random.default_rng(42)
    A = rand(1024, 1024, 0.01, rng, np.float64)
    B = rand(1024, 1024, 0.01, rng, np.float64)
    cases.append(save("config1_n1024_d0.01_f64", A, B, note="BASELINE config 1"))

    # fp32, standard-normal values (the profilers' data_rvs, SpGEMM_alg_comparison/
    # profiler.py:149-151): signed values, so cancellations are possible.
    rng = np.random.default_rng(7)
    A = rand(512, 512, 0.05, rng, np.float32, rng.standard_normal)
    B = rand(512, 512, 0.05, rng, np.float32, rng.standard_normal)
    cases.append(save("normal_n512_d0.05_f32", A, B, note="standard-normal fp32"))

    # rectangular m x k x n with empty rows in A and B
    rng = np.random.default_rng(11)
    A = rand(300, 500, 0.02, rng, np.float64, rng.standard_normal).tolil()
    A[5, :] = 0
    A[17, :] = 0
    B = rand(500, 200, 0.03, rng, np.float64, rng.standard_normal).tolil()
    B[:40, :] = 0
    A = sp.csr_matrix(A); A.eliminate_zeros()
    B = sp.csr_matrix(B); B.eliminate_zeros()
    cases.append(save("rect_300x500x200_f64", A, B, alpha=-1.25, note="rectangular, alpha"))

    # exact cancellation: products that sum to exactly 0 (scipy drops them; cuSPARSE keeps a
    # structural zero).  Values are small integers so every sum is exact.
    rng = np.random.default_rng(5)
    A = sp.random(128, 128, density=0.08, format="csr", random_state=rng,
                  data_rvs=lambda s: rng.choice([-2.0, -1.0, 1.0, 2.0], size=s))
    B = sp.random(128, 128, density=0.08, format="csr", random_state=rng,
                  data_rvs=lambda s: rng.choice([-1.0, 1.0], size=s))
    A.sort_indices(); B.sort_indices()
    cases.append(save("cancel_n128_f64", A, B, note="exact cancellations -> dropped zeros"))

    # skewed rows: a dense row and a heavy column in A -> long output rows
    rng = np.random.default_rng(3)
    A = rand(1024, 1024, 0.005, rng, np.float64).tolil()
    A[7, :] = rng.uniform(0.5, 1.5, 1024)
    A[100, ::3] = 1.0
    A = sp.csr_matrix(A)
    B = rand(1024, 1024, 0.02, rng, np.float64, rng.standard_normal)
    cases.append(save("skew_n1024_f64", A, B, note="dense row + strided row"))

    # wide output: n = 300000 columns (multiple column windows on the device)
    rng = np.random.default_rng(9)
    A = rand(96, 2000, 0.02, rng, np.float64, rng.standard_normal)
    B = rand(2000, 300000, 1e-4, rng, np.float64, rng.standard_normal)
    cases.append(save("wide_96x2000x300000_f64", A, B, note="wide C (300k columns)"))

    # empty operands
    A = sp.csr_matrix((64, 32), dtype=np.float64)
    B = rand(32, 48, 0.2, np.random.default_rng(1), np.float64)
    cases.append(save("emptyA_64x32x48_f64", A, B, note="A has no entries"))

    # complex values (upstream TestSpgemm dtypes complex64/complex128, test_cusparse.py:
    # 372-375): the shapes with alpha 0.5, and larger random products with complex normal
    # values (scipy's complex_wrapper arithmetic: (ac - bd) + (ad + bc)i, no FMA)
    for dt in (np.complex64, np.complex128):
        tag = "c64" if dt == np.complex64 else "c128"
        for (m, n, k) in [(2, 3, 4), (4, 3, 2)]:
            rng = np.random.default_rng(2000 + m)
            a = rand(m, k, 0.5, rng, dt)
            b = rand(k, n, 0.5, rng, dt)
            a.data = a.data + 1j * rng.uniform(size=a.nnz)
            b.data = b.data + 1j * rng.uniform(size=b.nnz)
            cases.append(save(f"testspgemm_{m}x{n}x{k}_{tag}", a, b, alpha=0.5,
                              note="upstream TestSpgemm complex, alpha=0.5"))
        rng = np.random.default_rng(31 if dt == np.complex64 else 32)
        cn = lambda s: rng.standard_normal(s) + 1j * rng.standard_normal(s)
        A = rand(400, 300, 0.03, rng, dt, cn)
        B = rand(300, 500, 0.03, rng, dt, cn)
        cases.append(save(f"normal_400x300x500_{tag}", A, B, alpha=-0.75, note="complex normal, alpha"))

    spmv_cases = make_spmv()

    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "truth": f"scipy {scipy.__version__} csr@csr, numpy {np.__version__}",
                   "cases": cases, "spmv_cases": spmv_cases}, f, indent=1)
    print(f"wrote {len(cases)} cases")


if __name__ == "__main__":
    main()
