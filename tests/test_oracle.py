"""Pin the CPU oracle (oracle/gustavson.c) to scipy's own outputs (tests/golden/)."""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle
from tests.golden_cases import case_names, load, load_spmv, spmv_case_names

CASES = case_names()


def test_golden_present():
    assert len(CASES) >= 20


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_scipy_bitwise(name):
    A, B, C, alpha = load(name)
    # scipy semantics: zero sums dropped, linked-list column order -- must be identical,
    # array for array, bit for bit.
    p, j, x = oracle.spgemm(A, B, alpha=alpha, keep_zeros=False, sort=False)
    assert np.array_equal(p, C.indptr.astype(np.int64))
    assert np.array_equal(j, C.indices)
    assert x.dtype == C.data.dtype
    assert np.array_equal(x.view(np.uint8), C.data.view(np.uint8))


@pytest.mark.parametrize("name", CASES)
def test_oracle_structural_vs_scipy(name):
    A, B, C, alpha = load(name)
    p, j, x = oracle.spgemm(A, B, alpha=alpha, keep_zeros=True, sort=True)
    assert np.array_equal(p, oracle.symbolic(A, B))
    M = sp.csr_matrix((x, j, p), shape=C.shape)
    assert M.has_sorted_indices
    M.eliminate_zeros()
    Cs = C.copy()
    Cs.sort_indices()
    assert np.array_equal(M.indptr, Cs.indptr)
    assert np.array_equal(M.indices, Cs.indices)
    assert np.array_equal(M.data.view(np.uint8), Cs.data.view(np.uint8))


@pytest.mark.parametrize("name", [n for n in CASES if "fixture" in n or "testspgemm" in n
                                  or "cancel" in n or "rect" in n])
def test_python_restatement_agrees(name):
    A, B, _, alpha = load(name)
    p, j, x = oracle.spgemm(A, B, alpha=alpha, keep_zeros=True, sort=True)
    p2, j2, x2 = oracle.spgemm_py(A, B, alpha=alpha, keep_zeros=True)
    assert np.array_equal(p, p2) and np.array_equal(j, j2)
    assert np.array_equal(x.view(np.uint8), x2.view(np.uint8))


def test_cancellation_case_has_structural_zeros():
    A, B, C, _ = load("cancel_n128_f64")
    p = oracle.symbolic(A, B)
    assert p[-1] > C.nnz  # scipy dropped exact zeros that cuSPARSE semantics keep


def test_num_products():
    A, B, _, _ = load("config1_n1024_d0.01_f64")
    assert oracle.num_products(A, B) == 107449


def test_openmp_variant_identical():
    A, B, _, _ = load("skew_n1024_f64")
    p, j, x = oracle.spgemm(A, B, keep_zeros=True, sort=True)
    p2, j2, x2 = oracle.spgemm(A, B, keep_zeros=True, sort=True, threads=4)
    assert np.array_equal(p, p2) and np.array_equal(j, j2)
    assert np.array_equal(x.view(np.uint8), x2.view(np.uint8))


@pytest.mark.parametrize("name", ["fixture_make_unordered_f64", "fixture_make_duplicate_f64",
                                  "config1_n1024_d0.01_f64"])
def test_canonical_check(name):
    A, _, _, _ = load(name)
    assert oracle.has_canonical_format(A) == bool(A.has_canonical_format)


@pytest.mark.parametrize("name", spmv_case_names())
def test_oracle_spmv_matches_scipy_golden(name):
    """The SpMV restatement (scipy csr_matvec order) equals scipy's committed output bit for bit."""
    A, x, y, alpha = load_spmv(name)
    got = oracle.spmv(A, x, alpha=alpha)
    assert got.dtype == y.dtype
    assert np.array_equal(got.view(np.uint8), y.view(np.uint8))
