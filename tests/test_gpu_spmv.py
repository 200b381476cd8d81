"""SpMV parity (the SpMV half of SpGEMM_vs_SpMV/profiler.py:410-411; cupyx.cusparse.spmv,
modify_src/cupy-src/cupyx/cusparse.py:1373-1432), through the C ABI (spg_spmv).

Bar: CSR A @ x bit-exact against scipy's csr_matvec (golden vectors and the oracle's
restatement); y = alpha*A x + beta*y bit-exact against the same elementwise expression in
numpy; CSC / COO operands and op(A) = A^T within a stated tolerance (they reach CSR through
a conversion, and scipy sums those in a different order): |y - y_ref| <= 1e-12 (f64),
1e-4 (f32) relative to sum |a||x|.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle
from tests.golden_cases import load_spmv, spmv_case_names

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _bits(v):
    return np.ascontiguousarray(v).view(np.uint8)


def _run(A, x, **kw):
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    dA = csr_matrix(A, device="cuda:0")
    y = cusparse.spmv(dA, torch.from_numpy(np.ascontiguousarray(x)).cuda(), **kw)
    torch.cuda.synchronize()
    return y.cpu().numpy()


@pytest.mark.parametrize("name", spmv_case_names())
def test_spmv_golden_bitexact(name):
    A, x, y, alpha = load_spmv(name)
    got = _run(A, x, alpha=alpha)
    assert got.dtype == y.dtype
    assert np.array_equal(_bits(got), _bits(y))


@pytest.mark.parametrize("dt", [np.float32, np.float64, np.complex64, np.complex128])
def test_spmv_random_bitexact(dt):
    rng = np.random.default_rng(5)
    A = sp.random(5000, 3000, density=0.004, format="lil", random_state=rng)
    A[10, :] = rng.standard_normal(3000)          # a row longer than one LDS chunk (1024)
    A[11:80, :] = 0                               # a run of empty rows
    A = sp.csr_matrix(A)
    if np.dtype(dt).kind == "c":
        A.data = A.data + 1j * rng.standard_normal(A.nnz)
    A = A.astype(dt)
    A.sort_indices()
    x = rng.standard_normal(3000).astype(dt)
    assert np.array_equal(_bits(_run(A, x)), _bits(oracle.spmv(A, x)))
    assert np.array_equal(_bits(A @ x), _bits(oracle.spmv(A, x)))


def test_spmv_int64_indptr_alpha_beta():
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    rng = np.random.default_rng(6)
    A = sp.random(2000, 2000, density=0.01, format="csr", random_state=rng)
    x = rng.standard_normal(2000)
    y0 = rng.standard_normal(2000)
    dA = csr_matrix(A, device="cuda:0")
    dA.indptr = dA.indptr.to(torch.int64)
    y = torch.from_numpy(y0.copy()).cuda()
    cusparse.spmv(dA, torch.from_numpy(x).cuda(), y=y, alpha=-1.5, beta=0.25)
    want = np.float64(-1.5) * oracle.spmv(A, x) + np.float64(0.25) * y0
    assert np.array_equal(_bits(y.cpu().numpy()), _bits(want))


def test_spmv_formats_and_transpose():
    from spmm_amd import cusparse
    from spmm_amd.sparse import coo_matrix, csc_matrix, csr_matrix
    rng = np.random.default_rng(7)
    A = sp.random(700, 400, density=0.02, format="csr", random_state=rng)
    A.data = rng.standard_normal(A.nnz)
    x = rng.standard_normal(400)
    xt = rng.standard_normal(700)
    tol = 1e-12 * (abs(A) @ np.abs(x)).max()
    xd = torch.from_numpy(x).cuda()
    for M in (csc_matrix(A, device="cuda:0"), coo_matrix(A, device="cuda:0")):
        np.testing.assert_allclose((M @ xd).cpu().numpy(), A @ x, rtol=0, atol=tol)
    y = cusparse.spmv(csr_matrix(A, device="cuda:0"), torch.from_numpy(xt).cuda(), transa=True)
    np.testing.assert_allclose(y.cpu().numpy(), A.T @ xt, rtol=0, atol=1e-12 * (abs(A.T) @ np.abs(xt)).max())
    # numpy x is uploaded; csr @ x dispatches to spmv
    yy = csr_matrix(A, device="cuda:0") @ x
    assert np.array_equal(_bits(yy.cpu().numpy()), _bits(A @ x))


def test_spmv_reference_errors():
    """cusparse.py:1394-1409: TypeError for an unsupported operand, ValueError for a
    length mismatch; nnz == 0 gives zeros."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    A = sp.random(30, 20, density=0.2, format="csr", random_state=1)
    with pytest.raises(ValueError):
        cusparse.spmv(csr_matrix(A, device="cuda:0"), torch.zeros(21, dtype=torch.float64).cuda())
    with pytest.raises(TypeError):
        cusparse.spmv(A, torch.zeros(20, dtype=torch.float64).cuda())
    Z = csr_matrix(sp.csr_matrix((30, 20)), device="cuda:0")
    y = torch.ones(30, dtype=torch.float64).cuda()
    assert torch.count_nonzero(cusparse.spmv(Z, torch.ones(20, dtype=torch.float64).cuda(), y=y)) == 0
