"""Parity of the HIP SpGEMM (through the C ABI) with the CPU oracle and scipy.

Bar: row pointers and column indices bit-exact; values bit-exact too, because
the engine accumulates every C(i,j) in A's entry order with separately rounded mul/add,
exactly scipy's rule (the fp tolerance of the north star, |c - c_ref| <= gamma_m (|A||B|)_ij,
is therefore met with margin 0).  Structural zeros are kept (cuSPARSE semantics); after
eliminate_zeros() the result must equal scipy's, array for array.
"""
import os
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle
from tests.golden_cases import case_names, load

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

# "3c": ALG3 with its chunks kept even where the unchunked workspace is within the cap
# (SPG_ALG3_CHUNK_ALWAYS, a schedule-only switch): the chunked paths on small inputs
ALGS = [(1, 0.2), (2, 0.2), (3, 0.2), ("3c", 0.2), ("3c", 0.05), (0, 0.2)]


def _dev():
    return "cuda:0"


def _gpu(A, B, alg=2, alpha=1.0, cf=0.2):
    import os
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    if alg == "3c":
        os.environ["SPG_ALG3_CHUNK_ALWAYS"] = "1"
        try:
            return _gpu(A, B, 3, alpha, cf)
        finally:
            del os.environ["SPG_ALG3_CHUNK_ALWAYS"]
    dA = csr_matrix(A, device=_dev())
    dB = csr_matrix(B, device=_dev())
    if not (dA.has_canonical_format and dB.has_canonical_format):
        dA.sum_duplicates()
        dB.sum_duplicates()
    C = cusparse.spgemm(dA, dB, alpha=alpha, alg=alg, chunk_fraction=cf)
    torch.cuda.synchronize()
    return (C.indptr.cpu().numpy().astype(np.int64), C.indices.cpu().numpy(),
            C.data.cpu().numpy(), C.shape)


def _bits(x):
    return x.view(np.uint32 if x.dtype == np.float32 else np.uint64)


def _assert_same(got, ref):
    p, j, x = got[:3]
    rp, rj, rx = ref
    assert np.array_equal(p, rp), "row pointer"
    assert np.array_equal(j, rj), "column indices"
    assert x.dtype == rx.dtype
    assert np.array_equal(_bits(x), _bits(rx)), \
        f"values differ at {np.flatnonzero(_bits(x) != _bits(rx))[:5]}"


def _canon(A):
    A = sp.csr_matrix(A, copy=True)
    A.sum_duplicates()
    return A


@pytest.mark.parametrize("alg,cf", ALGS)
@pytest.mark.parametrize("name", case_names())
def test_golden_bitexact(name, alg, cf):
    A, B, C, alpha = load(name)
    got = _gpu(A, B, alg=alg, alpha=alpha, cf=cf)
    # engine vs oracle (structural entries kept, sorted), on the canonicalised inputs
    ref = oracle.spgemm(_canon(A), _canon(B), alpha=alpha, keep_zeros=True, sort=True)
    _assert_same(got, ref)
    if A.has_canonical_format and B.has_canonical_format:
        # and vs scipy's own output (zeros dropped, columns sorted)
        M = sp.csr_matrix((got[2], got[1], got[0]), shape=got[3])
        M.eliminate_zeros()
        Cs = C.copy()
        Cs.sort_indices()
        assert np.array_equal(M.indptr, Cs.indptr)
        assert np.array_equal(M.indices, Cs.indices)
        assert np.array_equal(_bits(M.data), _bits(Cs.data))
    else:
        np.testing.assert_allclose(sp.csr_matrix((got[2], got[1], got[0]), shape=got[3]).toarray(),
                                   C.toarray(), rtol=1e-6, atol=0)


@pytest.mark.parametrize("n,density,dtype", [
    (1024, 0.01, np.float64), (2048, 0.02, np.float32), (16384, 1e-3, np.float64),
    (8192, 1e-4, np.float64), (8192, 1e-3, np.float64), (4096, 0.05, np.float64),
    (3000, 0.3, np.float32)])
@pytest.mark.parametrize("alg", [1, 2, 3, "3c"])
def test_random_bitexact(n, density, dtype, alg):
    from spmm_amd import gen
    A, B = gen.scipy_pair(n, density, seed=n + int(density * 1e6), dtype=dtype, normal=True)
    got = _gpu(A, B, alg=alg)
    _assert_same(got, oracle.spgemm(A, B, keep_zeros=True, sort=True))


def test_config2_nnz_and_products():
    """BASELINE config 2: N=16384, density 1e-3, fp64, seed 42 (SURVEY 8d numbers)."""
    from spmm_amd import cusparse, gen
    from spmm_amd.sparse import csr_matrix
    A, B = gen.scipy_pair(16384, 1e-3, seed=42)
    dA, dB = csr_matrix(A, device=_dev()), csr_matrix(B, device=_dev())
    assert cusparse.num_products(dA, dB) == 4402284
    C = cusparse.spgemm(dA, dB, alg=1)
    assert C.nnz == 4366124
    _assert_same((C.indptr.cpu().numpy().astype(np.int64), C.indices.cpu().numpy(),
                  C.data.cpu().numpy()), oracle.spgemm(A, B, keep_zeros=True, sort=True))


def test_determinism_run_to_run():
    """The reference's deterministic/ check, as a test: same inputs twice, same bits."""
    from spmm_amd import gen
    A, B = gen.scipy_pair(4096, 0.01, seed=2008, normal=True)
    for alg in (1, 2, 3):
        r1 = _gpu(A, B, alg=alg)
        r2 = _gpu(A, B, alg=alg)
        for a, b in zip(r1[:3], r2[:3]):
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


def test_algs_agree_bitwise():
    """numerical_error/error.py compares ALG1 with ALG3 (max abs error); here all three
    algorithms must agree bit for bit for every chunk_fraction."""
    from spmm_amd import gen
    A, B = gen.scipy_pair(2048, 0.05, seed=10, dtype=np.float32, normal=True)
    ref = _gpu(A, B, alg=1)
    for alg, cf in [(2, 0.2), (3, 0.3), (3, 0.01), (3, 1.0)]:
        _assert_same(_gpu(A, B, alg=alg, cf=cf), ref[:3])


def test_dense_rows_multiwindow():
    """Rows of C with more entries than one LDS window holds (window halving path) and
    wide C (cursor walk over many windows)."""
    rng = np.random.default_rng(1)
    A = sp.random(64, 512, density=0.9, format="csr", random_state=rng)
    B = sp.random(512, 6000, density=0.3, format="csr", random_state=rng)
    A.sort_indices(); B.sort_indices()
    for alg in (1, 2, 3):
        _assert_same(_gpu(A, B, alg=alg), oracle.spgemm(A, B, keep_zeros=True, sort=True))
    A = sp.random(200, 3000, density=0.05, format="csr", random_state=rng)
    B = sp.random(3000, 400000, density=2e-4, format="csr", random_state=rng)
    A.sort_indices(); B.sort_indices()
    for alg in (1, 2):
        _assert_same(_gpu(A, B, alg=alg), oracle.spgemm(A, B, keep_zeros=True, sort=True))


def test_edge_shapes():
    rng = np.random.default_rng(4)
    cases = [
        (sp.csr_matrix((0, 5)), sp.random(5, 7, density=0.5, format="csr", random_state=rng)),
        (sp.random(6, 5, density=0.5, format="csr", random_state=rng), sp.csr_matrix((5, 0))),
        (sp.random(6, 0, density=0.5, format="csr", random_state=rng), sp.csr_matrix((0, 9))),
        (sp.random(1, 300, density=0.5, format="csr", random_state=rng),
         sp.random(300, 1, density=0.5, format="csr", random_state=rng)),
        (sp.csr_matrix(np.ones((3, 3))), sp.csr_matrix(np.eye(3))),
    ]
    for A, B in cases:
        A = sp.csr_matrix(A, dtype=np.float64); B = sp.csr_matrix(B, dtype=np.float64)
        A.sort_indices(); B.sort_indices()
        for alg in (1, 2, 3):
            got = _gpu(A, B, alg=alg)
            _assert_same(got, oracle.spgemm(A, B, keep_zeros=True, sort=True))
            assert got[3] == (A.shape[0], B.shape[1])


def test_int64_row_pointers():
    from spmm_amd import cusparse, gen
    from spmm_amd.sparse import csr_matrix
    A, B = gen.scipy_pair(2048, 0.01, seed=5)
    dA, dB = csr_matrix(A, device=_dev()), csr_matrix(B, device=_dev())
    dA.indptr = dA.indptr.to(torch.int64)
    dB.indptr = dB.indptr.to(torch.int64)
    C = cusparse.spgemm(dA, dB, alg=2)
    _assert_same((C.indptr.cpu().numpy().astype(np.int64), C.indices.cpu().numpy(),
                  C.data.cpu().numpy()), oracle.spgemm(A, B, keep_zeros=True, sort=True))


def test_matmul_dispatch_and_formats():
    """A @ B with CSR / CSC / COO right operands (CuPy _csr.py:151-184) and unsorted /
    duplicate left operands (test_csr.py fixtures)."""
    from spmm_amd.sparse import coo_matrix, csc_matrix, csr_matrix
    A, B, _, _ = load("fixture_make_duplicate_f64")
    x = B
    for make in (lambda M: csr_matrix(M, device=_dev()), lambda M: csc_matrix(M, device=_dev()),
                 lambda M: coo_matrix(M, device=_dev())):
        dA = csr_matrix(A, device=_dev())
        C = dA @ make(x)
        np.testing.assert_allclose(C.toarray(), (A @ x).toarray(), rtol=1e-7, atol=0)


def test_reference_error_behaviour():
    """test_cusparse.py:413-454: TypeError for CSC, ValueError for mismatched shapes."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csc_matrix, csr_matrix
    rng = np.random.default_rng(0)
    a = sp.random(2, 4, density=0.5, dtype=np.float32, random_state=rng)
    b = sp.random(4, 3, density=0.5, dtype=np.float32, random_state=rng)
    with pytest.raises(TypeError):
        cusparse.spgemm(csc_matrix(a, device=_dev()), csr_matrix(b, device=_dev()))
    with pytest.raises(TypeError):
        cusparse.spgemm(csr_matrix(a, device=_dev()), csc_matrix(b, device=_dev()))
    with pytest.raises(ValueError):
        cusparse.spgemm(csc_matrix(a, device=_dev()).T, csr_matrix(b, device=_dev()))
    with pytest.raises(ValueError):
        cusparse.spgemm(csr_matrix(a, device=_dev()), csc_matrix(b, device=_dev()).T)
    assert cusparse.check_availability("spgemm")


def test_upstream_testspgemm_alpha():
    """test_cusparse.py:372-411: f32/f64, shapes (2,3,4), (4,3,2) and the (100000, 100000,
    50) run-only case, alpha = 0.5."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    for dt in (np.float32, np.float64):
        for (m, n, k) in [(2, 3, 4), (4, 3, 2), (100000, 100000, 50)]:
            rng = np.random.default_rng(m + n + k)
            a = sp.random(m, k, density=0.5, dtype=dt, random_state=rng, format="csr")
            b = sp.random(k, n, density=0.5, dtype=dt, random_state=rng, format="csr")
            a.sort_indices(); b.sort_indices()
            c = cusparse.spgemm(csr_matrix(a, device=_dev()), csr_matrix(b, device=_dev()),
                                alpha=0.5)
            if m == 100000:
                assert c.nnz > 0
                continue
            np.testing.assert_array_almost_equal(c.toarray(), (0.5 * a.dot(b)).toarray())


def test_validate_csr():
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    for name, want in [("fixture_make_unordered_f64", 0), ("fixture_make_duplicate_f64", 0),
                       ("config1_n1024_d0.01_f64", 1)]:
        A, _, _, _ = load(name)
        d = csr_matrix((A.data, A.indices, A.indptr), shape=A.shape, device=_dev())
        assert cusparse.validate_csr(d) == want
    bad = csr_matrix((np.ones(2), np.array([0, 9], np.int32), np.array([0, 1, 2])),
                     shape=(2, 4), device=_dev())
    assert cusparse.validate_csr(bad) == -1


def test_short_kernel_long_rows():
    """Rows beyond the short-row kernel's register path: more than 640 products (with more
    than 512 output entries, and with heavy column overlap), and rows whose repeated
    columns overflow its fix-up list -- all handed to the general kernel, same bits."""
    rng = np.random.default_rng(21)
    cases = [
        (sp.random(200, 2000, density=0.02, format="csr", random_state=rng),
         sp.random(2000, 8000, density=0.005, format="csr", random_state=rng)),   # P~1600, nnz~1450
        (sp.random(150, 2000, density=0.03, format="csr", random_state=rng),
         sp.random(2000, 300, density=0.05, format="csr", random_state=rng)),    # P~900, nnz<=300
        (sp.random(100, 3000, density=0.02, format="csr", random_state=rng),
         sp.random(3000, 16384, density=0.01, format="csr", random_state=rng)),  # widest short case
        # ~350 products into 200 columns: k_row's list of products in flagged (repeated)
        # bitmap words overflows 64 entries -> the general kernel, in every algorithm
        (sp.random(1000, 2000, density=0.0175, format="csr", random_state=rng),
         sp.random(2000, 200, density=0.05, format="csr", random_state=rng)),
    ]
    for A, B in cases:
        A.sort_indices(); B.sort_indices()
        for alg in (1, 2, 3):
            _assert_same(_gpu(A, B, alg=alg), oracle.spgemm(A, B, keep_zeros=True, sort=True))


def _skewed(rng, rows, k, n, dense_rows, base_density, b_density, dtype=np.float64):
    """A: sparse rows plus a few full rows and some empty ones; B: uniform random."""
    A = sp.random(rows, k, density=base_density, format="lil", random_state=rng, dtype=dtype)
    for r in dense_rows:
        A[r, :] = rng.standard_normal(k).astype(dtype)
    for r in range(3, rows, 37):
        A[r, :] = 0
    A = sp.csr_matrix(A)
    B = sp.random(k, n, density=b_density, format="csr", random_state=rng, dtype=dtype)
    for M in (A, B):
        M.sum_duplicates()
        M.sort_indices()
    return A, B


def test_tile_path_windows_and_skew():
    """Wide-row (row, column tile) path: 4096-column tiles whose dense rows need several
    LDS windows per tile, empty A rows, a ragged last tile (n % 4096 != 0), alpha != 1,
    every algorithm (ALG3 with many chunks)."""
    rng = np.random.default_rng(31)
    A, B = _skewed(rng, 384, 4096, 100003, dense_rows=[0, 17, 200, 383], base_density=0.05,
                   b_density=0.001)
    ref = oracle.spgemm(A, B, alpha=-0.75, keep_zeros=True, sort=True)
    assert np.diff(ref[0]).max() > 4 * 1024        # some tiles hold several windows
    for alg, cf in [(1, 0.2), (2, 0.2), (3, 0.2), (3, 0.02)]:
        _assert_same(_gpu(A, B, alg=alg, alpha=-0.75, cf=cf), ref)


@pytest.mark.parametrize("neg", [False, True])
def test_tile_path_dense_2048(neg):
    """fp64 C rows over half dense and >= 16384 columns take 2048-column dense tiles
    (k_tile_dn<double, .., 2048>; config 4's shape): a ragged last tile, an empty A row, B
    with empty rows, every algorithm with ALG3's chunks forced; `neg` sets 30 % of B's values
    to -0.0 (the accumulator's -0.0 start and its re-walk).  plan_info confirms the width."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    rng = np.random.default_rng(33)
    A = sp.random(257, 17000, density=0.01, format="lil", random_state=rng, dtype=np.float64)
    A[5, :] = 0
    A = sp.csr_matrix(A)
    B = sp.random(17000, 17000, density=0.01, format="lil", random_state=rng, dtype=np.float64)
    B[100:140, :] = 0
    B = sp.csr_matrix(B)
    if neg:
        A.data = np.abs(A.data) + 0.5
        B.data = np.where(rng.random(B.nnz) < 0.3, -0.0, B.data)
    for M in (A, B):
        M.sort_indices()
    ref = oracle.spgemm(A, B, keep_zeros=True, sort=True)
    dA, dB = csr_matrix(A, device=_dev()), csr_matrix(B, device=_dev())
    info = cusparse.plan_info(dA, dB, alg=2)
    assert info["tile_width"] == 2048 and info["dense_tiles"], info
    for alg, cf in [(1, 0.2), (2, 0.2), ("3c", 0.1)]:
        _assert_same(_gpu(A, B, alg=alg, cf=cf), ref)


def test_tile_path_dense_2048_width_band():
    """fp64 C rows 24-48 % dense over >= 16384 columns reach 2048-column DENSE tiles through
    the width loop (spgemm.hip want_tile: 2048 columns hold <= 0.95 * 1024 expected entries),
    not through the >= 50 % rule: a case in that band,
    C rows ~30 % dense (expected entries per row / columns = 1 - exp(-avgA * avgB / N)), a
    ragged last tile, every algorithm with ALG3's chunks forced, bit-exact."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    rng = np.random.default_rng(38)
    n = 20000
    A = sp.random(180, n, density=0.0042, format="csr", random_state=rng)
    B = sp.random(n, n, density=0.0042, format="csr", random_state=rng)
    for M in (A, B):
        M.sort_indices()
    ref = oracle.spgemm(A, B, keep_zeros=True, sort=True)
    frac = (np.diff(ref[0]).mean()) / n
    assert 0.24 < frac < 0.45, frac
    dA, dB = csr_matrix(A, device=_dev()), csr_matrix(B, device=_dev())
    info = cusparse.plan_info(dA, dB, alg=2)
    assert info["tile_width"] == 2048 and info["dense_tiles"] and info["record_group"] == 1, info
    for alg, cf in [(1, 0.2), (2, 0.2), ("3c", 0.1)]:
        _assert_same(_gpu(A, B, alg=alg, cf=cf), ref)


def _random_rows(rng, rows, cols, per_row):
    """CSR with ~per_row random entries per row (numpy, no N^2 sampling), canonical."""
    r = np.repeat(np.arange(rows), per_row)
    c = rng.integers(0, cols, size=rows * per_row)
    M = sp.csr_matrix((rng.random(rows * per_row), (r, c)), shape=(rows, cols))
    M.sum_duplicates()
    M.sort_indices()
    return M


@pytest.mark.parametrize("ncols,choices", [(20000, [0, 40, 300, 700, 1500]), (140000, [0, 100, 300, 600, 900])])
def test_symbolic_segments_long_and_ragged(ncols, choices):
    """The segment symbolic kernel's round-6 loop (k_tile_sym_seg, SPG_SYM_PF): a round's first
    three steps of column loads together, the next round's extents as raw words a round later,
    then the extra steps of segments longer than 384 columns.  B rows of 0 to 1500 entries,
    A rows whose entry counts are not multiples of 16, an empty A row; whole-row symbolic tiles
    (20000 columns, dense 2048-column numeric tiles) and 65536-column symbolic tiles of a
    140000-column B (three per row, the last ragged; sparse numeric tiles); bit-exact for every
    algorithm."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    rng = np.random.default_rng(41)
    k = 20000
    lens = rng.choice(choices, size=k, p=[0.05, 0.25, 0.4, 0.2, 0.1])
    r = np.repeat(np.arange(k), lens)
    B = sp.csr_matrix((rng.standard_normal(r.size), (r, rng.integers(0, ncols, size=r.size))), shape=(k, ncols))
    B.sum_duplicates()
    B.sort_indices()
    alen = rng.integers(1, 40, size=160)
    alen[7] = 0
    ra = np.repeat(np.arange(160), alen)
    A = sp.csr_matrix((rng.standard_normal(ra.size), (ra, rng.integers(0, k, size=ra.size))), shape=(160, k))
    A.sum_duplicates()
    A.sort_indices()
    dA, dB = csr_matrix(A, device=_dev()), csr_matrix(B, device=_dev())
    info = cusparse.plan_info(dA, dB, alg=2)
    assert info["path"] == "tile", info
    ref = oracle.spgemm(A, B, keep_zeros=True, sort=True)
    for alg, cf in [(1, 0.2), (2, 0.2), ("3c", 0.1)]:
        _assert_same(_gpu(A, B, alg=alg, cf=cf), ref)


def test_tile_path_cooperative_groups_with_padding():
    """Config 5's cooperative record groups on a shape whose tile count does not divide by 8:
    300000 columns -> 37 numeric tiles of 8192 (record groups of 8: the last holds 5 real tiles
    and 3 padding tiles), 5 symbolic tiles of 65536.  Bit-exact for ALG2 and chunked ALG3, and
    the same with the one-wave kernel (SPG_SP_RECORD_GROUP=1)."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    rng = np.random.default_rng(39)
    n = 300000
    A = _random_rows(rng, 200, n, 600)
    B = _random_rows(rng, n, n, 60)
    dA, dB = csr_matrix(A, device=_dev()), csr_matrix(B, device=_dev())
    info = cusparse.plan_info(dA, dB, alg=2)
    assert info["tile_width"] == 8192 and info["tiles_per_row"] == 37 and info["record_group"] == 8, info
    ref = oracle.spgemm(A, B, alpha=1.5, keep_zeros=True, sort=True, threads=16)
    for alg, cf in [(2, 0.2), ("3c", 0.1)]:
        _assert_same(_gpu(A, B, alg=alg, alpha=1.5, cf=cf), ref)
    os.environ["SPG_SP_RECORD_GROUP"] = "1"
    try:
        _assert_same(_gpu(A, B, alg=2, alpha=1.5), ref)
    finally:
        del os.environ["SPG_SP_RECORD_GROUP"]


def test_tile_path_sparse_8192():
    """fp64 C rows 10-24 % dense over >= 16384 columns take 8192-column sparse tiles
    (k_tile_sp<double, .., 2048>; config 5's shape): skewed A rows whose items need several
    2048-slot windows, an empty A row, a ragged last tile, alpha != 1, every algorithm (ALG3
    with many chunks).  plan_info confirms the width."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    rng = np.random.default_rng(34)
    A = sp.random(300, 40000, density=0.0075, format="lil", random_state=rng)
    for r in (0, 7, 151, 299):   # 3000-entry rows: ~35,800 C entries, several windows per item
        A[r, :] = sp.random(1, 40000, density=0.075, format="lil", random_state=rng)
    for r in range(3, 300, 37):
        A[r, :] = 0
    A = sp.csr_matrix(A)
    B = sp.random(40000, 40000, density=0.00075, format="csr", random_state=rng)
    for M in (A, B):
        M.sum_duplicates()
        M.sort_indices()
    dA, dB = csr_matrix(A, device=_dev()), csr_matrix(B, device=_dev())
    info = cusparse.plan_info(dA, dB, alg=2)
    assert info["tile_width"] == 8192 and not info["dense_tiles"], info
    # cooperative record groups of 8 tiles (k_tile_sp<.., SpCfgRG, 8>): G = 5 tiles, so the
    # one group holds five real tiles and three padding tiles
    assert info["record_group"] == 8 and info["tiles_per_row"] == 5, info
    ref = oracle.spgemm(A, B, alpha=0.5, keep_zeros=True, sort=True)
    assert np.diff(ref[0]).max() > 2 * 2048 * 4   # dense rows: several windows per item
    for alg, cf in [(1, 0.2), (2, 0.2), (3, 0.2), ("3c", 0.02)]:
        _assert_same(_gpu(A, B, alg=alg, alpha=0.5, cf=cf), ref)
    # the one-wave kernel over plain tile-major records (SPG_SP_RECORD_GROUP=1): same bits
    os.environ["SPG_SP_RECORD_GROUP"] = "1"
    try:
        assert cusparse.plan_info(dA, dB, alg=2)["record_group"] == 1
        for alg, cf in [(2, 0.2), ("3c", 0.02)]:
            _assert_same(_gpu(A, B, alg=alg, alpha=0.5, cf=cf), ref)
    finally:
        del os.environ["SPG_SP_RECORD_GROUP"]


def test_tile_path_dense_tiles_fp32_int64():
    """1024-column tiles over a dense C (batches of 64 A entries with > 1024 products per
    batch and tile), fp32 values, int64 row pointers, B with empty rows."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    rng = np.random.default_rng(32)
    A = sp.random(300, 2500, density=0.2, format="csr", random_state=rng, dtype=np.float32)
    B = sp.random(2500, 5000, density=0.25, format="lil", random_state=rng, dtype=np.float32)
    B[10:40, :] = 0
    B = sp.csr_matrix(B)
    for M in (A, B):
        M.sort_indices()
    ref = oracle.spgemm(A, B, keep_zeros=True, sort=True)
    dA, dB = csr_matrix(A, device=_dev()), csr_matrix(B, device=_dev())
    dA.indptr = dA.indptr.to(torch.int64)
    dB.indptr = dB.indptr.to(torch.int64)
    for alg in (1, 2, 3):
        C = cusparse.spgemm(dA, dB, alg=alg, chunk_fraction=0.1)
        _assert_same((C.indptr.cpu().numpy().astype(np.int64), C.indices.cpu().numpy(),
                      C.data.cpu().numpy()), ref)


def test_alg1_single_pass_fallback_long_row():
    """ALG1 runs as one fused pass for short-row shapes; a row with more than 64 entries
    makes the pass hand over to the upper-bound path, with the same result."""
    rng = np.random.default_rng(41)
    A = sp.random(3000, 2000, density=0.004, format="lil", random_state=rng)
    A[1234, :300] = rng.standard_normal(300)
    A = sp.csr_matrix(A)
    B = sp.random(2000, 3000, density=0.004, format="csr", random_state=rng)
    A.sort_indices(); B.sort_indices()
    ref = oracle.spgemm(A, B, alpha=2.5, keep_zeros=True, sort=True)
    _assert_same(_gpu(A, B, alg=1, alpha=2.5), ref)
    _assert_same(_gpu(A, B, alg=2, alpha=2.5), ref)


def test_alg1_single_pass_abi_sequence():
    """C-ABI sequence of the fused ALG1: repeated spg_symbolic (int32 then int64 row
    pointer, the overflow retry) rewrites the row pointer from the look-back words; C in
    the workspace is scaled once in place; C elsewhere gets a copy; a second in-place
    scaling is refused."""
    import ctypes
    from spmm_amd import _lib, gen
    from spmm_amd._lib import SpgCsr
    from spmm_amd.sparse import csr_matrix
    Ah, Bh = gen.scipy_pair(4096, 2e-3, seed=77)
    ref = oracle.spgemm(Ah, Bh, alpha=-3.0, keep_zeros=True, sort=True)
    A, B = csr_matrix(Ah, device=_dev()), csr_matrix(Bh, device=_dev())
    h = _lib.get_handle(0)
    h.set_stream(torch.cuda.current_stream().cuda_stream)
    lib = h.lib

    def view(M):
        return SpgCsr(M.shape[0], M.shape[1], M.nnz, M.indptr.data_ptr(), M.indices.data_ptr(),
                      M.data.data_ptr(), _lib.SPG_INDEX_32I, _lib.SPG_R_64F)

    va, vb = view(A), view(B)
    for in_place in (True, False):
        wsb = ctypes.c_size_t(0)
        _lib.check(lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), _lib.SPG_ALG1, 0.2,
                                ctypes.byref(wsb), None, None))
        ws = torch.empty(wsb.value, dtype=torch.uint8, device=_dev())
        plan = ctypes.c_void_p()
        _lib.check(lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), _lib.SPG_ALG1, 0.2,
                                ctypes.byref(wsb), ctypes.c_void_p(ws.data_ptr()), ctypes.byref(plan)))
        p32 = torch.empty(4097, dtype=torch.int32, device=_dev())
        p64 = torch.empty(4097, dtype=torch.int64, device=_dev())
        nnz = ctypes.c_int64(0)
        _lib.check(lib.spg_symbolic(h.ptr, plan, ctypes.c_void_p(p32.data_ptr()), _lib.SPG_INDEX_32I,
                                    ctypes.byref(nnz)))
        _lib.check(lib.spg_symbolic(h.ptr, plan, ctypes.c_void_p(p64.data_ptr()), _lib.SPG_INDEX_64I,
                                    ctypes.byref(nnz)))
        assert nnz.value == len(ref[1])
        assert np.array_equal(p32.cpu().numpy().astype(np.int64), ref[0])
        assert np.array_equal(p64.cpu().numpy(), ref[0])
        pj, px = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(lib.spg_result_in_workspace(plan, ctypes.byref(pj), ctypes.byref(px)))
        assert pj.value and px.value
        n = nnz.value
        if in_place:
            cj = ws[pj.value - ws.data_ptr():][:4 * n].view(torch.int32)
            cx = ws[px.value - ws.data_ptr():][:8 * n].view(torch.float64)
        else:
            cj = torch.empty(n, dtype=torch.int32, device=_dev())
            cx = torch.empty(n, dtype=torch.float64, device=_dev())
        vc = SpgCsr(4096, 4096, n, p64.data_ptr(), cj.data_ptr(), cx.data_ptr(), _lib.SPG_INDEX_64I,
                    _lib.SPG_R_64F)
        al = ctypes.c_double(-3.0)
        _lib.check(lib.spg_numeric(h.ptr, plan, ctypes.byref(al), ctypes.byref(vc)))
        if in_place:
            assert lib.spg_numeric(h.ptr, plan, ctypes.byref(al), ctypes.byref(vc)) == 3
        torch.cuda.synchronize()
        _assert_same((p64.cpu().numpy(), cj.cpu().numpy(), cx.cpu().numpy()), ref)
        lib.spg_plan_destroy(plan)


def test_alg1_single_pass_estimate_overflow():
    """ALG1's single pass sizes its output from the expected product count; when A's
    entries select B's longest rows, the output outgrows the estimate and the product is
    redone two-phase, with the same bits."""
    rng = np.random.default_rng(43)
    B = sp.random(2000, 3000, density=0.001, format="lil", random_state=rng)
    for r in range(10):
        B[r, rng.choice(3000, 1500, replace=False)] = rng.standard_normal(1500)
    B = sp.csr_matrix(B)
    rows, cols = [], []
    for i in range(3000):
        for c in rng.choice(10, 5, replace=False):
            rows.append(i); cols.append(c)
    A = sp.csr_matrix((rng.standard_normal(len(rows)), (rows, cols)), shape=(3000, 2000))
    for M in (A, B):
        M.sum_duplicates(); M.sort_indices()
    ref = oracle.spgemm(A, B, alpha=1.5, keep_zeros=True, sort=True)
    assert len(ref[1]) > 10 * A.nnz * (B.nnz / B.shape[0])
    _assert_same(_gpu(A, B, alg=1, alpha=1.5), ref)


def _cplx_random(m, n, density, rng, dt):
    M = sp.random(m, n, density=density, format="csr", random_state=rng, dtype=np.float64)
    M = sp.csr_matrix((M.data + 1j * rng.standard_normal(M.nnz), M.indices, M.indptr),
                      shape=M.shape).astype(dt)
    M.sort_indices()
    return M


@pytest.mark.parametrize("dt", [np.complex64, np.complex128])
@pytest.mark.parametrize("m,k,n,density", [
    (2048, 2048, 2048, 0.004),      # short-row kernel
    (600, 3000, 4000, 0.03),        # tile path (dense C rows)
    (300, 2000, 200000, 2e-4),      # general windowed kernel (very wide, sparse C)
])
@pytest.mark.parametrize("alg", [1, 2, 3])
def test_complex_bitexact(dt, m, k, n, density, alg):
    """complex64 / complex128 (the reference's TestSpgemm dtypes): scipy's complex product
    (ac - bd) + (ad + bc)i, summed in A's entry order, alpha complex."""
    rng = np.random.default_rng(m + n + (7 if dt == np.complex64 else 9))
    A = _cplx_random(m, k, density, rng, dt)
    B = _cplx_random(k, n, density, rng, dt)
    alpha = 0.5 - 0.25j
    _assert_same(_gpu(A, B, alg=alg, alpha=alpha), oracle.spgemm(A, B, alpha=alpha, keep_zeros=True, sort=True))


def test_upstream_testspgemm_complex():
    """test_cusparse.py:372-411 with dtype complex64 / complex128 (alpha 0.5), including
    the (100000, 100000, 50) run-only case."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    for dt in (np.complex64, np.complex128):
        for (m, n, k) in [(2, 3, 4), (4, 3, 2), (100000, 100000, 50)]:
            rng = np.random.default_rng(m + n + k + 5)
            a = sp.random(m, k, density=0.5, dtype=dt, random_state=rng, format="csr")
            b = sp.random(k, n, density=0.5, dtype=dt, random_state=rng, format="csr")
            a.data = (a.data + 1j * rng.uniform(size=a.nnz)).astype(dt)
            b.data = (b.data + 1j * rng.uniform(size=b.nnz)).astype(dt)
            a.sort_indices(); b.sort_indices()
            c = cusparse.spgemm(csr_matrix(a, device=_dev()), csr_matrix(b, device=_dev()), alpha=0.5)
            assert c.dtype == dt
            if m == 100000:
                assert c.nnz > 0
                continue
            np.testing.assert_array_almost_equal(c.toarray(), (0.5 * a.dot(b)).toarray())


def test_shim_paths_agree(monkeypatch):
    """The native shim (csrc/fastpath.cpp) and the ctypes shim run the same C ABI: bit-equal
    results, the same stats, for every algorithm, alpha != 1 and fp32."""
    from spmm_amd import _fastpath
    rng = np.random.default_rng(61)
    for dt in (np.float64, np.float32):
        A = sp.random(3000, 2500, density=0.006, format="csr", random_state=rng, dtype=dt)
        B = sp.random(2500, 4000, density=0.005, format="csr", random_state=rng, dtype=dt)
        A.sort_indices(); B.sort_indices()
        ref = oracle.spgemm(A, B, alpha=-1.25, keep_zeros=True, sort=True)
        for alg in (1, 2, 3):
            fast = _gpu(A, B, alg=alg, alpha=-1.25, cf=0.3)
            _assert_same(fast, ref)
            monkeypatch.setattr(_fastpath, "_mod", None)
            monkeypatch.setattr(_fastpath, "_tried", True)   # ctypes path only
            slow = _gpu(A, B, alg=alg, alpha=-1.25, cf=0.3)
            monkeypatch.undo()
            _assert_same(slow, ref)


def test_spgemm_ws_abi():
    """spg_spgemm_ws through ctypes: ALG1 returns C in the workspace (complete, scaled), ALG2
    returns the live plan for the caller's spg_numeric; both bit-exact."""
    import ctypes
    from spmm_amd import _lib, gen
    from spmm_amd._lib import SpgCsr
    from spmm_amd.sparse import csr_matrix
    Ah, Bh = gen.scipy_pair(4096, 1.5e-3, seed=71)
    ref = oracle.spgemm(Ah, Bh, alpha=0.5, keep_zeros=True, sort=True)
    A, B = csr_matrix(Ah, device=_dev()), csr_matrix(Bh, device=_dev())
    h = _lib.get_handle(0)
    h.set_stream(torch.cuda.current_stream().cuda_stream)
    lib = h.lib

    def view(M):
        return SpgCsr(M.shape[0], M.shape[1], M.nnz, M.indptr.data_ptr(), M.indices.data_ptr(),
                      M.data.data_ptr(), _lib.SPG_INDEX_32I, _lib.SPG_R_64F)

    va, vb = view(A), view(B)
    al = ctypes.c_double(0.5)
    for alg in (_lib.SPG_ALG1, _lib.SPG_ALG2):
        wsb = ctypes.c_size_t(0)
        _lib.check(lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), alg, 0.2, ctypes.byref(wsb), None, None))
        ws = torch.empty(wsb.value, dtype=torch.uint8, device=_dev())
        indptr = torch.empty(4097, dtype=torch.int32, device=_dev())
        nnz, peak = ctypes.c_int64(0), ctypes.c_size_t(0)
        pj, px, plan = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(lib.spg_spgemm_ws(h.ptr, ctypes.byref(va), ctypes.byref(vb), alg, 0.2, ctypes.byref(al),
                                     ctypes.c_void_p(ws.data_ptr()), wsb.value, ctypes.c_void_p(indptr.data_ptr()),
                                     _lib.SPG_INDEX_32I, ctypes.byref(nnz), ctypes.byref(pj), ctypes.byref(px),
                                     ctypes.byref(peak), ctypes.byref(plan)))
        n = nnz.value
        assert n == len(ref[1]) and peak.value > 0
        if alg == _lib.SPG_ALG1:
            assert pj.value and px.value and not plan.value
            cj = ws[pj.value - ws.data_ptr():][:4 * n].view(torch.int32)
            cx = ws[px.value - ws.data_ptr():][:8 * n].view(torch.float64)
        else:
            assert not pj.value and plan.value
            cj = torch.empty(n, dtype=torch.int32, device=_dev())
            cx = torch.empty(n, dtype=torch.float64, device=_dev())
            vc = SpgCsr(4096, 4096, n, indptr.data_ptr(), cj.data_ptr(), cx.data_ptr(), _lib.SPG_INDEX_32I,
                        _lib.SPG_R_64F)
            _lib.check(lib.spg_numeric(h.ptr, plan, ctypes.byref(al), ctypes.byref(vc)))
            lib.spg_plan_destroy(plan)
        torch.cuda.synchronize()
        _assert_same((indptr.cpu().numpy().astype(np.int64), cj.cpu().numpy(), cx.cpu().numpy()), ref)


def _oracle_ref(A, B):
    return oracle.spgemm(A, B, keep_zeros=True, sort=True)


@pytest.mark.parametrize("alg", [1, 2])
def test_back_to_back_calls_stream_ordered(alg):
    """ALG1/ALG2 calls return once nnz(C) is known, with the numeric pass still queued
    (the scan mirrors its scalars into pinned memory).  Many back-to-back products with
    different shapes, all results held, read only after one synchronize: each must match
    its own oracle product."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    rng = np.random.default_rng(11)
    cases, outs = [], []
    for i in range(12):
        n = int(rng.integers(200, 3000))
        A = sp.random(n, n, density=float(rng.uniform(2e-3, 2e-2)), format="csr", random_state=100 + i)
        B = sp.random(n, n, density=float(rng.uniform(2e-3, 2e-2)), format="csr", random_state=200 + i)
        cases.append((A, B))
        outs.append(cusparse.spgemm(csr_matrix(A, device=_dev()), csr_matrix(B, device=_dev()), alg=alg))
    torch.cuda.synchronize()
    for (A, B), C in zip(cases, outs):
        got = (C.indptr.cpu().numpy().astype(np.int64), C.indices.cpu().numpy(), C.data.cpu().numpy())
        _assert_same(got, _oracle_ref(A, B))


def test_side_stream_and_stream_switch():
    """A product issued on a side stream is ordered on that stream (the handle follows
    torch's current stream; switching streams drains the old one first)."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    A = sp.random(4096, 4096, density=2e-3, format="csr", random_state=5)
    B = sp.random(4096, 4096, density=2e-3, format="csr", random_state=6)
    dA, dB = csr_matrix(A, device=_dev()), csr_matrix(B, device=_dev())
    ref = _oracle_ref(A, B)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())   # dA, dB were copied in on the default stream
    with torch.cuda.stream(s):
        C1 = cusparse.spgemm(dA, dB, alg=1)
        got1 = (C1.indptr.cpu().numpy().astype(np.int64), C1.indices.cpu().numpy(), C1.data.cpu().numpy())
    C2 = cusparse.spgemm(dA, dB, alg=1)   # back on the default stream
    torch.cuda.synchronize()
    _assert_same(got1, ref)
    _assert_same((C2.indptr.cpu().numpy().astype(np.int64), C2.indices.cpu().numpy(), C2.data.cpu().numpy()), ref)


def test_inputs_freed_while_side_stream_product_runs():
    """An ALG1 call returns while its numeric pass is still queued on the side stream.
    Inputs freed right after the call and their memory reused on another stream stay safe
    when the caller records the side stream on them (torch's rule for any stream-ordered
    library, cuSPARSE included): the caching allocator then holds the blocks until the
    side stream's work is done."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    A = sp.random(8192, 8192, density=1e-3, format="csr", random_state=11)
    B = sp.random(8192, 8192, density=1e-3, format="csr", random_state=12)
    ref = _oracle_ref(A, B)
    dA, dB = csr_matrix(A, device=_dev()), csr_matrix(B, device=_dev())
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        C = cusparse.spgemm(dA, dB, alg=1)
    for t in (dA.data, dA.indices, dA.indptr, dB.data, dB.indices, dB.indptr):
        t.record_stream(s)
    del dA, dB
    junk = [torch.full((1 << 20,), -1.0, dtype=torch.float64, device=_dev()) for _ in range(8)]
    torch.cuda.synchronize()
    del junk
    _assert_same((C.indptr.cpu().numpy().astype(np.int64), C.indices.cpu().numpy(), C.data.cpu().numpy()), ref)


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="needs two GPUs")
def test_product_on_non_current_device_keeps_current_device():
    """The library switches to the handle's device for a call and restores the caller's
    (cuSPARSE does not move the current device either)."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    A = sp.random(1024, 1024, density=1e-2, format="csr", random_state=1)
    torch.cuda.set_device(0)
    dA = csr_matrix(A, device="cuda:1")
    C = cusparse.spgemm(dA, dA, alg=2)
    assert torch.cuda.current_device() == 0
    torch.cuda.synchronize(1)
    _assert_same((C.indptr.cpu().numpy().astype(np.int64), C.indices.cpu().numpy(), C.data.cpu().numpy()),
                 _oracle_ref(A, A))


def test_alg1_lb_direct_path_bitexact(tmp_path):
    """The ALG1 numeric launch bounds every wait (its scan tiles' look-back, the rows' wait
    for their 64-row group prefix): a wait past the bound computes the prefix directly from
    the row counts.  SPG_LB_SPIN_TICKS=0 (read when a handle is created) sends EVERY wait down
    that path; config 2 through it must equal the oracle bit for bit, in a fresh process."""
    import os
    import subprocess
    import sys
    out = tmp_path / "c.npz"
    code = (
        "import numpy as np, torch, sys\n"
        f"sys.path.insert(0, {repr(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))})\n"
        "from spmm_amd import cusparse, gen\n"
        "from spmm_amd.sparse import csr_matrix\n"
        "A, B = gen.scipy_pair(16384, 1e-3, seed=42)\n"
        "C = cusparse.spgemm(csr_matrix(A, device='cuda:0'), csr_matrix(B, device='cuda:0'), alg=1)\n"
        "torch.cuda.synchronize()\n"
        f"np.savez({repr(str(out))}, p=C.indptr.cpu().numpy(), j=C.indices.cpu().numpy(), x=C.data.cpu().numpy())\n")
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SPG_LB_SPIN_TICKS="0"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    from spmm_amd import gen
    A, B = gen.scipy_pair(16384, 1e-3, seed=42)
    got = np.load(out)
    _assert_same((got["p"].astype(np.int64), got["j"], got["x"]), oracle.spgemm(A, B, keep_zeros=True, sort=True))


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("frac", [1.0, 0.3])
def test_tile_dense_negative_zero_products(frac, dtype):
    """Dense fp64 tiles start every accumulator slot at -0.0 and take the item's structure
    from the slots that left it (spgemm_tile_dn.hpp, dn_sent).  A column reached only by
    -0.0 products keeps -0.0 there while scipy's sum (from +0.0) is +0.0: such items take the
    re-walk path.  B values set to -0.0 (all of them, or 30 %) must still give the oracle's
    structure and +0.0 values, bit for bit."""
    from spmm_amd import gen
    A, B = gen.scipy_pair(2048, 0.02, seed=5, dtype=dtype)
    A.data = np.abs(A.data) + dtype(0.5)
    rng = np.random.default_rng(1)
    B.data = np.where(rng.random(B.nnz) < frac, dtype(-0.0), B.data).astype(dtype)
    for alg in (1, 2):
        _assert_same(_gpu(A, B, alg=alg), oracle.spgemm(A, B, keep_zeros=True, sort=True))


@pytest.mark.parametrize("n,density,neg", [(4096, 0.1, 0.0), (2048, 0.2, 0.3), (4096, 0.05, 0.0)])
def test_tile_fp32_entry_runs(n, density, neg):
    """fp32 dense tiles whose B segments hold >= 48 entries per 1024-column tile run
    k_tile_dn<float, .., 1024>: each A entry's run of a 64-product chunk adds with a plain LDS
    read-add-write (its columns are distinct), runs in entry order, the third and later runs of a
    chunk with one ordered ds_add_f32 (config 3 at density 0.1: 102-entry segments; 0.05: 51).
    Bit-exact against the oracle for ALG1 / ALG2 / chunked ALG3 and alpha != 1, with `neg` of
    B's values set to -0.0 (the -0.0 accumulator start and its re-walk), and equal to k_tile's
    owner rounds (SPG_F32_RUNS=0)."""
    from spmm_amd import gen
    A, B = gen.scipy_pair(n, density, seed=7, dtype=np.float32)
    if neg:
        A.data = np.abs(A.data) + np.float32(0.5)
        rng = np.random.default_rng(2)
        B.data = np.where(rng.random(B.nnz) < neg, np.float32(-0.0), B.data).astype(np.float32)
    ref = oracle.spgemm(A, B, alpha=1.5, keep_zeros=True, sort=True, threads=16)
    for alg, cf in [(1, 0.2), (2, 0.2), ("3c", 0.1)]:
        _assert_same(_gpu(A, B, alg=alg, alpha=1.5, cf=cf), ref)
    os.environ["SPG_F32_RUNS"] = "0"
    try:
        _assert_same(_gpu(A, B, alg=2, alpha=1.5), ref)
    finally:
        del os.environ["SPG_F32_RUNS"]
