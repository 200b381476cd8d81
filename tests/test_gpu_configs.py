"""BASELINE.json's GPU configurations at their full sizes, through the C ABI.

* Config 3 (dense_vs_sparseGEMM sweep, N = 8192): the upper half of the sweep in full,
  density 1e-2 and 1e-1 (ALG2), bit-exact against the CPU oracle over every row (the OpenMP
  oracle for 1e-1: 5.5e9 products).
* Config 4 (N = 65536, density 5e-3, ALG3 chunked): nnz(C) = 3.46e9 needs an int64 row
  pointer.  >= 2048 stratified rows bit-exact against the oracle (the first and last rows of
  every ALG3 chunk, the longest A and C rows, rows with a tile item past one accumulator
  window, uniform fill), plus size-independent properties
  over the whole result: int64 row pointer, monotone, row_ptr[-1] = nnz(C) within the
  analytic expectation, every row's columns strictly increasing and in range, no row longer
  than its product count or N, and P (getNumProducts) equal to sum over A's entries of the
  B row lengths.
* Config 5 on one GPU (N = 262144, density 1e-3, ALG2 and ALG3): the same checks (200 GB of
  C and workspace fit the 288 GB of one MI355X).
* ALG3's working-set cap on a sparse-tile shape: peak bytes fall as chunk_fraction falls,
  with bit-identical results; on dense tiles ALG3 stays within ALG2's peak.

Inputs of configs 4/5 are generated on the device (spmm_amd.gen.random_csr); the oracle
sees only the sampled rows of A (and all of B).
"""

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEV = "cuda:0"
THREADS = 16   # the GPU box's CPU share


def _bits(x):
    return x.view(np.uint32 if x.dtype == np.float32 else np.uint64)


def _full_bitexact(Ah, Bh, alg, cf=0.2, threads=0):
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    C = cusparse.spgemm(csr_matrix(Ah, device=DEV), csr_matrix(Bh, device=DEV), alg=alg, chunk_fraction=cf)
    torch.cuda.synchronize()
    rp, rj, rx = oracle.spgemm(Ah, Bh, keep_zeros=True, sort=True, threads=threads)
    assert np.array_equal(C.indptr.cpu().numpy().astype(np.int64), rp), "row pointer"
    assert np.array_equal(C.indices.cpu().numpy(), rj), "column indices"
    assert np.array_equal(_bits(C.data.cpu().numpy()), _bits(rx)), "values"
    return C


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("density", [1e-2, 1e-1])
def test_config3_full_bitexact(density, dtype):
    """fp32 at density 0.1 is bench.py's `config3_fp32` point (the fp32 entry-run kernel)."""
    from spmm_amd import gen
    Ah, Bh = gen.scipy_pair(8192, density, seed=42, dtype=dtype)
    C = _full_bitexact(Ah, Bh, alg=2, threads=THREADS if density >= 0.1 else 0)
    if density >= 0.1:
        assert C.nnz == 8192 * 8192   # every entry of C is reached at density 0.1


def test_config3_fp32_bench_matrices_bitexact():
    """The exact matrices of bench.py's `config3_fp32` key (gen.random_csr on the device, seeds
    42 and 43, fp32, N = 8192, density 0.1): every row bit-exact against the OpenMP oracle."""
    from spmm_amd import cusparse, gen
    A = gen.random_csr(8192, 8192, 0.1, seed=42, dtype=torch.float32, device=DEV)
    B = gen.random_csr(8192, 8192, 0.1, seed=43, dtype=torch.float32, device=DEV)
    C = cusparse.spgemm(A, B, alg=2)
    torch.cuda.synchronize()
    rp, rj, rx = oracle.spgemm(A.get(), B.get(), keep_zeros=True, sort=True, threads=THREADS)
    assert np.array_equal(C.indptr.cpu().numpy().astype(np.int64), rp)
    assert np.array_equal(C.indices.cpu().numpy(), rj)
    assert np.array_equal(_bits(C.data.cpu().numpy()), _bits(rx))


def _expected_nnz(a_lens, n, density):
    """E[nnz(C)] for B with independent uniform columns: sum_i n (1 - (1 - d)^{a_i})."""
    a = a_lens.astype(np.float64)
    return float(np.sum(n * (1.0 - np.power(1.0 - density, a))))


@torch.no_grad()
def _check_structure(A, B, C, n, density, tile_width, record_group=1):
    """Size-independent properties of C over every row (device-side, in row chunks).
    Returns (P, per-row nnz(C) on the host, rows with a tile item over TILE_CAP entries)."""
    m = A.shape[0]
    p = C.indptr
    assert p.dtype == torch.int64, "nnz(C) >= 2^31 needs an int64 row pointer"
    assert int(p[0]) == 0 and int(p[-1]) == C.nnz
    lens = p[1:] - p[:-1]
    assert bool((lens >= 0).all()), "row pointer not monotone"
    # P = sum over A's entries of B's row lengths; every row holds <= min(P_i, n) entries
    blen = (B.indptr[1:] - B.indptr[:-1]).to(torch.int64)
    prod = blen[A.indices.to(torch.int64)]
    rows = torch.repeat_interleave(torch.arange(m, device=p.device),
                                   (A.indptr[1:] - A.indptr[:-1]).to(torch.int64))
    P_i = torch.zeros(m, dtype=torch.int64, device=p.device).index_add_(0, rows, prod)
    assert bool((lens <= torch.clamp(P_i, max=n)).all())
    # nnz(C) against its expectation (relative std ~1e-5 at these sizes)
    exp = _expected_nnz((A.indptr[1:] - A.indptr[:-1]).cpu().numpy(), n, density)
    assert abs(C.nnz - exp) / exp < 2e-3, (C.nnz, exp)
    # columns in range and strictly increasing inside every row; entries per (row, tile)
    G = (n + tile_width - 1) // tile_width
    over_cap = []
    step = max(1, int(4e8 // max(1, C.nnz // m)))   # ~4e8 entries per chunk
    for r0 in range(0, m, step):
        r1 = min(m, r0 + step)
        s, e = int(p[r0]), int(p[r1])
        if e <= s:
            continue
        cols = C.indices[s:e]
        lo, hi = torch.aminmax(cols)
        assert int(lo) >= 0 and int(hi) < n
        start = torch.zeros(e - s, dtype=torch.bool, device=cols.device)
        start[(p[r0:r1] - s)[lens[r0:r1] > 0]] = True
        ok = (cols[1:] > cols[:-1]) | start[1:]
        assert bool(ok.all()), f"columns not increasing in rows [{r0}, {r1})"
        rid = torch.repeat_interleave(torch.arange(r1 - r0, device=cols.device), lens[r0:r1])
        items = torch.bincount(rid * G + (cols // tile_width).to(torch.int64), minlength=(r1 - r0) * G)
        big = torch.nonzero(items.view(r1 - r0, G).max(dim=1).values > window_cap(tile_width, record_group)).flatten() + r0
        over_cap.append(big.cpu().numpy())
        del cols, start, ok, rid, items
    return int(P_i.sum()), lens.cpu().numpy(), np.concatenate(over_cap) if over_cap else np.zeros(0, np.int64)


TILE_CAP = 1024   # entries of one tile-item accumulator window (spgemm_tile.hpp)


def window_cap(tile_width, record_group=1):
    """Accumulator window of a sparse tile item: on 8192-column tiles 2048 slots
    (k_tile_sp<double, .., SpCfg2048, 1>) or, in cooperative record groups, 2032
    (SpCfgRG: two 4-wave blocks per CU); else TILE_CAP."""
    if tile_width == 8192:
        return 2032 if record_group > 1 else 2048
    return TILE_CAP


def _stratified_rows(A, C_lens, chunk_rows, over_cap, total=2048, seed=0):
    """Rows where the schedule changes, then uniform ones up to `total`:
    * the first and last row of every row chunk (ALG3's chunk cut) and their neighbours;
    * the longest A rows and the largest C rows;
    * rows with a tile item past its accumulator window (windowed items, sparse tiles);
    * the first and last rows of the matrix."""
    m = A.shape[0]
    a_lens = (A.indptr[1:] - A.indptr[:-1]).cpu().numpy()
    pick = set()
    for r in chunk_rows:
        for d in (-2, -1, 0, 1):
            if 0 <= r + d < m:
                pick.add(r + d)
    pick.update(np.argsort(a_lens)[-32:].tolist())
    pick.update(np.argsort(C_lens)[-32:].tolist())
    pick.update(np.argsort(C_lens)[:16].tolist())
    rng = np.random.default_rng(seed)
    if len(over_cap):
        pick.update(rng.choice(over_cap, size=min(len(over_cap), 512), replace=False).tolist())
    pick.update([0, 1, m - 2, m - 1])
    rest = np.setdiff1d(np.arange(m), np.fromiter(pick, np.int64))
    pick.update(rng.choice(rest, size=max(0, total - len(pick)), replace=False).tolist())
    return np.array(sorted(pick), dtype=np.int64)


@torch.no_grad()
def _sampled_bitexact(A, B, C, rows):
    """The sampled rows of C against the oracle on the same rows of A (all of B), bit for bit:
    the rows' entries gathered on the device in one index op, one copy to the host."""
    Ah, Bh = A.get(), B.get()
    rp, rj, rx = oracle.spgemm(sp.csr_matrix(Ah[rows]), Bh, keep_zeros=True, sort=True, threads=THREADS)
    p = C.indptr
    tr = torch.from_numpy(rows).to(p.device)
    s, e = p[tr], p[tr + 1]
    got_lens = (e - s).cpu().numpy()
    bad = np.nonzero(got_lens != np.diff(rp))[0]
    assert len(bad) == 0, f"nnz differs in rows {rows[bad[:8]].tolist()}"
    idx = torch.repeat_interleave(s, e - s) + (torch.arange(int((e - s).sum()), device=p.device)
                                               - torch.repeat_interleave(torch.cumsum(e - s, 0) - (e - s), e - s))
    gj = C.indices[idx].cpu().numpy()
    gx = C.data[idx].cpu().numpy()
    if not np.array_equal(gj, rj):
        q = int(np.searchsorted(rp, int(np.nonzero(gj != rj)[0][0]), side="right") - 1)
        raise AssertionError(f"row {rows[q]}: columns")
    if not np.array_equal(_bits(gx), _bits(rx)):
        q = int(np.searchsorted(rp, int(np.nonzero(_bits(gx) != _bits(rx))[0][0]), side="right") - 1)
        raise AssertionError(f"row {rows[q]}: values")


@pytest.mark.parametrize("n,density,alg,cf,expect_products,chunks", [
    (65536, 5e-3, 3, 0.2, 7.04e9, 1),      # config 4: the workspace is within ALG3's cap, one chunk
    (262144, 1e-3, 2, 0.2, 1.80e10, 1),    # config 5, one GPU
    (262144, 1e-3, 3, 0.02, 1.80e10, 50),  # config 5, ALG3 chunked (sparse tiles: the cap binds)
])
def test_large_config_stratified_and_properties(n, density, alg, cf, expect_products, chunks):
    """Configs 4 and 5 at full size: whole-result properties over every row, and >= 2048
    stratified rows (ALG3 chunk boundaries, extreme A/C rows, windowed tile items, uniform
    fill) bit-exact against the oracle."""
    from spmm_amd import cusparse, gen
    A = gen.random_csr(n, n, density, seed=42, device=DEV)
    B = gen.random_csr(n, n, density, seed=43, device=DEV)
    info = cusparse.plan_info(A, B, alg=alg, chunk_fraction=cf)
    assert info["path"] == "tile"
    # ALG3 chunks only when the unchunked workspace exceeds chunk_fraction of the single-pass
    # buffer (P entries of C); then at least ceil(1/chunk_fraction) chunks of equal products
    assert len(info["chunk_rows"]) - 1 >= chunks if chunks > 1 else len(info["chunk_rows"]) == 2, info
    C = cusparse.spgemm(A, B, alg=alg, chunk_fraction=cf)
    torch.cuda.synchronize()
    P, C_lens, over_cap = _check_structure(A, B, C, n, density, info["tile_width"],
                                          info.get("record_group", 1))
    assert P == cusparse.num_products(A, B)
    assert abs(P - expect_products) / expect_products < 0.02
    rows = _stratified_rows(A, C_lens, info["chunk_rows"], over_cap)
    assert len(rows) >= 2048
    _sampled_bitexact(A, B, C, rows)
    del C
    torch.cuda.empty_cache()


def test_alg3_peak_falls_with_chunk_fraction():
    """ALG3 caps the tile path's working set where it has one: on sparse tiles (4096-column
    tiles, compact windows) the symbolic bitmaps are sized by the largest chunk and reused
    chunk by chunk, so peak bytes fall as chunk_fraction falls, the result does not change
    (the reference's alg3.cu:195-202 / BASELINE.md 1a behaviour)."""
    from spmm_amd import cusparse, gen
    from spmm_amd.sparse import csr_matrix
    Ah, Bh = gen.scipy_pair(32768, 1e-3, seed=42)
    A, B = csr_matrix(Ah, device=DEV), csr_matrix(Bh, device=DEV)
    peaks, ref = [], None
    for cf in (1.0, 0.2, 0.05):
        C = cusparse.spgemm(A, B, alg=3, chunk_fraction=cf)
        torch.cuda.synchronize()
        peaks.append(cusparse.last_stats.peak_bytes)
        got = (C.indptr.cpu().numpy(), C.indices.cpu().numpy(), _bits(C.data.cpu().numpy()))
        if ref is None:
            ref = got
        else:
            assert all(np.array_equal(x, y) for x, y in zip(got, ref)), f"cf={cf} changed C"
    assert peaks[0] > peaks[1] > peaks[2], peaks
    # the workspace part (peak minus C's arrays) shrinks by at least 1.5x from cf=1 to
    # cf=0.05 (what stays is the tile-major copy of B, independent of cf)
    c_bytes = 12 * len(ref[1]) + 4 * len(ref[0])
    assert (peaks[2] - c_bytes) * 1.5 <= (peaks[0] - c_bytes), (peaks, c_bytes)
    rp, rj, rx = oracle.spgemm(Ah[:512], Bh, keep_zeros=True, sort=True)
    assert np.array_equal(ref[0][:513].astype(np.int64), rp) and np.array_equal(ref[1][:rp[-1]], rj)
    assert np.array_equal(ref[2][:rp[-1]], _bits(rx))


def test_alg3_dense_tiles_within_alg2_peak():
    """On dense tiles (<= 1024 columns: config 4's shape) an item keeps only its 8-byte
    offset -- the numeric tiles take the structure from their accumulation -- so there is
    no per-chunk working set left to cap: every chunk_fraction gives the same C as ALG2,
    at no more memory, without recomputing the chunks' counts."""
    from spmm_amd import cusparse, gen
    from spmm_amd.sparse import csr_matrix
    Ah, Bh = gen.scipy_pair(8192, 1e-2, seed=42)
    A, B = csr_matrix(Ah, device=DEV), csr_matrix(Bh, device=DEV)
    C2 = cusparse.spgemm(A, B, alg=2)
    torch.cuda.synchronize()
    peak2 = cusparse.last_stats.peak_bytes
    ref = (C2.indptr.cpu().numpy(), C2.indices.cpu().numpy(), _bits(C2.data.cpu().numpy()))
    del C2
    for cf in (1.0, 0.2, 0.05):
        C = cusparse.spgemm(A, B, alg=3, chunk_fraction=cf)
        torch.cuda.synchronize()
        assert cusparse.last_stats.peak_bytes <= peak2 * 1.01, (cf, cusparse.last_stats.peak_bytes, peak2)
        got = (C.indptr.cpu().numpy(), C.indices.cpu().numpy(), _bits(C.data.cpu().numpy()))
        assert all(np.array_equal(x, y) for x, y in zip(got, ref)), f"cf={cf} changed C"
