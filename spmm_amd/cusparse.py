"""``spgemm`` -- the drop-in for ``cupyx.cusparse.spgemm`` (the reference's hot-path
boundary, modify_src/cupy-src/cupyx/cusparse.py:2007-2142), backed by libmi355_spgemm.so.

Same signature, argument meaning and error behaviour as the reference:

* ``RuntimeError('spgemm is not available.')`` when the engine cannot run
  (``check_availability``, cusparse.py:169-186 / :2022-2023);
* ``TypeError`` for a non-CSR operand (:2026-2029), ``ValueError('mismatched shape')``
  (:2032-2033), ``assert a.has_canonical_format`` (:2030-2031);
* dtype promotion of the operands (``_cast_common_type``, :52-56);
* ``alg``: 1 -> ALG1 (single pass), 2 -> ALG2 (two phase), 3 -> ALG3 (chunked two phase,
  uses ``chunk_fraction``), anything else -> the library default.  Note: the reference maps
  ``alg=1`` to CUSPARSE_SPGEMM_DEFAULT (cusparse.py:2056-2057) while its C++ "ALG1" driver
  uses CUSPARSE_SPGEMM_ALG1; here ``alg=1`` always means ALG1.
* ``verbose`` prints the workspace size like the reference prints buff2 (:2106-2107).

Device memory comes from torch's caching allocator on the current device; work runs on the
current torch stream.  The result's ``indptr`` is int32 when nnz(C) < 2**31, int64 beyond.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _fastpath, _lib
from ._lib import SpgCsr, SpgError, check
from .sparse import csr_matrix

_VT = {torch.float32: _lib.SPG_R_32F, torch.float64: _lib.SPG_R_64F,
       torch.complex64: _lib.SPG_C_32F, torch.complex128: _lib.SPG_C_64F}
# host alpha of C's value type: one scalar, or a (real, imag) pair for complex
_ALPHA_CT = {torch.float32: (ctypes.c_float, 1), torch.float64: (ctypes.c_double, 1),
             torch.complex64: (ctypes.c_float, 2), torch.complex128: (ctypes.c_double, 2)}
_IT = {torch.int32: _lib.SPG_INDEX_32I, torch.int64: _lib.SPG_INDEX_64I}
_ALG = {1: _lib.SPG_ALG1, 2: _lib.SPG_ALG2, 3: _lib.SPG_ALG3}


@dataclass
class SpgemmStats:
    """Accounting of the last spgemm call on this process (for the profilers)."""
    alg: int = 0
    workspace_bytes: int = 0
    peak_bytes: int = 0        # workspace + C (spg_peak_bytes)
    num_products: int = -1
    nnz: int = 0


last_stats = SpgemmStats()


_available = None


def check_availability(name: str) -> bool:
    """True when the named routine can run here (a gfx950 device and the built library).
    Memoized like the reference's ``@_util.memoize()`` check (cusparse.py:169-186)."""
    global _available
    if name not in ("spgemm", "spmv", "validate_csr"):
        raise ValueError(f"No available version information specified for {name}")
    if _available is None:
        try:
            _available = bool(torch.cuda.is_available())
            if _available:
                _lib.get_handle(torch.cuda.current_device())
        except Exception:
            _available = False
    return _available


def _csr_view(m: csr_matrix) -> SpgCsr:
    return SpgCsr(m.shape[0], m.shape[1], m.nnz, m.indptr.data_ptr(),
                  m.indices.data_ptr() if m.nnz else 0, m.data.data_ptr() if m.nnz else 0,
                  _IT[m.indptr.dtype], _VT[m.data.dtype])


def _current_stream_ptr(dev: int) -> int:
    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)   # (no Stream object per call)
    return raw(dev) if raw is not None else torch.cuda.current_stream(dev).cuda_stream


def _handle_for(m: csr_matrix) -> _lib.Handle:
    d = m.device
    dev = d.index if d.index is not None else torch.cuda.current_device()
    h = _lib.get_handle(dev)
    h.set_stream(_current_stream_ptr(dev))
    return h


def validate_csr(m: csr_matrix) -> int:
    """1 canonical, 0 unsorted/duplicates, -1 malformed (spg_validate_csr)."""
    if m.device.type != "cuda":
        raise RuntimeError("validate_csr needs device-resident operands")
    h = _handle_for(m)
    v = _csr_view(m)
    res = ctypes.c_int(0)
    check(h.lib.spg_validate_csr(h.ptr, ctypes.byref(v), ctypes.byref(res)), "spg_validate_csr")
    return res.value


def _cols16_nb1(cols: int) -> int:
    """Interior 65536-column block starts per row (include/spgemm.h, spg_cols16_*)."""
    return max(0, -(-int(cols) // 65536) - 1)


def _cols16_split(m: csr_matrix):
    """(block_starts int32 [rows, nb1], lo16 int16 [nnz]) of a device CSR (spg_cols16_split)."""
    rows, nb1 = m.shape[0], _cols16_nb1(m.shape[1])
    starts = torch.empty((rows, nb1), dtype=torch.int32, device=m.device)
    lo16 = torch.empty(m.nnz, dtype=torch.int16, device=m.device)
    h = _handle_for(m)
    v = SpgCsr(rows, m.shape[1], m.nnz, m.indptr.data_ptr(), m.indices.data_ptr() if m.nnz else 0, 0,
               _IT[m.indptr.dtype], _VT[torch.float64])
    check(h.lib.spg_cols16_split(h.ptr, ctypes.byref(v), ctypes.c_void_p(starts.data_ptr() if starts.numel() else 0),
                                 ctypes.c_void_p(lo16.data_ptr() if m.nnz else 0)), "spg_cols16_split")
    return starts, lo16


def _cols16_join(indptr: torch.Tensor, starts: torch.Tensor, lo16: torch.Tensor, shape) -> torch.Tensor:
    """int32 column indices from a device (indptr, block starts, low halves) (spg_cols16_join)."""
    rows, cols = shape
    nnz = lo16.numel()
    out = torch.empty(nnz, dtype=torch.int32, device=indptr.device)
    dev = indptr.device.index if indptr.device.index is not None else torch.cuda.current_device()
    h = _lib.get_handle(dev)
    h.set_stream(_current_stream_ptr(dev))
    v = SpgCsr(rows, cols, nnz, indptr.data_ptr(), out.data_ptr() if nnz else 0, 0, _IT[indptr.dtype],
               _VT[torch.float64])
    check(h.lib.spg_cols16_join(h.ptr, ctypes.byref(v), ctypes.c_void_p(starts.data_ptr() if starts.numel() else 0),
                                ctypes.c_void_p(lo16.data_ptr() if nnz else 0)), "spg_cols16_join")
    return out


_VALUE_DTYPES = (torch.float32, torch.float64, torch.complex64, torch.complex128)


def _cast_common_type(a: csr_matrix, b: csr_matrix):
    if a.data.dtype is b.data.dtype and a.data.dtype in _VALUE_DTYPES:   # (the per-call common case)
        return a, b
    dt = np.promote_types(a.dtype, b.dtype)
    if dt not in (np.float32, np.float64, np.complex64, np.complex128):
        raise TypeError(f"spgemm supports float32/float64/complex64/complex128, got {dt}")
    return a.astype(dt), b.astype(dt)


def spgemm(a, b, alpha=1, alg=0, chunk_fraction=0.2, verbose=False):
    """Matrix-matrix product for CSR matrices: ``C = alpha * A * B``.

    Args:
        a (csr_matrix): sparse matrix A (m x k), canonical format.
        b (csr_matrix): sparse matrix B (k x n), canonical format.
        alpha (scalar): coefficient.
        alg (int): 1, 2, 3 select ALG1/ALG2/ALG3; other values the default.
        chunk_fraction (float): ALG3 chunk size as a fraction of the products, (0, 1].
        verbose (bool): print the workspace size.

    Returns:
        csr_matrix: C, with sorted column indices and structural entries kept.
    """
    return _spgemm(a, b, alpha, alg, chunk_fraction, verbose)


def _spgemm(a, b, alpha=1, alg=0, chunk_fraction=0.2, verbose=False, before_numeric=None, by_tiles=None,
            values_first=True):
    """spgemm, plus `before_numeric`: a callable run after the symbolic pass and before the
    numeric pass reads the values (the multi-GPU path waits there for B's values to arrive
    over RCCL; spmm_amd.distributed).  With it the call takes the ctypes path (the native
    shim runs both passes in one call); ALG1 runs it first (its count and numeric passes
    are queued together).

    `by_tiles(geom)`: the numeric pass by column-tile groups (spg_numeric_tiles), called
    exactly once per product, BEFORE the symbolic pass (the plan's tile layout needs only
    B's structure, so B's values can travel while the symbolic pass runs; _spgemm_by_tiles;
    ``values_first=False``: after it, round 4's order, for the bench's comparison).
    `geom` is None when the plan cannot
    run by tiles (not the tile path, several row chunks, ALG1); then `by_tiles` makes
    b.data complete and returns None, and spg_numeric runs.  Otherwise geom is a dict
    (tile_width, tiles, offsets: the tiles + 1 tile-major value offsets, tile_values(): B's
    values permuted tile-major by this plan, dtype: the plan's value type) and `by_tiles` returns (tm, groups): the
    tile-major values tensor and an iterable of (tile_begin, tile_end) ranges, each yielded
    once its slice of tm is ready on the current stream, together covering every tile."""
    if not check_availability("spgemm"):
        raise RuntimeError("spgemm is not available.")
    assert a.ndim == b.ndim == 2
    if not isinstance(a, csr_matrix):
        raise TypeError("unsupported type (actual: {})".format(type(a)))
    if not isinstance(b, csr_matrix):
        raise TypeError("unsupported type (actual: {})".format(type(b)))
    assert a.has_canonical_format
    assert b.has_canonical_format
    if a.shape[1] != b.shape[0]:
        raise ValueError("mismatched shape")
    if a.device != b.device:
        raise ValueError("operands are on different devices")

    m, _ = a.shape
    _, n = b.shape
    a, b = _cast_common_type(a, b)
    if a.indptr.dtype != b.indptr.dtype:   # the engine takes one row-pointer type for A and B
        a = csr_matrix((a.data, a.indices, a.indptr.to(torch.int64)), shape=a.shape, canonical=True)
        b = csr_matrix((b.data, b.indices, b.indptr.to(torch.int64)), shape=b.shape, canonical=True)
        a.indptr, b.indptr = a.indptr.to(torch.int64), b.indptr.to(torch.int64)
    algo = _ALG.get(alg, _lib.SPG_ALG_DEFAULT)
    if algo == _lib.SPG_ALG3 and not (0.0 < float(chunk_fraction) <= 1.0):
        raise ValueError(f"chunk_fraction must be in (0,1], got {chunk_fraction}")

    dev = a.device
    h = _handle_for(a)
    cf = float(chunk_fraction)
    fp = _fastpath.get() if before_numeric is None and by_tiles is None else None
    if before_numeric is not None and algo == _lib.SPG_ALG1:
        before_numeric()
        before_numeric = None
    if by_tiles is not None and algo == _lib.SPG_ALG1:
        if by_tiles(None) is not None:
            raise RuntimeError("by_tiles must complete B's values when geom is None")
        by_tiles = None
    if by_tiles is not None:
        return _spgemm_by_tiles(h, a, b, alpha, algo, cf, by_tiles, verbose, values_first)
    if fp is not None:   # the same sequence in one native call (csrc/fastpath.cpp)
        al = complex(alpha)
        st, data, indices, indptr, wsb, peak = fp.spgemm(
            h.ptr.value, m, a.shape[1], n, a.indptr, a.indices, a.data, b.indptr, b.indices, b.data,
            int(algo), cf, al.real, al.imag)
        check(st, "spg_spgemm_ws")
        if verbose:
            print("USING ALG", alg, "workspace GB =", wsb / (1024 ** 3))
        last_stats.alg, last_stats.workspace_bytes = int(algo), int(wsb)
        last_stats.peak_bytes, last_stats.nnz = int(peak), int(indices.numel())
        return csr_matrix._from_parts(data, indices, indptr, (m, n), canonical=True)
    lib = h.lib
    va, vb = _csr_view(a), _csr_view(b)
    ws_bytes = ctypes.c_size_t(0)
    check(lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), algo, cf,
                       ctypes.byref(ws_bytes), None, None), "spg_plan")
    if verbose:
        print("USING ALG", alg, "workspace GB =", ws_bytes.value / (1024 ** 3))
    # workspace from torch's caching allocator on the current stream (the library works on
    # that stream, so a later reuse of the block is ordered after this product)
    ws = torch.empty(max(ws_bytes.value, 1), dtype=torch.uint8, device=dev)
    ct, nparts = _ALPHA_CT[a.data.dtype]
    al = (ct * 2)(complex(alpha).real, complex(alpha).imag) if nparts == 2 else ct(float(alpha))
    nnz, peak = ctypes.c_int64(0), ctypes.c_size_t(0)
    pj, px, plan = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    # plan -> symbolic (nnz(C) to the host) -> numeric in one call (spg_spgemm_ws)
    # int64 row pointer once nnz(C) >= 2**31; int64 first when the expected product count
    # reaches 2**31 (an overflowing int32 try would redo the plan and the symbolic pass)
    wide = a.nnz * (b.nnz / max(b.shape[0], 1)) >= 2 ** 31
    for it in ((torch.int64,) if wide else (torch.int32, torch.int64)):
        indptr = torch.empty(m + 1, dtype=it, device=dev)
        st = lib.spg_spgemm_ws(h.ptr, ctypes.byref(va), ctypes.byref(vb), algo, cf, ctypes.byref(al),
                               ctypes.c_void_p(ws.data_ptr()), ws_bytes.value,
                               ctypes.c_void_p(indptr.data_ptr()), _IT[it], ctypes.byref(nnz),
                               ctypes.byref(pj), ctypes.byref(px), ctypes.byref(peak), ctypes.byref(plan))
        if st != _lib.STATUS_OVERFLOW:
            break
    check(st, "spg_spgemm_ws")
    nnzc = int(nnz.value)
    if pj.value:
        # ALG1: C sits compact (scaled) in the workspace -- views of it
        base = ws.data_ptr()
        oj, ox = pj.value - base, px.value - base
        indices = ws[oj:oj + 4 * nnzc].view(torch.int32)
        data = ws[ox:ox + a.data.element_size() * nnzc].view(a.data.dtype)
    else:
        try:
            indices = torch.empty(nnzc, dtype=torch.int32, device=dev)
            data = torch.empty(nnzc, dtype=a.data.dtype, device=dev)
            vc = SpgCsr(m, n, nnzc, indptr.data_ptr(), indices.data_ptr() if nnzc else 0,
                        data.data_ptr() if nnzc else 0, _IT[indptr.dtype], _VT[data.dtype])
            if before_numeric is not None:
                before_numeric()
            check(lib.spg_numeric(h.ptr, plan, ctypes.byref(al), ctypes.byref(vc)), "spg_numeric")
        finally:
            lib.spg_plan_destroy(plan)
    if wide and nnzc < 2 ** 31:
        indptr = indptr.to(torch.int32)   # the int32 contract when the result fits
    last_stats.alg, last_stats.workspace_bytes = int(algo), int(ws_bytes.value)
    last_stats.peak_bytes, last_stats.nnz = int(peak.value), nnzc
    return csr_matrix._from_parts(data, indices, indptr, (m, n), canonical=True)


def _alpha_of(dtype, alpha):
    ct, nparts = _ALPHA_CT[dtype]
    return (ct * 2)(complex(alpha).real, complex(alpha).imag) if nparts == 2 else ct(float(alpha))


def _spgemm_by_tiles(h, a, b, alpha, algo, cf, by_tiles, verbose, values_first=True):
    """_spgemm with `by_tiles` (the row-block step of spmm_amd.distributed): spg_plan, then
    the tile geometry -- spg_tile_value_offsets builds the plan's tile layout from B's
    structure alone -- and ``by_tiles(geom)``, which starts B's values travelling group by
    group; only then spg_symbolic, which runs while they arrive, and the numeric tiles of
    each group as it is released (spg_numeric after the row-major fallback)."""
    lib = h.lib
    m, n = a.shape[0], b.shape[1]
    dev = a.device
    va, vb = _csr_view(a), _csr_view(b)
    ws_bytes = ctypes.c_size_t(0)
    check(lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), algo, cf, ctypes.byref(ws_bytes), None, None),
          "spg_plan")
    if verbose:
        print("USING ALG", algo, "workspace GB =", ws_bytes.value / (1024 ** 3))
    ws = torch.empty(max(ws_bytes.value, 1), dtype=torch.uint8, device=dev)
    plan = ctypes.c_void_p()
    check(lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), algo, cf, ctypes.byref(ws_bytes),
                       ctypes.c_void_p(ws.data_ptr()), ctypes.byref(plan)), "spg_plan")
    al = _alpha_of(a.data.dtype, alpha)
    try:
        if values_first:
            geom = _tile_geometry(h, plan, b)
            got = by_tiles(geom)
        nnz = ctypes.c_int64(0)
        wide = a.nnz * (b.nnz / max(b.shape[0], 1)) >= 2 ** 31
        for it in ((torch.int64,) if wide else (torch.int32, torch.int64)):
            indptr = torch.empty(m + 1, dtype=it, device=dev)
            st = lib.spg_symbolic(h.ptr, plan, ctypes.c_void_p(indptr.data_ptr()), _IT[it], ctypes.byref(nnz))
            if st != _lib.STATUS_OVERFLOW:
                break
        check(st, "spg_symbolic")
        if not values_first:
            geom = _tile_geometry(h, plan, b)
            got = by_tiles(geom)
        if got is not None and geom is None:
            raise RuntimeError("by_tiles returned tile groups for a plan that cannot run by tiles")
        nnzc = int(nnz.value)
        indices = torch.empty(nnzc, dtype=torch.int32, device=dev)
        data = torch.empty(nnzc, dtype=a.data.dtype, device=dev)
        vc = SpgCsr(m, n, nnzc, indptr.data_ptr(), indices.data_ptr() if nnzc else 0,
                    data.data_ptr() if nnzc else 0, _IT[indptr.dtype], _VT[data.dtype])
        if got is None:
            check(lib.spg_numeric(h.ptr, plan, ctypes.byref(al), ctypes.byref(vc)), "spg_numeric")
        else:
            _numeric_groups(h, plan, al, vc, got, geom)
        peak = ctypes.c_size_t(0)
        check(lib.spg_peak_bytes(plan, ctypes.byref(peak)), "spg_peak_bytes")
    finally:
        lib.spg_plan_destroy(plan)
    if wide and nnzc < 2 ** 31:
        indptr = indptr.to(torch.int32)   # the int32 contract when the result fits
    last_stats.alg, last_stats.workspace_bytes = int(algo), int(ws_bytes.value)
    last_stats.peak_bytes, last_stats.nnz = int(peak.value), nnzc
    return csr_matrix._from_parts(data, indices, indptr, (m, n), canonical=True)


def _tile_geometry(h, plan, b):
    """The by_tiles geometry of a plan (see _spgemm), or None when it cannot run by tiles."""
    lib = h.lib
    info = _lib.SpgPlanInfo()
    check(lib.spg_plan_info(plan, ctypes.byref(info), None, 0), "spg_plan_info")
    # (a development library built without the tile-group entry points: spg_numeric)
    has_tiles = all(hasattr(lib, f) for f in ("spg_tile_value_offsets", "spg_tile_values", "spg_numeric_tiles"))
    if not (has_tiles and info.path == 2 and info.n_chunks == 1):
        return None
    # value tiles: record_group adjacent numeric tiles (include/spgemm.h)
    rg = max(1, int(info.record_group))
    G = (int(info.tiles_per_row) + rg - 1) // rg
    offs = (ctypes.c_int64 * (G + 1))()
    st = lib.spg_tile_value_offsets(h.ptr, plan, offs, G + 1)
    if st == _lib.STATUS_NOT_SUPPORTED:
        return None
    check(st, "spg_tile_value_offsets")

    def tile_values():
        tm = torch.empty(max(b.nnz, 1), dtype=b.data.dtype, device=b.data.device)
        check(lib.spg_tile_values(h.ptr, plan, ctypes.c_void_p(tm.data_ptr())), "spg_tile_values")
        return tm[:b.nnz]
    return {"tile_width": int(info.tile_width) * rg, "tiles": G,
            "offsets": np.frombuffer(offs, dtype=np.int64).copy(), "tile_values": tile_values,
            "dtype": b.data.dtype}


def _numeric_groups(h, plan, al, vc, got, geom):
    """spg_numeric_tiles for each (tile_begin, tile_end) group `by_tiles` releases."""
    tm, groups = got
    covered = 0
    for g0, g1 in groups:
        if g0 != covered:
            raise RuntimeError(f"tile groups must be consecutive: expected {covered}, got {g0}")
        check(h.lib.spg_numeric_tiles(h.ptr, plan, ctypes.byref(al), ctypes.byref(vc),
                                      ctypes.c_void_p(tm.data_ptr() if tm.numel() else 0), int(g0), int(g1)),
              "spg_numeric_tiles")
        covered = g1
    if covered != geom["tiles"]:
        raise RuntimeError(f"tile groups covered {covered} of {geom['tiles']} tiles")


def spmv(a, x, y=None, alpha=1, beta=0, transa=False):
    """y = alpha * op(A) x + beta * y -- the drop-in for ``cupyx.cusparse.spmv``
    (modify_src/cupy-src/cupyx/cusparse.py:1373-1432), on ``spg_spmv``.

    A is csr_matrix, csc_matrix or coo_matrix (CSC goes through its transpose as the
    reference does, COO through CSR).  x, y are 1-D tensors (or numpy arrays, uploaded).
    With CSR A, alpha = 1 and beta = 0 the result equals scipy's ``A @ x`` bit for bit.
    """
    from .sparse import coo_matrix, csc_matrix
    if not check_availability("spmv"):
        raise RuntimeError("spmv is not available.")
    if isinstance(a, csc_matrix):
        a = a.T
        transa = not transa
    if not isinstance(a, (csr_matrix, coo_matrix)):
        raise TypeError("unsupported type (actual: {})".format(type(a)))
    if isinstance(a, coo_matrix):
        a = a.tocsr()
    if transa:
        a = a.transpose_csr()
    dev = a.device
    if not isinstance(x, torch.Tensor):
        x = torch.from_numpy(np.ascontiguousarray(x))
    x = x.to(dev)
    if a.shape[1] != x.numel():
        raise ValueError("dimension mismatch")
    assert a.has_canonical_format
    m = a.shape[0]
    dt = np.promote_types(a.dtype, np.dtype(str(x.dtype).replace("torch.", "")))
    if dt not in (np.float32, np.float64, np.complex64, np.complex128):
        raise TypeError(f"spmv supports float32/float64/complex64/complex128, got {dt}")
    a = a.astype(dt)
    tdt = a.data.dtype
    x = x.to(tdt).contiguous()
    if y is None:
        y = torch.zeros(m, dtype=tdt, device=dev)
    else:
        if not isinstance(y, torch.Tensor) or y.numel() != m:
            raise ValueError("dimension mismatch")
        if y.dtype != tdt or not y.is_contiguous():
            raise TypeError("y must be a contiguous tensor of the result type")
    if a.nnz == 0:       # the reference fills 0 (cusparse.py:1414-1416)
        y.fill_(0)
        return y
    h = _handle_for(a)
    va = _csr_view(a)
    ct, nparts = _ALPHA_CT[tdt]
    def host(v):
        return (ct * 2)(complex(v).real, complex(v).imag) if nparts == 2 else ct(float(v))
    al, be = host(alpha), host(beta)
    check(h.lib.spg_spmv(h.ptr, ctypes.byref(va), ctypes.c_void_p(x.data_ptr()), ctypes.byref(al),
                         ctypes.byref(be), ctypes.c_void_p(y.data_ptr())), "spg_spmv")
    return y


def num_products(a: csr_matrix, b: csr_matrix) -> int:
    """P = number of scalar products of A.B (cusparseSpGEMM_getNumProducts); GFLOPS = 2P/t."""
    h = _handle_for(a)
    va, vb = _csr_view(a), _csr_view(b)
    ws_bytes = ctypes.c_size_t(0)
    check(h.lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), _lib.SPG_ALG2, 0.2,
                         ctypes.byref(ws_bytes), None, None), "spg_plan")
    ws = torch.empty(max(ws_bytes.value, 1), dtype=torch.uint8, device=a.device)
    plan = ctypes.c_void_p()
    check(h.lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), _lib.SPG_ALG2, 0.2,
                         ctypes.byref(ws_bytes), ctypes.c_void_p(ws.data_ptr()),
                         ctypes.byref(plan)), "spg_plan")
    try:
        p = ctypes.c_int64(0)
        check(h.lib.spg_num_products(h.ptr, plan, ctypes.byref(p)), "spg_num_products")
        return int(p.value)
    finally:
        h.lib.spg_plan_destroy(plan)


def plan_info(a: csr_matrix, b: csr_matrix, alg: int = 0, chunk_fraction: float = 0.2) -> dict:
    """What spgemm(a, b, alg, chunk_fraction) runs (spg_plan_info): the kernel path, the
    tile geometry and the row chunks (ALG3's chunk cut).  A diagnostic for tests/profilers."""
    h = _handle_for(a)
    va, vb = _csr_view(a), _csr_view(b)
    algo = _ALG.get(alg, _lib.SPG_ALG_DEFAULT)
    ws_bytes = ctypes.c_size_t(0)
    check(h.lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), algo, float(chunk_fraction),
                         ctypes.byref(ws_bytes), None, None), "spg_plan")
    ws = torch.empty(max(ws_bytes.value, 1), dtype=torch.uint8, device=a.device)
    plan = ctypes.c_void_p()
    check(h.lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), algo, float(chunk_fraction),
                         ctypes.byref(ws_bytes), ctypes.c_void_p(ws.data_ptr()), ctypes.byref(plan)), "spg_plan")
    try:
        info = _lib.SpgPlanInfo()
        check(h.lib.spg_plan_info(plan, ctypes.byref(info), None, 0), "spg_plan_info")
        rows = (ctypes.c_int64 * (info.n_chunks + 1))()
        check(h.lib.spg_plan_info(plan, ctypes.byref(info), rows, info.n_chunks + 1), "spg_plan_info")
        return {"path": ("general", "short", "tile")[info.path], "tile_width": info.tile_width,
                "tiles_per_row": info.tiles_per_row, "dense_tiles": bool(info.dense_tiles),
                "lds_ordered": bool(info.lds_ordered), "record_group": int(info.record_group),
                "chunk_rows": [int(x) for x in rows]}
    finally:
        h.lib.spg_plan_destroy(plan)
        torch.cuda.current_stream(a.device).synchronize()


__all__ = ["spgemm", "spmv", "check_availability", "num_products", "validate_csr", "SpgError",
           "last_stats"]
