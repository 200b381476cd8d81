"""Device-resident sparse containers for the SpGEMM path (torch tensors in HBM).

Mirrors the part of ``cupyx.scipy.sparse`` that the reference's hot path goes through:

* ``csr_matrix`` with int32 ``indices``, int32 (or int64 when nnz >= 2**31) ``indptr`` and
  f32/f64 ``data`` (modify_src/cupy-src/cupyx/scipy/sparse/_compressed.py:229-230,286-287
  force int32; int64 is added so configs with nnz >= 2**31 are representable);
* ``A @ B`` dispatch: ``__matmul__`` -> ``__mul__`` -> ``sum_duplicates()`` on both operands
  -> ``spgemm`` (_base.py:130-134, _csr.py:151-166);
* ``has_canonical_format`` evaluated on the device (the reference's
  ``_has_canonical_format_kern``, _compressed.py:177-192, here ``spg_validate_csr``);
* ``csc_matrix`` / ``coo_matrix`` operands of ``@`` are converted to CSR first
  (_csr.py:167-184).

Format conversions and duplicate summing run as torch device ops; the multiply itself runs
only in libmi355_spgemm.so.
"""
from __future__ import annotations

import numpy as np
import torch

_TORCH_OF = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
             np.dtype(np.complex64): torch.complex64, np.dtype(np.complex128): torch.complex128,
             np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64}
_NP_OF = {v: k for k, v in _TORCH_OF.items()}

INT32_MAX = 2 ** 31 - 1


def _as_tensor(x, dtype: torch.dtype, device) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype).contiguous()
    return torch.from_numpy(np.ascontiguousarray(x)).to(device=device, dtype=dtype)


def _default_device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")


class _SparseBase:
    ndim = 2

    @property
    def shape(self):
        return self._shape

    @property
    def dtype(self):
        return _NP_OF[self.data.dtype]

    @property
    def nnz(self) -> int:
        return int(self.data.numel())

    @property
    def device(self):
        return self.data.device

    def toarray(self) -> np.ndarray:
        return self.get().toarray()

    def __matmul__(self, other):
        return self.tocsr().__matmul__(other)


class csr_matrix(_SparseBase):
    """Compressed sparse row matrix on the device.

    ``csr_matrix(S)``            from a scipy.sparse matrix (uploaded),
    ``csr_matrix((data, indices, indptr), shape=(m, n))`` from arrays / tensors,
    ``csr_matrix((m, n), dtype=...)`` empty matrix.
    """
    format = "csr"

    def __init__(self, arg1, shape=None, dtype=None, device=None, canonical=None):
        device = torch.device(device) if device is not None else None
        if isinstance(arg1, csr_matrix):
            device = device or arg1.device
            self.data = arg1.data.to(device)
            self.indices, self.indptr = arg1.indices.to(device), arg1.indptr.to(device)
            self._shape = arg1.shape
            self._canonical = arg1._canonical
        elif isinstance(arg1, tuple) and len(arg1) == 2 and all(isinstance(s, (int, np.integer)) for s in arg1):
            device = device or _default_device()
            m, n = int(arg1[0]), int(arg1[1])
            dt = _TORCH_OF[np.dtype(dtype or np.float64)]
            self.data = torch.empty(0, dtype=dt, device=device)
            self.indices = torch.empty(0, dtype=torch.int32, device=device)
            self.indptr = torch.zeros(m + 1, dtype=torch.int32, device=device)
            self._shape = (m, n)
            self._canonical = True
        elif isinstance(arg1, tuple) and len(arg1) == 3:
            if shape is None:
                raise ValueError("shape is required for (data, indices, indptr)")
            device = device or (arg1[0].device if isinstance(arg1[0], torch.Tensor) else _default_device())
            data, indices, indptr = arg1
            ddt = np.dtype(dtype) if dtype is not None else (
                _NP_OF[data.dtype] if isinstance(data, torch.Tensor) else np.asarray(data).dtype)
            self.data = _as_tensor(data, _TORCH_OF[np.dtype(ddt)], device)
            self.indices = _as_tensor(indices, torch.int32, device)
            # int32 row pointers whenever they fit (CuPy casts to int32), int64 beyond
            ipd = torch.int32 if self.data.numel() <= INT32_MAX else torch.int64
            self.indptr = _as_tensor(indptr, ipd, device)
            self._shape = (int(shape[0]), int(shape[1]))
            self._canonical = canonical
        elif hasattr(arg1, "tocsr"):   # scipy.sparse matrix / array
            device = device or _default_device()
            S = arg1.tocsr()
            if dtype is not None:
                S = S.astype(dtype)
            canon = bool(S.has_canonical_format)
            ipd = torch.int32 if S.nnz <= INT32_MAX else torch.int64
            self.data = _as_tensor(S.data, _TORCH_OF[np.dtype(S.dtype)], device)
            self.indices = _as_tensor(S.indices, torch.int32, device)
            self.indptr = _as_tensor(S.indptr, ipd, device)
            self._shape = tuple(int(s) for s in S.shape)
            self._canonical = canon
        else:
            raise TypeError(f"unsupported csr_matrix argument {type(arg1)}")
        if self.data.dtype not in (torch.float32, torch.float64, torch.complex64, torch.complex128):
            raise TypeError(f"unsupported dtype {self.data.dtype}")
        if self.indptr.numel() != self._shape[0] + 1:
            raise ValueError("indptr length must be rows + 1")

    @classmethod
    def _from_parts(cls, data, indices, indptr, shape, canonical=True):
        """Wrap device tensors as-is (no conversion, no copy) -- the shim's result path."""
        self = cls.__new__(cls)
        self.data, self.indices, self.indptr = data, indices, indptr
        self._shape = (int(shape[0]), int(shape[1]))
        self._canonical = canonical
        return self

    # ------------------------------------------------------------------ structure
    @property
    def has_canonical_format(self) -> bool:
        """indices sorted strictly increasing inside each row (no duplicates).  Evaluated
        on the device with spg_validate_csr and cached, as CuPy caches it."""
        if self._canonical is None:
            from . import cusparse
            self._canonical = cusparse.validate_csr(self) == 1
        return self._canonical

    @has_canonical_format.setter
    def has_canonical_format(self, v: bool):
        self._canonical = bool(v)

    @property
    def has_sorted_indices(self) -> bool:
        return self.has_canonical_format

    def _row_ids(self) -> torch.Tensor:
        counts = (self.indptr[1:] - self.indptr[:-1]).to(torch.int64)
        return torch.repeat_interleave(torch.arange(self._shape[0], device=self.device), counts)

    def sum_duplicates(self) -> None:
        """Sort indices and add up duplicates in place (cupyx _compressed.py:971-991).
        Duplicates are added in stored order, sequentially."""
        if self._canonical is True or (self._canonical is None and self.has_canonical_format):
            return
        m, n = self._shape
        rows = self._row_ids()
        key = rows * max(n, 1) + self.indices.to(torch.int64)
        key_s, order = torch.sort(key, stable=True)
        data_s = self.data[order]
        uniq, counts = torch.unique_consecutive(key_s, return_counts=True)
        if uniq.numel() == key_s.numel():
            new_data = data_s
        else:
            new_data = _segmented_sequential_sum(data_s, counts)
        urow = torch.div(uniq, max(n, 1), rounding_mode="floor")
        self.indices = (uniq - urow * max(n, 1)).to(torch.int32)
        self.data = new_data.contiguous()
        self.indptr = _indptr_from_rows(urow, m, self.indptr.dtype)
        self._canonical = True

    def sort_indices(self) -> None:
        self.sum_duplicates() if self._canonical is not True else None

    def eliminate_zeros(self) -> None:
        keep = self.data != 0
        if bool(keep.all()):
            return
        rows = self._row_ids()[keep]
        self.data = self.data[keep].contiguous()
        self.indices = self.indices[keep].contiguous()
        self.indptr = _indptr_from_rows(rows, self._shape[0], self.indptr.dtype)

    # ------------------------------------------------------------------ conversion
    def astype(self, dtype):
        dt = _TORCH_OF[np.dtype(dtype)]
        if dt == self.data.dtype:
            return self
        out = csr_matrix(self)
        out.data = self.data.to(dt)
        return out

    def copy(self):
        out = csr_matrix(self)
        out.data, out.indices, out.indptr = self.data.clone(), self.indices.clone(), self.indptr.clone()
        return out

    def tocsr(self, copy=False):
        return self.copy() if copy else self

    def get(self):
        """Copy to the host as a scipy.sparse.csr_matrix (cupy's .get())."""
        import scipy.sparse as sp
        return sp.csr_matrix((self.data.cpu().numpy(), self.indices.cpu().numpy(),
                              self.indptr.cpu().numpy()), shape=self._shape)

    # ------------------------------------------------------------------ products
    def __mul__(self, other):
        """CSR x sparse: CuPy's _csr.py:151-166 order -- canonicalise both, then spgemm.
        CSR x dense vector (_csr.py:190-216): canonicalise, then spmv."""
        from . import cusparse
        if isinstance(other, (csc_matrix, coo_matrix)):
            other = other.tocsr()
        if isinstance(other, csr_matrix):
            self.sum_duplicates()
            other.sum_duplicates()
            return cusparse.spgemm(self, other)
        if _is_vector(other):
            self.sum_duplicates()
            return cusparse.spmv(self, other)
        return NotImplemented

    def transpose_csr(self) -> "csr_matrix":
        """A^T as a canonical CSR matrix (through COO with rows and columns swapped)."""
        m, n = self._shape
        counts = (self.indptr[1:] - self.indptr[:-1]).to(torch.int64)
        rows = torch.repeat_interleave(torch.arange(m, device=self.device), counts)
        return coo_matrix((self.data, (self.indices.to(torch.int64), rows)), shape=(n, m),
                          device=self.device).tocsr()

    def __matmul__(self, other):
        return self.__mul__(other)

    def dot(self, other):
        return self.__mul__(other)

    def __repr__(self):
        return (f"<{self._shape[0]}x{self._shape[1]} csr_matrix of type {self.dtype} with "
                f"{self.nnz} stored elements on {self.device}>")


def _is_vector(x) -> bool:
    return (isinstance(x, torch.Tensor) or isinstance(x, np.ndarray)) and x.ndim == 1


class coo_matrix(_SparseBase):
    """Coordinate-format operand (only what CSR conversion needs)."""
    format = "coo"

    def __matmul__(self, other):
        """COO x dense vector -> spmv (through CSR)."""
        if _is_vector(other):
            from . import cusparse
            return cusparse.spmv(self, other)
        return super().__matmul__(other)

    def __init__(self, arg1, shape=None, device=None):
        if hasattr(arg1, "tocoo"):
            S = arg1.tocoo()
            device = device or _default_device()
            self.data = _as_tensor(S.data, _TORCH_OF[np.dtype(S.dtype)], device)
            self.row = _as_tensor(S.row, torch.int64, device)
            self.col = _as_tensor(S.col, torch.int64, device)
            self._shape = tuple(int(s) for s in S.shape)
        else:
            data, (row, col) = arg1
            device = device or (data.device if isinstance(data, torch.Tensor) else _default_device())
            self.data = data.to(device) if isinstance(data, torch.Tensor) else _as_tensor(
                data, _TORCH_OF[np.asarray(data).dtype], device)
            self.row = _as_tensor(row, torch.int64, device)
            self.col = _as_tensor(col, torch.int64, device)
            self._shape = (int(shape[0]), int(shape[1]))

    def tocsr(self) -> csr_matrix:
        m, n = self._shape
        key = self.row * max(n, 1) + self.col
        key_s, order = torch.sort(key, stable=True)
        data_s = self.data[order]
        uniq, counts = torch.unique_consecutive(key_s, return_counts=True)
        data_u = data_s if uniq.numel() == key_s.numel() else _segmented_sequential_sum(data_s, counts)
        urow = torch.div(uniq, max(n, 1), rounding_mode="floor")
        ipd = torch.int32 if uniq.numel() <= INT32_MAX else torch.int64
        return csr_matrix((data_u, (uniq - urow * max(n, 1)).to(torch.int32),
                           _indptr_from_rows(urow, m, ipd)), shape=(m, n), canonical=True)

    def get(self):
        import scipy.sparse as sp
        return sp.coo_matrix((self.data.cpu().numpy(), (self.row.cpu().numpy(), self.col.cpu().numpy())),
                             shape=self._shape)


class csc_matrix(_SparseBase):
    """Compressed-column operand (only what CSR conversion needs)."""
    format = "csc"

    def __matmul__(self, other):
        """CSC x dense vector -> spmv (cusparse.py:1395-1401: csc.T is CSR, transposed op)."""
        if _is_vector(other):
            from . import cusparse
            return cusparse.spmv(self, other)
        return super().__matmul__(other)

    def __init__(self, arg1, device=None):
        S = arg1.tocsc()
        device = device or _default_device()
        self.data = _as_tensor(S.data, _TORCH_OF[np.dtype(S.dtype)], device)
        self.indices = _as_tensor(S.indices, torch.int32, device)
        self.indptr = _as_tensor(S.indptr, torch.int64, device)
        self._shape = tuple(int(s) for s in S.shape)

    @property
    def T(self) -> csr_matrix:
        """Transpose as CSR without data movement (CuPy returns csr for csc.T)."""
        m, n = self._shape
        ipd = torch.int32 if self.nnz <= INT32_MAX else torch.int64
        return csr_matrix((self.data, self.indices, self.indptr.to(ipd)), shape=(n, m))

    def tocsr(self) -> csr_matrix:
        m, n = self._shape
        counts = (self.indptr[1:] - self.indptr[:-1]).to(torch.int64)
        cols = torch.repeat_interleave(torch.arange(n, device=self.device), counts)
        return coo_matrix((self.data, (self.indices.to(torch.int64), cols)), shape=(m, n),
                          device=self.device).tocsr()

    def get(self):
        import scipy.sparse as sp
        return sp.csc_matrix((self.data.cpu().numpy(), self.indices.cpu().numpy(),
                              self.indptr.cpu().numpy()), shape=self._shape)


def isspmatrix_csr(x) -> bool:
    return isinstance(x, csr_matrix)


def _indptr_from_rows(rows: torch.Tensor, m: int, dtype) -> torch.Tensor:
    counts = torch.bincount(rows, minlength=m) if rows.numel() else torch.zeros(
        m, dtype=torch.int64, device=rows.device)
    indptr = torch.zeros(m + 1, dtype=torch.int64, device=rows.device)
    indptr[1:] = torch.cumsum(counts, 0)
    return indptr.to(dtype)


def _segmented_sequential_sum(vals: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """Sum consecutive runs of `vals` (run lengths `counts`), each run left to right.
    Deterministic: runs are summed element by element in stored order."""
    nseg = counts.numel()
    starts = torch.zeros(nseg, dtype=torch.int64, device=vals.device)
    starts[1:] = torch.cumsum(counts, 0)[:-1]
    out = vals[starts].clone()
    maxc = int(counts.max()) if nseg else 0
    for r in range(1, maxc):
        sel = counts > r
        idx = starts[sel] + r
        out[sel] = out[sel] + vals[idx]
    return out
