"""Synthetic CSR inputs for the SpGEMM benchmarks and tests.

* ``scipy_random``: ``scipy.sparse.random(n, n, density, random_state=default_rng(seed))``,
  A then B from the same rng stream (fixes the reference's A == B bug,
  SpGEMM_alg_comparison/profiler.py:176-177).  Used up to config 3 sizes; at config 2
  (N=16384, density 1e-3, seed 42) it gives nnz(C) = 4,366,124 as in SURVEY 8d.
* ``random_csr``: O(nnz) generator for configs 4/5 where scipy's
  ``rng.choice(N*N, ...)`` is too slow: per-row Binomial(n, density) counts (the per-row
  binomial idea of others/profiler.py:34-67), columns uniform without replacement inside
  a row (duplicates redrawn), values standard normal (the profilers' data_rvs,
  SpGEMM_alg_comparison/profiler.py:149-151).  Runs with torch on the target device.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch

from .sparse import csr_matrix


def scipy_random(m: int, n: int, density: float, rng, dtype=np.float64, normal: bool = False):
    M = sp.random(m, n, density=density, format="csr", dtype=dtype, random_state=rng,
                  data_rvs=(rng.standard_normal if normal else None))
    M.sort_indices()
    return M


def scipy_pair(n: int, density: float, seed: int = 42, dtype=np.float64, normal: bool = False):
    """(A, B) host matrices, A first then B from one default_rng(seed) stream."""
    rng = np.random.default_rng(seed)
    A = scipy_random(n, n, density, rng, dtype, normal)
    B = scipy_random(n, n, density, rng, dtype, normal)
    return A, B


@torch.no_grad()
def random_csr(m: int, n: int, density: float, seed: int = 0, dtype=torch.float64,
               device="cuda", row_offset: int = 0) -> csr_matrix:
    """Uniform random m x n CSR with ~density*n entries per row, canonical, on `device`.

    `row_offset` makes row r of the result identical to row (row_offset + r) of the full
    matrix generated with the same seed -- the row-block shards of the multi-GPU path draw
    their own block without materialising the whole A.
    """
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    # one independent stream per 65536-row block keeps row blocks reproducible
    blk = 65536
    parts_cnt, parts_cols, parts_val = [], [], []
    r = row_offset
    end = row_offset + m
    while r < end:
        b0 = (r // blk) * blk
        g.manual_seed(seed * 1000003 + b0 // blk)
        nb = blk
        counts_b = torch.binomial(torch.full((nb,), float(n), dtype=torch.float64, device=dev),
                                  torch.full((nb,), float(density), dtype=torch.float64, device=dev),
                                  generator=g).to(torch.int64)
        lo, hi = r - b0, min(end, b0 + blk) - b0
        cols_b = _distinct_cols(counts_b, n, g, dev)
        ptr = torch.zeros(nb + 1, dtype=torch.int64, device=dev)
        ptr[1:] = torch.cumsum(counts_b, 0)
        vals_b = torch.randn(cols_b.numel(), dtype=dtype, device=dev, generator=g)
        parts_cnt.append(counts_b[lo:hi])
        parts_cols.append(cols_b[ptr[lo]:ptr[hi]])
        parts_val.append(vals_b[ptr[lo]:ptr[hi]])
        r = b0 + hi
    counts = torch.cat(parts_cnt)
    cols = torch.cat(parts_cols).to(torch.int32)
    indptr = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    indptr[1:] = torch.cumsum(counts, 0)
    nnz = int(indptr[-1])
    data = torch.cat(parts_val)
    ipd = torch.int32 if nnz < 2 ** 31 else torch.int64
    return csr_matrix((data, cols, indptr.to(ipd)), shape=(m, n), canonical=True)


def _distinct_cols(counts: torch.Tensor, n: int, g: torch.Generator, dev) -> torch.Tensor:
    """Sorted distinct columns per row, row-major, len = counts.sum()."""
    rows = torch.repeat_interleave(torch.arange(counts.numel(), device=dev), counts)
    cols = torch.randint(0, n, (rows.numel(),), device=dev, generator=g, dtype=torch.int64)
    for _ in range(64):
        key, _ = torch.sort(rows * n + cols)
        dup = torch.zeros_like(key, dtype=torch.bool)
        dup[1:] = key[1:] == key[:-1]
        rows = torch.div(key, n, rounding_mode="floor")
        cols = key - rows * n
        if not bool(dup.any()):
            return cols
        # redraw the duplicates (rejection until every row has distinct columns)
        cols = torch.where(dup, torch.randint(0, n, cols.shape, device=dev, generator=g,
                                              dtype=torch.int64), cols)
    raise RuntimeError("could not draw distinct columns (density too close to 1?)")
