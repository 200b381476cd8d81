"""Multi-GPU C = A.B: 1-D row-block sharding of A, B broadcast over RCCL/xGMI.

Rows of C depend only on the same rows of A and on all of B, so each rank
owns a contiguous row block of A, receives B once, and writes its own C slab -- there is no
cross-GPU reduction.  The only collectives are

* ``broadcast_csr``: B from ``src`` to every rank, as a 5-int64 metadata broadcast
  followed by three payload broadcasts (indptr, indices, data) -- the protocol of the
  reference's vendored sparse broadcast, modify_src/cupy-src/cupyx/distributed/
  _nccl_comm.py:651-674 (metadata exchange :506-530), on torch.distributed (backend
  "nccl" = RCCL on ROCm, "gloo" in CPU tests);
* ``allgather_nnz``: every rank's nnz(C slab) -> global row-pointer offsets, when a
  stitched C is wanted.

``row_blocks`` balances rows by the product-count prefix (equal FLOPs per rank); for
uniform random inputs that is close to equal rows.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .sparse import csr_matrix

_DT_CODE = {torch.float32: 0, torch.float64: 1}
_CODE_DT = {v: k for k, v in _DT_CODE.items()}
_IP_CODE = {torch.int32: 0, torch.int64: 1}
_CODE_IP = {v: k for k, v in _IP_CODE.items()}


def broadcast_csr(M: csr_matrix | None, src: int, device, group=None) -> csr_matrix:
    """Broadcast a CSR matrix held by rank `src` to every rank of `group`."""
    rank = dist.get_rank(group)
    meta = torch.zeros(5, dtype=torch.int64, device=device)
    if rank == src:
        meta = torch.tensor([M.shape[0], M.shape[1], M.nnz, _DT_CODE[M.data.dtype],
                             _IP_CODE[M.indptr.dtype]], dtype=torch.int64, device=device)
    dist.broadcast(meta, src, group=group)
    rows, cols, nnz, dtc, ipc = (int(x) for x in meta.tolist())
    if rank == src:
        indptr, indices, data = (M.indptr.to(device), M.indices.to(device), M.data.to(device))
    else:
        indptr = torch.empty(rows + 1, dtype=_CODE_IP[ipc], device=device)
        indices = torch.empty(nnz, dtype=torch.int32, device=device)
        data = torch.empty(nnz, dtype=_CODE_DT[dtc], device=device)
    for t in (indptr, indices, data):
        if t.numel():
            dist.broadcast(t, src, group=group)
    out = csr_matrix((data, indices, indptr), shape=(rows, cols), canonical=True)
    out.indptr = indptr
    return out


def row_blocks(n_rows: int, world: int, product_prefix: np.ndarray | None = None):
    """[(r0, r1)] per rank.  With a product-count prefix (length n_rows + 1) the cuts fall
    where the cumulative products cross k/world of the total; otherwise equal rows."""
    if product_prefix is None:
        cuts = [(n_rows * r) // world for r in range(world + 1)]
    else:
        pp = np.asarray(product_prefix, dtype=np.int64)
        total = int(pp[-1])
        cuts = [0]
        for r in range(1, world):
            cuts.append(int(np.searchsorted(pp, (total * r) // world, side="left")))
        cuts.append(n_rows)
        for i in range(1, len(cuts)):
            cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def allgather_nnz(nnz: int, device, group=None) -> list[int]:
    """nnz of every rank's C slab (in rank order)."""
    world = dist.get_world_size(group)
    mine = torch.tensor([nnz], dtype=torch.int64, device=device)
    out = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(out, mine, group=group)
    return [int(t.item()) for t in out]


def spgemm_rowblock(A_block: csr_matrix, B: csr_matrix, alg: int = 0, chunk_fraction: float = 0.2):
    """This rank's C slab = A_block . B (row block r0:r1 of the global C)."""
    from . import cusparse
    return cusparse.spgemm(A_block, B, alg=alg, chunk_fraction=chunk_fraction)


def stitch_indptr(slab_indptrs, slab_nnz):
    """Global row pointer from per-rank slab row pointers (host numpy, int64): slab r's
    pointers shifted by the nnz of slabs 0..r-1 (the offsets allgather_nnz provides)."""
    out = [np.zeros(1, np.int64)]
    base = 0
    for p, nz in zip(slab_indptrs, slab_nnz):
        p = np.asarray(p, dtype=np.int64)
        out.append(p[1:] + base)
        base += int(nz)
    return np.concatenate(out)
