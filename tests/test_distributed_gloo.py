"""The multi-GPU plumbing on CPU with the gloo backend (world_size 2): B broadcast
(metadata + 3 payloads), row-block partition, nnz allgather and slab stitching.  The
per-rank multiply is stood in for by the CPU oracle here (the device multiply is covered
by the gpu tests); what is tested is the distributed bookkeeping."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import scipy.sparse as sp
    import torch.distributed as dist
    from oracle import oracle
    from spmm_amd import distributed
    from spmm_amd.sparse import csr_matrix
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 300
    rng = np.random.default_rng(7)
    A = sp.random(n, n, density=0.03, format="csr", random_state=rng)
    Bh = sp.random(n, n, density=0.03, format="csr", random_state=rng)
    A.sort_indices(); Bh.sort_indices()
    B0 = csr_matrix(Bh, device="cpu") if rank == 0 else None
    B = distributed.broadcast_csr(B0, 0, torch.device("cpu"))
    assert B.shape == Bh.shape and B.nnz == Bh.nnz
    assert np.array_equal(B.indptr.numpy(), Bh.indptr)
    assert np.array_equal(B.indices.numpy(), Bh.indices)
    assert np.array_equal(B.data.numpy(), Bh.data)
    pref = np.zeros(n + 1, np.int64)
    pref[1:] = np.cumsum([sum(Bh.indptr[k + 1] - Bh.indptr[k] for k in A.indices[A.indptr[i]:A.indptr[i + 1]])
                          for i in range(n)])
    r0, r1 = distributed.row_blocks(n, world, pref)[rank]
    p, j, x = oracle.spgemm(A[r0:r1], B.get(), keep_zeros=True, sort=True)
    nnzs = distributed.allgather_nnz(len(j), torch.device("cpu"))
    gathered = [None] * world
    dist.all_gather_object(gathered, (p.tolist(), j.tolist(), x.tolist()))
    if rank == 0:
        ip = distributed.stitch_indptr([g[0] for g in gathered], nnzs)
        jj = np.concatenate([np.asarray(g[1], np.int32) for g in gathered])
        xx = np.concatenate([np.asarray(g[2]) for g in gathered])
        rp, rj, rx = oracle.spgemm(A, Bh, keep_zeros=True, sort=True)
        out["ok"] = bool(np.array_equal(ip, rp) and np.array_equal(jj, rj) and np.array_equal(xx, rx))
    dist.barrier()
    dist.destroy_process_group()


def test_rowblock_broadcast_gloo():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert out.get("ok") is True


def test_row_blocks_balanced():
    from spmm_amd import distributed
    assert distributed.row_blocks(10, 3) == [(0, 3), (3, 6), (6, 10)]
    pref = np.array([0, 100, 101, 102, 103, 200])   # heavy first and last rows
    blocks = distributed.row_blocks(5, 2, pref)
    assert blocks[0][0] == 0 and blocks[-1][1] == 5
    assert all(b[0] <= b[1] for b in blocks)
