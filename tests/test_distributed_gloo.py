"""The multi-GPU row-block path on CPU with the gloo backend (world_size 2), driven through
the same functions bench.py's config-5 workload runs (spmm_amd.distributed.rowblock_setup
and rowblock_step): B broadcast from rank 0 (metadata, packed structure, values left in
flight), the product-prefix row cut, each rank's slab, the nnz allgather and the stitched
row pointer.  The per-rank multiply is the CPU oracle (the device multiply is covered by the
gpu tests); the stitched C must equal the oracle's C for the whole matrix, bit for bit."""
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


def _worker(rank, world, port, dtype, out):
    import scipy.sparse as sp
    import torch.distributed as dist
    from oracle import oracle
    from spmm_amd import distributed
    from spmm_amd.sparse import csr_matrix
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cpu = torch.device("cpu")
    n = 300
    rng = np.random.default_rng(7)
    Ah = sp.random(n, n, density=0.03, format="csr", random_state=rng).astype(dtype)
    Bh = sp.random(n, n, density=0.03, format="csr", random_state=rng).astype(dtype)
    if np.issubdtype(dtype, np.complexfloating):
        Ah.data = Ah.data + 1j * rng.standard_normal(Ah.nnz)
        Bh.data = Bh.data + 1j * rng.standard_normal(Bh.nnz)
    Ah.sort_indices(); Bh.sort_indices()
    A = csr_matrix(Ah, device=cpu)
    B_src = csr_matrix(Bh, device=cpu) if rank == 0 else None
    # setup as bench.py: one broadcast for B's row lengths, the product-prefix cut
    Bw = distributed.broadcast_csr(B_src, 0, cpu)
    assert np.array_equal(Bw.indptr.numpy(), Bh.indptr) and np.array_equal(Bw.indices.numpy(), Bh.indices)
    assert np.array_equal(Bw.data.numpy(), Bh.data)
    (r0, r1), A_blk, P_r = distributed.rowblock_setup(A, Bw.indptr, world, rank)
    assert P_r == oracle.num_products(Ah[r0:r1], Bh)

    def multiply(A_b, B, wait_values):
        wait_values()   # the values broadcast was left in flight
        return oracle.spgemm(A_b.get(), B.get(), keep_zeros=True, sort=True)

    (p, j, x), B = distributed.rowblock_step(A_blk, B_src, 0, cpu, multiply=multiply)
    assert B.nnz == Bh.nnz
    nnzs = distributed.allgather_nnz(len(j), cpu)
    P_all = distributed.allgather_nnz(P_r, cpu)
    gathered = [None] * world
    dist.all_gather_object(gathered, (p.tolist(), j.tolist(), x.tolist(), (r0, r1)))
    if rank == 0:
        ip = distributed.stitch_indptr([g[0] for g in gathered], nnzs)
        jj = np.concatenate([np.asarray(g[1], np.int32) for g in gathered])
        xx = np.concatenate([np.asarray(g[2], dtype=dtype) for g in gathered])
        rp, rj, rx = oracle.spgemm(Ah, Bh, keep_zeros=True, sort=True)
        blocks = [g[3] for g in gathered]
        out["ok"] = bool(np.array_equal(ip, rp) and np.array_equal(jj, rj) and
                         np.array_equal(xx.view(np.uint8), rx.view(np.uint8)))
        out["blocks"] = blocks
        out["products"] = P_all
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_rowblock_step_gloo(dtype):
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), dtype, out), nprocs=world, join=True)
    assert out.get("ok") is True
    (a0, a1), (b0, b1) = out["blocks"]
    assert a0 == 0 and a1 == b0 and b1 == 300   # contiguous cover of the rows
    p0, p1 = out["products"]
    assert abs(p0 - p1) <= 0.2 * (p0 + p1)     # cut on the product prefix: balanced


def test_row_blocks_balanced():
    from spmm_amd import distributed
    assert distributed.row_blocks(10, 3) == [(0, 3), (3, 6), (6, 10)]
    pref = np.array([0, 100, 101, 102, 103, 200])   # heavy first and last rows
    blocks = distributed.row_blocks(5, 2, pref)
    assert blocks[0][0] == 0 and blocks[-1][1] == 5
    assert all(b[0] <= b[1] for b in blocks)


def test_product_prefix_matches_oracle():
    import scipy.sparse as sp
    from oracle import oracle
    from spmm_amd import distributed
    from spmm_amd.sparse import csr_matrix
    rng = np.random.default_rng(3)
    Ah = sp.random(200, 150, density=0.05, format="csr", random_state=rng)
    Bh = sp.random(150, 120, density=0.05, format="csr", random_state=rng)
    A = csr_matrix(Ah, device="cpu")
    pref = distributed.product_prefix(A, torch.from_numpy(Bh.indptr.astype(np.int64))).numpy()
    assert pref[0] == 0 and pref[-1] == oracle.num_products(Ah, Bh)
    for i in (0, 17, 199):
        assert pref[i + 1] - pref[i] == oracle.num_products(Ah[i:i + 1], Bh)


def _tile_major(Bh, tw, G):
    rows = np.repeat(np.arange(Bh.shape[0]), np.diff(Bh.indptr))
    t = Bh.indices // tw
    order = np.lexsort((np.arange(Bh.nnz), rows, t))
    offs = np.zeros(G + 1, dtype=np.int64)
    np.cumsum(np.bincount(t, minlength=G), out=offs[1:])
    return Bh.data[order], offs


def _tiles_worker(rank, world, port, out):
    """TileValueBroadcast on gloo: the protocol of the pipelined values broadcast (the device
    permutation and spg_numeric_tiles are the gpu tests'; here `tile_values` is numpy's)."""
    import scipy.sparse as sp
    import torch.distributed as dist
    from spmm_amd import distributed
    from spmm_amd.sparse import csr_matrix
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cpu = torch.device("cpu")
    rng = np.random.default_rng(11)
    Bh = sp.random(500, 1000, density=0.02, format="csr", random_state=rng)
    Bh.sort_indices()
    tw = 64
    G = (1000 + tw - 1) // tw
    tv, offs = _tile_major(Bh, tw, G)
    B = distributed.broadcast_csr(csr_matrix(Bh, device=cpu) if rank == 0 else None, 0, cpu, values=False)
    assert np.array_equal(B.indices.numpy(), Bh.indices)
    geom = {"tile_width": tw, "tiles": G, "offsets": offs, "dtype": torch.float64,
            "tile_values": lambda: torch.from_numpy(tv.copy())}
    bc = distributed.TileValueBroadcast(B, 0, cpu, n_groups=4)
    tm, groups = bc(geom)
    covered = []
    for g0, g1 in groups:   # a group is released only once its slice has landed
        a, b = int(offs[g0]), int(offs[g1])
        ok = np.array_equal(tm[a:b].numpy(), tv[a:b]) or rank == 0
        covered.append((g0, g1, ok))
    bc.finish()
    res = {"pipelined": bc.pipelined, "covered": covered, "full": bool(np.array_equal(tm.numpy(), tv))}
    # disagreement (rank 1 plans another tile width) -> row-major values in one broadcast
    B2 = distributed.broadcast_csr(csr_matrix(Bh, device=cpu) if rank == 0 else None, 0, cpu, values=False)
    geom2 = dict(geom, tile_width=tw * (1 + rank))
    bc2 = distributed.TileValueBroadcast(B2, 0, cpu)
    res["fallback"] = bc2(geom2) is None and not bc2.pipelined
    res["fallback_values"] = bool(np.array_equal(B2.data.numpy(), Bh.data))
    # a rank without a tile plan (geom None) also sends everyone to the fallback
    B3 = distributed.broadcast_csr(csr_matrix(Bh, device=cpu) if rank == 0 else None, 0, cpu, values=False)
    bc3 = distributed.TileValueBroadcast(B3, 0, cpu)
    res["fallback_none"] = bc3(geom if rank == 0 else None) is None
    res["fallback_none_values"] = bool(np.array_equal(B3.data.numpy(), Bh.data))
    # plans of different value types (the ranks would send different byte counts)
    B4 = distributed.broadcast_csr(csr_matrix(Bh, device=cpu) if rank == 0 else None, 0, cpu, values=False)
    bc4 = distributed.TileValueBroadcast(B4, 0, cpu)
    res["fallback_dtype"] = bc4(dict(geom, dtype=torch.float64 if rank == 0 else torch.float32)) is None
    res["fallback_dtype_values"] = bool(np.array_equal(B4.data.numpy(), Bh.data))
    out[rank] = res
    dist.barrier()
    dist.destroy_process_group()


def test_tile_value_broadcast_gloo():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_tiles_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        res = out[r]
        assert res["pipelined"] and res["full"], (r, res)
        assert [c[:2] for c in res["covered"]] == [c[:2] for c in out[0]["covered"]]
        assert len(res["covered"]) == 4 and all(c[2] for c in res["covered"]), (r, res)
        assert res["covered"][0][0] == 0 and res["covered"][-1][1] == 16
        assert res["fallback"] and res["fallback_values"], (r, res)
        assert res["fallback_none"] and res["fallback_none_values"], (r, res)
        assert res["fallback_dtype"] and res["fallback_dtype_values"], (r, res)


def test_tile_groups_cover_and_balance():
    from spmm_amd import distributed
    offs = np.array([0, 10, 20, 30, 1000, 1010, 1020, 1030, 1040])
    g = distributed.tile_groups(offs, 4)
    assert g[0][0] == 0 and g[-1][1] == 8 and len(g) == 4
    assert all(a < b for a, b in g) and all(g[i][1] == g[i + 1][0] for i in range(3))
    assert distributed.tile_groups(offs, 100) == [(i, i + 1) for i in range(8)]
    assert distributed.tile_groups(np.array([0, 5]), 8) == [(0, 1)]
    assert distributed.tile_groups(np.array([0, 0, 0, 0]), 2) == [(0, 1), (1, 3)]


def _wide_worker(rank, world, port, out):
    """broadcast_csr on both structure encodings: 16-bit columns (with each row's 65536-column
    block starts when B is wider) and 32-bit ones (a B so wide and sparse that the starts
    would cost more: 10**7 columns, 2 entries per row), each received exactly."""
    import scipy.sparse as sp
    import torch.distributed as dist
    from spmm_amd import distributed
    from spmm_amd.sparse import csr_matrix
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cpu = torch.device("cpu")
    ok = []
    for cols in (65536, 65537, 200000, 10 ** 7):
        rng = np.random.default_rng(cols)
        per_row = 2.0 if cols == 10 ** 7 else 40.0
        Bh = sp.random(40, cols, density=per_row / cols, format="csr", random_state=rng)
        Bh.indices[-1] = cols - 1 if Bh.nnz else 0   # the widest column travels too
        Bh.sort_indices()
        B = distributed.broadcast_csr(csr_matrix(Bh, device=cpu) if rank == 0 else None, 0, cpu)
        ok.append(bool(np.array_equal(B.indices.numpy(), Bh.indices) and np.array_equal(B.indptr.numpy(), Bh.indptr)
                       and np.array_equal(B.data.numpy(), Bh.data) and B.indices.dtype == torch.int32))
    out[rank] = ok
    dist.barrier()
    dist.destroy_process_group()


def test_broadcast_csr_column_encodings_gloo():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_wide_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert out[0] == [True] * 4 and out[1] == [True] * 4, dict(out)
    from spmm_amd import distributed
    assert distributed.cols16_layout(40, 65536, 1600) == 0
    assert distributed.cols16_layout(40, 200000, 1600) == 3
    assert distributed.cols16_layout(40, 10 ** 7, 80) == -1


def _edge_csr(cols):
    """Rows that exercise the block starts: empty rows, a row only in the last block, a row
    on the block edges (c * 65536 - 1, c * 65536), a row in the first block only."""
    import scipy.sparse as sp
    nb = -(-cols // 65536)
    edges = sorted({min(cols - 1, max(0, c * 65536 + d)) for c in range(nb) for d in (-1, 0)})
    rows = [[], [cols - 1], edges, [0, 5, 65535 if cols > 65535 else cols - 1], [],
            sorted(set(np.random.default_rng(cols).integers(0, cols, 300).tolist()))]
    ip = np.cumsum([0] + [len(r) for r in rows])
    return sp.csr_matrix((np.arange(ip[-1], dtype=np.float64) + 1.0, np.concatenate([np.array(r, dtype=np.int32) for r in rows]),
                          ip), shape=(len(rows), cols))


@pytest.mark.parametrize("cols", [7, 65536, 65537, 131072, 131073, 300000])
def test_cols16_host_roundtrip(cols):
    """The host split/join (the CPU tensors of the gloo tests; spg_cols16_split/join on the
    GPU): starts[r, c-1] = the first entry of row r with column >= c * 65536, and the join
    gives the columns back exactly."""
    from spmm_amd import distributed
    from spmm_amd.sparse import csr_matrix
    Bh = _edge_csr(cols)
    M = csr_matrix(Bh, device="cpu")
    nb1 = max(0, -(-cols // 65536) - 1)
    starts, lo16 = distributed._cols16_split_host(M, nb1)
    assert starts.shape == (Bh.shape[0], nb1) and lo16.numel() == Bh.nnz
    for r in range(Bh.shape[0]):
        row = Bh.indices[Bh.indptr[r]:Bh.indptr[r + 1]]
        want = [int(np.searchsorted(row, c * 65536, side="left")) for c in range(1, nb1 + 1)]
        assert starts[r].tolist() == want, (r, starts[r].tolist(), want)
    assert np.array_equal(lo16.numpy().view(np.uint16), (Bh.indices & 0xffff).astype(np.uint16))
    back = distributed._cols16_join_host(M.indptr, starts, lo16)
    assert back.dtype == torch.int32 and np.array_equal(back.numpy(), Bh.indices)


def _cpu_tiles_hook(rank, fail_rank=None, tw=64):
    """rowblock_step's `multiply_tiles` on the CPU: the by_tiles protocol of
    cusparse._spgemm_by_tiles (geometry from B's structure -> by_tiles(geom) -> groups as
    they land -> values back to row-major) around the oracle.  `fail_rank` raises where
    spg_tile_value_offsets would fail, before the agreement."""
    from oracle import oracle

    def hook(A_b, B, alg, cf, by_tiles, values_first):
        if by_tiles is None:   # row-major values complete (a rank whose A promotes B)
            return oracle.spgemm(A_b.get(), B.get(), keep_zeros=True, sort=True)
        if rank == fail_rank:
            raise RuntimeError("injected spg_tile_value_offsets failure")
        Bh = B.get()
        G = (Bh.shape[1] + tw - 1) // tw
        rows = np.repeat(np.arange(Bh.shape[0]), np.diff(Bh.indptr))
        t = Bh.indices // tw
        order = np.lexsort((np.arange(Bh.nnz), rows, t))
        offs = np.zeros(G + 1, dtype=np.int64)
        np.cumsum(np.bincount(t, minlength=G), out=offs[1:])
        geom = {"tile_width": tw, "tiles": G, "offsets": offs, "dtype": B.data.dtype,
                "tile_values": lambda: B.data[torch.from_numpy(order)].contiguous()}
        got = by_tiles(geom)
        if got is not None:
            tm, groups = got
            for _ in groups:
                pass
            vals = torch.empty_like(tm)
            vals[torch.from_numpy(order)] = tm
            Bh.data = vals.numpy()
        else:
            Bh = B.get()
        return oracle.spgemm(A_b.get(), Bh, keep_zeros=True, sort=True)
    return hook


def _hazard_worker(rank, world, port, mode, out):
    """Multi-rank hazards of the pipelined step: ranks whose A blocks have
    different value types, and a rank that fails before the agreement.  Every rank must
    finish the step (bit-exact) or raise; none may block in a collective its peers skip --
    the follow-up step proves the group's collectives are still aligned."""
    import scipy.sparse as sp
    import torch.distributed as dist
    from oracle import oracle
    from spmm_amd import distributed
    from spmm_amd.sparse import csr_matrix
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cpu = torch.device("cpu")
    rng = np.random.default_rng(5)
    Ah = sp.random(120, 700, density=0.03, format="csr", random_state=rng)
    Bh = sp.random(700, 900, density=0.03, format="csr", random_state=rng)
    Ah.sort_indices(); Bh.sort_indices()
    blk = Ah[rank * 60:(rank + 1) * 60]
    if mode == "dtype" and rank == 1:
        blk = blk.astype(np.complex128)
        blk.data = blk.data + 1j * rng.standard_normal(blk.nnz)
    A_b = csr_matrix(blk, device=cpu)
    B_src = csr_matrix(Bh, device=cpu) if rank == 0 else None
    res = {}
    try:
        (p, j, x), _ = distributed.rowblock_step(A_b, B_src, 0, cpu, pipeline=True,
                                                 multiply_tiles=_cpu_tiles_hook(rank, 1 if mode == "fail" else None))
        rp, rj, rx = oracle.spgemm(blk, Bh, keep_zeros=True, sort=True)
        res["exact"] = bool(np.array_equal(p, rp) and np.array_equal(j, rj) and x.dtype == rx.dtype
                            and np.array_equal(x.view(np.uint8), rx.view(np.uint8)))
        res["pipelined"] = distributed.rowblock_step.last.pipelined
    except Exception as e:   # noqa: BLE001 -- the test reports which error each rank raised
        res["raised"] = type(e).__name__
        res["msg"] = str(e)
    # a normal pipelined step afterwards: the ranks' collectives are still aligned
    A_ok = csr_matrix(Ah[rank * 60:(rank + 1) * 60], device=cpu)
    (p, j, x), _ = distributed.rowblock_step(A_ok, B_src, 0, cpu, pipeline=True, multiply_tiles=_cpu_tiles_hook(rank))
    rp, rj, rx = oracle.spgemm(Ah[rank * 60:(rank + 1) * 60], Bh, keep_zeros=True, sort=True)
    res["after"] = bool(np.array_equal(j, rj) and np.array_equal(x.view(np.uint8), rx.view(np.uint8))
                        and distributed.rowblock_step.last.pipelined)
    out[rank] = res
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("mode", ["dtype", "fail"])
def test_rowblock_step_hazards_gloo(mode):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_hazard_worker, args=(2, _free_port(), mode, out), nprocs=2, join=True)
    r0, r1 = out[0], out[1]
    if mode == "dtype":
        # rank 1's complex A block would promote B: everyone takes the row-major values
        assert r0.get("exact") and r1.get("exact"), (r0, r1)
        assert r0["pipelined"] is False and r1["pipelined"] is False
    else:
        assert r1.get("raised") == "RuntimeError" and "injected" in r1["msg"], r1
        assert r0.get("raised") == "StepFailed", r0
    assert r0["after"] and r1["after"], (r0, r1)


def _unsorted_worker(rank, world, port, out):
    """a B wider than 65536 columns whose rows are NOT sorted must arrive exactly
    as stored (int32 columns), not through the 16-bit encoding that needs sorted rows."""
    import scipy.sparse as sp
    import torch.distributed as dist
    from spmm_amd import distributed
    from spmm_amd.sparse import csr_matrix
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cpu = torch.device("cpu")
    rng = np.random.default_rng(9)
    Bh = sp.random(50, 200000, density=60 / 200000, format="csr", random_state=rng)
    Bh.sort_indices()
    for r in range(0, 50, 3):   # reverse some rows
        a, b = Bh.indptr[r], Bh.indptr[r + 1]
        Bh.indices[a:b] = Bh.indices[a:b][::-1].copy()
        Bh.data[a:b] = Bh.data[a:b][::-1].copy()
    Bh.has_sorted_indices = False
    src = csr_matrix((torch.from_numpy(Bh.data), torch.from_numpy(Bh.indices), torch.from_numpy(Bh.indptr)),
                     shape=Bh.shape, canonical=False) if rank == 0 else None
    B = distributed.broadcast_csr(src, 0, cpu)
    out[rank] = (bool(np.array_equal(B.indices.numpy(), Bh.indices) and np.array_equal(B.data.numpy(), Bh.data)),
                 B._canonical)
    dist.barrier()
    dist.destroy_process_group()


def test_broadcast_csr_unsorted_wide_gloo():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_unsorted_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert out[0] == (True, False) and out[1] == (True, False), dict(out)
    from spmm_amd import distributed
    from spmm_amd.sparse import csr_matrix
    import scipy.sparse as sp
    S = sp.random(30, 100000, density=1e-3, format="csr", random_state=np.random.default_rng(1))
    S.sort_indices()
    assert distributed._rows_sorted(csr_matrix(S, device="cpu"))
    M = csr_matrix((torch.from_numpy(S.data), torch.from_numpy(S.indices), torch.from_numpy(S.indptr)),
                   shape=S.shape, canonical=None)
    M._canonical = None
    assert distributed._rows_sorted(M)
    i = int(np.argmax(np.diff(S.indptr) > 1))
    a = S.indptr[i]
    S.indices[a], S.indices[a + 1] = S.indices[a + 1], S.indices[a]
    M2 = csr_matrix((torch.from_numpy(S.data), torch.from_numpy(S.indices), torch.from_numpy(S.indptr)),
                    shape=S.shape, canonical=None)
    assert not distributed._rows_sorted(M2)
