"""The numeric phase by column-tile groups (spg_tile_value_offsets / spg_tile_values /
spg_numeric_tiles, include/spgemm.h) -- the device half of the pipelined multi-GPU values
broadcast (spmm_amd.distributed.TileValueBroadcast).

* the tile-major order: offsets and permuted values equal a numpy restatement
  (entries of column tile 0 row by row, then tile 1, ...) bit for bit;
* groups: spg_numeric_tiles over consecutive tile ranges, fed values that did NOT come
  from the plan's B (whose values are NaN here: the call must never read them), gives C
  bit for bit as spgemm and as the oracle;
* the fallback: plans off the tile path report no tile geometry and take spg_numeric;
* a 2-rank rehearsal of rowblock_step(pipeline=True) on one GPU (gloo backend: RCCL
  refuses two ranks on one device), stitched C bit-exact against the oracle.
"""
import functools
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bits(x):
    return x.view({4: np.uint32, 8: np.uint64, 16: np.uint64}[x.dtype.itemsize])


def tile_major(B, tw, G):
    """B's values in tile-major order and the G + 1 tile offsets (numpy restatement)."""
    rows = np.repeat(np.arange(B.shape[0]), np.diff(B.indptr))
    t = B.indices // tw
    order = np.lexsort((np.arange(B.nnz), rows, t))
    offs = np.zeros(G + 1, dtype=np.int64)
    np.cumsum(np.bincount(t, minlength=G), out=offs[1:])
    return B.data[order], offs


def _canon(M):
    M.sum_duplicates()
    M.sort_indices()
    return M


@functools.lru_cache(maxsize=1)
def _cases():
    """(name, A, B, alpha): the lean dense (2048-column) and sparse (8192-column) fp64 shapes,
    config 3's, one over three 65536-column symbolic blocks, and f32 / complex128 tile
    plans (generated once per process)."""
    out = []
    rng = np.random.default_rng(33)
    A = sp.random(257, 17000, density=0.01, format="csr", random_state=rng, dtype=np.float64)
    B = sp.random(17000, 17000, density=0.01, format="csr", random_state=rng, dtype=np.float64)
    out.append(("dense2048_f64", A, B, 1.0))
    rng = np.random.default_rng(34)
    A = sp.random(300, 40000, density=0.0075, format="csr", random_state=rng)
    B = sp.random(40000, 40000, density=0.00075, format="csr", random_state=rng)
    out.append(("sparse8192_f64", A, B, 0.5))
    from spmm_amd import gen
    A, B = gen.scipy_pair(8192, 1e-2, seed=42)
    out.append(("config3_f64", A, B, 1.0))
    rng = np.random.default_rng(37)   # > 2 symbolic blocks of 65536 columns (wide symbolic tasks)
    A = sp.random(200, 140000, density=7e-4, format="csr", random_state=rng)
    B = sp.random(140000, 140000, density=7e-4, format="csr", random_state=rng)
    out.append(("wide140k_f64", A, B, 1.0))
    rng = np.random.default_rng(35)
    A = sp.random(400, 20000, density=0.01, format="csr", random_state=rng, dtype=np.float32)
    B = sp.random(20000, 20000, density=0.005, format="csr", random_state=rng, dtype=np.float32)
    out.append(("f32", A, B, 2.0))
    rng = np.random.default_rng(36)
    A = sp.random(300, 12000, density=0.01, format="csr", random_state=rng).astype(np.complex128)
    B = sp.random(12000, 12000, density=0.005, format="csr", random_state=rng).astype(np.complex128)
    A.data = A.data + 1j * rng.standard_normal(A.nnz)
    B.data = B.data + 1j * rng.standard_normal(B.nnz)
    out.append(("c128", A, B, 1.0))
    return [(n, _canon(a), _canon(b), al) for n, a, b, al in out]


@pytest.mark.parametrize("case", [c[0] for c in _cases()])
def test_numeric_by_tile_groups_bitexact(case):
    from spmm_amd import cusparse, distributed
    from spmm_amd.sparse import csr_matrix
    name, A, B, alpha = next(c for c in _cases() if c[0] == case)
    dA, dB = csr_matrix(A, device="cuda:0"), csr_matrix(B, device="cuda:0")
    seen = {}

    def probe(geom):   # the tile-major values as the plan lays them out
        assert geom is not None, f"{name}: expected a tile plan with one chunk"
        tv, offs = tile_major(B, geom["tile_width"], geom["tiles"])
        assert np.array_equal(geom["offsets"], offs), f"{name}: tile offsets"
        tm = geom["tile_values"]()
        assert np.array_equal(_bits(tm.cpu().numpy()), _bits(tv)), f"{name}: tile-major values"
        seen["geom"] = (geom["tile_width"], geom["tiles"])
        return tm, distributed.tile_groups(offs, 1)

    C0 = cusparse._spgemm(dA, dB, alpha=alpha, alg=2, by_tiles=probe)
    ref = cusparse.spgemm(dA, dB, alpha=alpha, alg=2)
    rp, rj, rx = oracle.spgemm(A, B, alpha=alpha, keep_zeros=True, sort=True, threads=16)
    # values from outside the plan: B's own values NaN, the tile-major values from numpy
    Bnan = B.copy()
    Bnan.data[:] = np.nan
    dBn = csr_matrix(Bnan, device="cuda:0")
    G = seen["geom"][1]
    for n_groups in (2, 5, G):
        def feed(geom):
            assert (geom["tile_width"], geom["tiles"]) == seen["geom"]
            tv, offs = tile_major(B, geom["tile_width"], geom["tiles"])
            return torch.from_numpy(tv).to("cuda:0"), distributed.tile_groups(offs, n_groups)
        C = cusparse._spgemm(dA, dBn, alpha=alpha, alg=2, by_tiles=feed)
        torch.cuda.synchronize()
        for got in (C, C0):
            assert np.array_equal(got.indptr.cpu().numpy().astype(np.int64), rp), (name, n_groups)
            assert np.array_equal(got.indices.cpu().numpy(), rj), (name, n_groups)
            assert np.array_equal(_bits(got.data.cpu().numpy()), _bits(rx)), (name, n_groups)
        assert np.array_equal(_bits(C.data.cpu().numpy()), _bits(ref.data.cpu().numpy()))


def test_numeric_tiles_fallback_off_tile_path():
    """A product off the tile path (config 2's shape) reports no tile geometry; by_tiles
    answers None and spg_numeric runs."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    rng = np.random.default_rng(5)
    A = _canon(sp.random(2000, 2000, density=0.002, format="csr", random_state=rng))
    B = _canon(sp.random(2000, 2000, density=0.002, format="csr", random_state=rng))
    calls = []

    def by_tiles(geom):
        calls.append(geom)
        return None

    C = cusparse._spgemm(csr_matrix(A, device="cuda:0"), csr_matrix(B, device="cuda:0"), alg=2, by_tiles=by_tiles)
    assert calls == [None]
    rp, rj, rx = oracle.spgemm(A, B, keep_zeros=True, sort=True)
    assert np.array_equal(C.indices.cpu().numpy(), rj)
    assert np.array_equal(_bits(C.data.cpu().numpy()), _bits(rx))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


_REHEARSAL = r"""
import os, sys, json
import numpy as np, torch, torch.distributed as dist
sys.path.insert(0, ROOT)
from tests.test_gpu_tiles import _cases
from spmm_amd import distributed
from spmm_amd.sparse import csr_matrix
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
dev = torch.device("cuda:0")
out = {}
runs = [("sparse8192_f64", 2), ("dense2048_f64", 2), ("c128", 2),
        ("dense2048_f64", 1),      # ALG1: no tile geometry -> the row-major values broadcast
        ("sparse8192_f64", 3),     # ALG3 with its chunks forced: several chunks -> the same
        ("wide140k_f64", 2)]       # B wider than 65536: 16-bit columns + block starts (spg_cols16_join)
cases = {c[0]: c for c in _cases()}
for name, alg in runs:
    _, A, B, alpha = cases[name]
    os.environ["SPG_ALG3_CHUNK_ALWAYS"] = "1" if alg == 3 else "0"
    dA = csr_matrix(A, device=dev)
    B_src = csr_matrix(B, device=dev) if rank == 0 else None
    (r0, r1), A_blk, _ = distributed.rowblock_setup(dA, dA.indptr.new_tensor(B.indptr), world, rank)
    C, _ = distributed.rowblock_step(A_blk, B_src, 0, dev, alg=alg, pipeline=True, n_groups=3)
    torch.cuda.synchronize()
    from spmm_amd import cusparse
    info = cusparse.plan_info(A_blk, csr_matrix(B, device=dev), alg=2)
    tv = distributed.rowblock_step.last
    np.savez(os.path.join(OUT, f"{name}_alg{alg}_{rank}.npz"), p=C.indptr.cpu().numpy().astype(np.int64),
             j=C.indices.cpu().numpy(), x=C.data.cpu().numpy(), rows=np.array([r0, r1]),
             pipelined=np.array([tv.pipelined]), groups=np.array(tv.groups).reshape(-1, 2),
             value_tiles=np.array([-(-info["tiles_per_row"] // max(1, info["record_group"]))]))
dist.destroy_process_group()
"""


def test_pipelined_rowblock_two_ranks_one_gpu(tmp_path):
    """rowblock_step(pipeline=True) with 2 ranks on cuda:0 (gloo): both plans agree on the
    tile geometry and the values go as 3 tile groups (ALG2), or both take the row-major
    fallback (ALG1; ALG3 with several chunks); the stitched C equals the oracle's bit for
    bit either way."""
    from spmm_amd import distributed
    port = _free_port()
    code = _REHEARSAL.replace("ROOT", repr(ROOT)).replace("OUT", repr(str(tmp_path)))
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=300)[0])
        except subprocess.TimeoutExpired:
            p.kill()
            logs.append(p.communicate()[0])
    assert all(p.returncode == 0 for p in procs), "\n".join(l[-3000:] for l in logs)
    cases = {c[0]: c for c in _cases()}
    for name, alg in [("sparse8192_f64", 2), ("dense2048_f64", 2), ("c128", 2), ("dense2048_f64", 1),
                      ("sparse8192_f64", 3), ("wide140k_f64", 2)]:
        _, A, B, alpha = cases[name]
        parts = [np.load(tmp_path / f"{name}_alg{alg}_{r}.npz") for r in range(2)]
        if alg == 2:   # pipelined: 3 value-tile groups on both ranks (fewer value tiles: one each)
            assert all(bool(q["pipelined"][0]) and len(q["groups"]) == min(3, int(q["value_tiles"][0]))
                       for q in parts), (name, alg)
        else:          # the fallback: one row-major values broadcast, spg_numeric
            assert not any(bool(q["pipelined"][0]) for q in parts), (name, alg)
        p = distributed.stitch_indptr([q["p"] for q in parts], [len(q["j"]) for q in parts])
        j = np.concatenate([q["j"] for q in parts])
        x = np.concatenate([q["x"] for q in parts])
        rp, rj, rx = oracle.spgemm(A, B, keep_zeros=True, sort=True, threads=16)
        assert np.array_equal(p, rp), name
        assert np.array_equal(j, rj), name
        assert np.array_equal(_bits(x), _bits(rx)), name


def test_numeric_tiles_argument_errors():
    """spg_numeric_tiles rejects a range past the last tile (SPG_STATUS_INVALID_VALUE), and the
    shim rejects groups that skip or leave out tiles."""
    from spmm_amd import _lib, cusparse
    from spmm_amd.sparse import csr_matrix
    name, A, B, alpha = next(c for c in _cases() if c[0] == "dense2048_f64")
    dA, dB = csr_matrix(A, device="cuda:0"), csr_matrix(B, device="cuda:0")

    def past_end(geom):
        return geom["tile_values"](), [(0, geom["tiles"] + 1)]

    with pytest.raises(_lib.SpgError) as e:
        cusparse._spgemm(dA, dB, alg=2, by_tiles=past_end)
    assert e.value.status == 3   # SPG_STATUS_INVALID_VALUE

    def gap(geom):
        return geom["tile_values"](), [(0, 1), (2, geom["tiles"])]

    with pytest.raises(RuntimeError, match="consecutive"):
        cusparse._spgemm(dA, dB, alg=2, by_tiles=gap)

    def short(geom):
        return geom["tile_values"](), [(0, geom["tiles"] - 1)]

    with pytest.raises(RuntimeError, match="covered"):
        cusparse._spgemm(dA, dB, alg=2, by_tiles=short)
    torch.cuda.synchronize()


@pytest.mark.parametrize("ip", [torch.int32, torch.int64])
def test_cols16_kernels(ip):
    """spg_cols16_split / spg_cols16_join (the structure broadcast's 16-bit columns) against
    the host split and the original columns: the block-edge rows of _edge_csr at several
    widths, and a 20000 x 300000 random B (nnz ~ 2.4M)."""
    import scipy.sparse as sp
    from spmm_amd import cusparse, distributed
    from spmm_amd.sparse import csr_matrix
    from tests.test_distributed_gloo import _edge_csr
    mats = [_edge_csr(c) for c in (7, 65536, 65537, 131073, 300000)]
    mats.append(sp.random(20000, 300000, density=4e-4, format="csr", random_state=np.random.default_rng(3)))
    for Bh in mats:
        Bh.sort_indices()
        M = csr_matrix(Bh, device="cuda:0")
        M = csr_matrix._from_parts(M.data, M.indices, M.indptr.to(ip), M.shape, canonical=True)
        nb1 = cusparse._cols16_nb1(Bh.shape[1])
        starts, lo16 = cusparse._cols16_split(M)
        hs, hl = distributed._cols16_split_host(csr_matrix(Bh, device="cpu"), nb1)
        assert torch.equal(starts.cpu(), hs), Bh.shape
        assert torch.equal(lo16.cpu(), hl), Bh.shape
        back = cusparse._cols16_join(M.indptr, starts, lo16, Bh.shape)
        torch.cuda.synchronize()
        assert back.dtype == torch.int32 and np.array_equal(back.cpu().numpy(), Bh.indices), Bh.shape
