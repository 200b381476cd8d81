"""Multi-GPU C = A.B: 1-D row-block sharding of A, B broadcast over RCCL/xGMI.

Rows of C depend only on the same rows of A and on all of B, so each rank
owns a contiguous row block of A, receives B, and writes its own C slab -- there is no
cross-GPU reduction.  The collectives are

* ``broadcast_csr``: B from ``src`` to every rank: one 7-int64 metadata broadcast (the
  reference's sparse broadcast protocol, modify_src/cupy-src/cupyx/distributed/
  _nccl_comm.py:651-674, metadata exchange :506-530), then the structure (row pointer and
  column indices packed into ONE buffer; the columns as 16-bit low halves, plus each row's
  65536-column block starts when B is wider -- spg_cols16_split / spg_cols16_join) and the
  values (a second buffer), each a single
  RCCL broadcast -- the reference groups its three payload broadcasts between
  groupStart/groupEnd (:669); two packed buffers are the same "few large collectives" on
  torch.distributed.  With ``async_values=True`` the values broadcast is left in flight and
  its work handle returned, so the symbolic pass (which reads only B's structure) runs
  while the values arrive (``spgemm_rowblock``'s ``before_numeric`` waits for them);
* ``TileValueBroadcast`` (``rowblock_step(..., pipeline=True)``, the default on GPUs):
  B's structure as above; each rank plans and lays out its tiles from the structure alone
  (spg_tile_value_offsets); then B's values go out in TILE-MAJOR order (spg_tile_values on
  ``src``: the entries of column tile 0 row by row, then tile 1, ...) as one async
  broadcast per group of column tiles, BEFORE the symbolic pass, which runs while they
  travel; each group's numeric tiles (spg_numeric_tiles) start when its slice lands, so
  the values broadcast overlaps the symbolic pass and the numeric pass.  The ranks first
  agree (one 4-int64 all_gather that every rank reaches exactly once per step, a local
  failure included) that every plan runs by tiles with the same tile width; otherwise the
  step falls back to the row-major values broadcast and spg_numeric, and a rank that failed
  before the agreement makes every rank raise (StepFailed) rather than hang;
* ``allgather_nnz``: every rank's nnz(C slab) -> global row-pointer offsets, when a
  stitched C is wanted.

``row_blocks`` balances rows by the product-count prefix (equal FLOPs per rank);
``product_prefix`` computes that prefix on the device.  Backend "nccl" = RCCL on ROCm;
"gloo" in the CPU tests.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .sparse import csr_matrix

_DT_CODE = {torch.float32: 0, torch.float64: 1, torch.complex64: 2, torch.complex128: 3}
_CODE_DT = {v: k for k, v in _DT_CODE.items()}
_IP_CODE = {torch.int32: 0, torch.int64: 1}
_CODE_IP = {v: k for k, v in _IP_CODE.items()}


def _bytes_of(t: torch.Tensor) -> torch.Tensor:
    return t.contiguous().view(-1).view(torch.uint8)


def cols16_layout(rows: int, cols: int, nnz: int) -> int:
    """Interior block starts per row when B's columns travel as 16-bit low halves, or -1
    when they travel as int32: a matrix at most 65536 wide needs no starts (nb1 = 0); a
    wider one uses them while 4 bytes per row and block + 2 per entry beat 4 per entry
    (config 5's B: 141 MB of structure instead of 276 MB)."""
    from .cusparse import _cols16_nb1
    nb1 = _cols16_nb1(cols)
    return nb1 if 4 * rows * nb1 + 2 * nnz < 4 * nnz or nb1 == 0 else -1


def _cols16_split_host(M: csr_matrix, nb1: int):
    """spg_cols16_split's result for a host CSR (the gloo tests' CPU tensors)."""
    rows = M.shape[0]
    ip = M.indptr.to(torch.int64)
    row = torch.repeat_interleave(torch.arange(rows), ip[1:] - ip[:-1])
    hi = (M.indices.to(torch.int64) >> 16).clamp(max=nb1)
    cnt = torch.bincount(row * (nb1 + 1) + hi, minlength=rows * (nb1 + 1)).view(rows, nb1 + 1)
    starts = cnt.cumsum(1)[:, :nb1].to(torch.int32).contiguous()
    return starts, M.indices.contiguous().view(torch.int16)[0::2].contiguous()


def _cols16_join_host(indptr: torch.Tensor, starts: torch.Tensor, lo16: torch.Tensor) -> torch.Tensor:
    """spg_cols16_join's result on host tensors."""
    ip = indptr.to(torch.int64)
    rows = ip.numel() - 1
    row = torch.repeat_interleave(torch.arange(rows), ip[1:] - ip[:-1])
    pos = torch.arange(lo16.numel()) - ip[:-1][row]
    blk = (pos[:, None] >= starts.to(torch.int64)[row]).sum(1) if starts.shape[1] else torch.zeros_like(pos)
    return ((blk << 16) | (lo16.to(torch.int64) & 0xffff)).to(torch.int32)


def _rows_sorted(M: csr_matrix) -> bool:
    """Column indices non-decreasing inside every row (what the 16-bit column encoding
    needs; duplicates are fine).  One device reduction and one host read."""
    if M._canonical is True or M.nnz < 2:
        return True
    idx = M.indices.to(torch.int64)
    ok = idx[1:] >= idx[:-1]
    starts = M.indptr[1:-1].to(torch.int64)   # first entry of rows 1..m-1
    starts = starts[(starts > 0) & (starts < M.nnz)]
    ok[starts - 1] = True                      # a row boundary may step down
    return bool(ok.all())


def broadcast_csr(M: csr_matrix | None, src: int, device, group=None, async_values: bool = False,
                  values: bool = True):
    """Broadcast a CSR matrix held by rank `src` to every rank of `group`.

    Returns the matrix, or ``(matrix, work)`` with ``async_values=True``: the values
    broadcast is still in flight and ``work.wait()`` orders the current stream after it
    (``work`` is None when there is nothing to wait for).  ``values=False`` broadcasts the
    structure only: off `src` the matrix's values are an uninitialised buffer (filled later,
    e.g. by ``send_values``).

    The metadata carries the column encoding `src` chose (so every rank decodes what was
    sent) and `src`'s canonical flag: a B whose rows are not sorted travels with int32
    columns, exactly in its stored order, and arrives marked as `src` knew it."""
    rank = dist.get_rank(group)
    meta = torch.zeros(7, dtype=torch.int64, device=device)
    if rank == src:
        # column indices travel as their low 16 bits (exact) plus, for a matrix wider than
        # 65536, each row's 65536-column block starts (cols16_layout): about half the
        # structure bytes -- the part of the step's broadcast every rank waits for before its
        # plan.  The encoding needs rows sorted by column; otherwise int32 (nb1 = -1).
        nb1 = cols16_layout(M.shape[0], M.shape[1], M.nnz)
        if nb1 > 0 and not _rows_sorted(M):
            nb1 = -1
        canon = {True: 1, False: 0, None: -1}[M._canonical]
        meta = torch.tensor([M.shape[0], M.shape[1], M.nnz, _DT_CODE[M.data.dtype],
                             _IP_CODE[M.indptr.dtype], nb1, canon], dtype=torch.int64, device=device)
    dist.broadcast(meta, src, group=group)
    rows, cols, nnz, dtc, ipc, nb1, canon = (int(x) for x in meta.tolist())
    canonical = {1: True, 0: False, -1: None}[canon]
    ipt = _CODE_IP[ipc]
    ib = torch.empty(0, dtype=ipt).element_size()
    pbytes = ib * (rows + 1)
    sbytes = pbytes + (4 * nnz if nb1 < 0 else 4 * rows * nb1 + 2 * nnz)   # indptr | [starts |] indices
    dev_t = torch.device(device).type
    if rank == src:
        parts = [_bytes_of(M.indptr.to(device))]
        if nb1 < 0:
            parts.append(_bytes_of(M.indices.to(device)))
        else:
            Mi = csr_matrix._from_parts(M.data.to(device), M.indices.to(device), M.indptr.to(device), M.shape,
                                        canonical=M._canonical)
            if dev_t == "cuda":
                from .cusparse import _cols16_split
                starts, lo16 = _cols16_split(Mi)
            else:
                starts, lo16 = _cols16_split_host(Mi, nb1)
            parts += [_bytes_of(starts), _bytes_of(lo16)] if nb1 else [_bytes_of(lo16)]
        struct = torch.cat(parts)
        data = M.data.to(device).contiguous()
    else:
        struct = torch.empty(sbytes, dtype=torch.uint8, device=device)
        data = torch.empty(nnz, dtype=_CODE_DT[dtc], device=device)
    dist.broadcast(struct, src, group=group)
    work = None
    if nnz and values:
        if async_values:
            work = dist.broadcast(_bytes_of(data), src, group=group, async_op=True)
        else:
            dist.broadcast(_bytes_of(data), src, group=group)
    indptr = struct[:pbytes].view(ipt)
    if rank == src:
        indices = M.indices.to(device)
    elif nb1 < 0:
        indices = struct[pbytes:].view(torch.int32)
    else:
        starts = struct[pbytes:pbytes + 4 * rows * nb1].view(torch.int32).view(rows, nb1)
        lo16 = struct[pbytes + 4 * rows * nb1:].view(torch.int16)
        if dev_t == "cuda":
            from .cusparse import _cols16_join
            indices = _cols16_join(indptr, starts, lo16, (rows, cols))
        else:
            indices = _cols16_join_host(indptr, starts, lo16)
    out = csr_matrix._from_parts(data, indices, indptr, (rows, cols), canonical=canonical)
    return (out, work) if async_values else out


@torch.no_grad()
def product_prefix(A: csr_matrix, b_indptr: torch.Tensor) -> torch.Tensor:
    """int64 prefix of the per-row product counts of A.B (length rows + 1), on A's device:
    P_i = sum over row i's entries k of B's row length (cusparse getNumProducts, per row)."""
    blen = (b_indptr[1:] - b_indptr[:-1]).to(torch.int64)
    prod = blen[A.indices.to(torch.int64)]
    pref = torch.zeros(A.nnz + 1, dtype=torch.int64, device=prod.device)
    torch.cumsum(prod, 0, out=pref[1:])
    return pref[A.indptr.to(torch.int64)]   # entry prefix at each row start


def row_slice(A: csr_matrix, r0: int, r1: int) -> csr_matrix:
    """Rows [r0, r1) of A as its own CSR (copies: the slab owns its arrays)."""
    ip = A.indptr
    s, e = int(ip[r0]), int(ip[r1])
    indptr = (ip[r0:r1 + 1] - ip[r0]).clone()
    return csr_matrix._from_parts(A.data[s:e].clone(), A.indices[s:e].clone(), indptr,
                                  (r1 - r0, A.shape[1]), canonical=True)


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


def spgemm_rowblock(A_block: csr_matrix, B: csr_matrix, alg: int = 0, chunk_fraction: float = 0.2,
                    before_numeric=None):
    """This rank's C slab = A_block . B (row block r0:r1 of the global C).  `before_numeric`
    (e.g. the values broadcast's ``work.wait``) runs after the symbolic pass, before the
    numeric pass reads B's values."""
    from . import cusparse
    if before_numeric is None:
        return cusparse.spgemm(A_block, B, alg=alg, chunk_fraction=chunk_fraction)
    return cusparse._spgemm(A_block, B, alg=alg, chunk_fraction=chunk_fraction, before_numeric=before_numeric)


def rowblock_setup(A: csr_matrix, b_indptr: torch.Tensor, world: int, rank: int):
    """This rank's row block of A: the cut on the product-count prefix (equal products per
    rank), the block as its own CSR, and its product count.  Returns ((r0, r1), A_block, P_r)."""
    pref = product_prefix(A, b_indptr).cpu().numpy()
    r0, r1 = row_blocks(A.shape[0], world, pref)[rank]
    return (r0, r1), row_slice(A, r0, r1), int(pref[r1] - pref[r0])


def rowblock_setup_drawn(draw, n_rows: int, b_indptr: torch.Tensor, world: int, rank: int, group=None):
    """rowblock_setup without any rank holding all of A: `draw(rows, row_offset)` returns
    rows [row_offset, row_offset + rows) of the global A (spmm_amd.gen.random_csr draws any
    row range of its matrix).  Every rank draws an equal-row block, its per-row product
    counts are gathered, every rank cuts the global product prefix the same way, and a rank
    whose cut block differs draws it.  Returns ((r0, r1), A_block, P_r)."""
    q = [(n_rows * r) // world for r in range(world + 1)]
    A0 = draw(q[rank + 1] - q[rank], q[rank])
    pre = product_prefix(A0, b_indptr)
    per_row = (pre[1:] - pre[:-1]).to(torch.int64)
    width = max(q[r + 1] - q[r] for r in range(world))
    mine = torch.zeros(width, dtype=torch.int64, device=per_row.device)
    mine[:per_row.numel()] = per_row
    parts = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    counts = torch.cat([parts[r][:q[r + 1] - q[r]] for r in range(world)]).cpu().numpy()
    pref = np.zeros(n_rows + 1, dtype=np.int64)
    np.cumsum(counts, out=pref[1:])
    r0, r1 = row_blocks(n_rows, world, pref)[rank]
    A = A0 if (r0, r1) == (q[rank], q[rank + 1]) else draw(r1 - r0, r0)
    return (r0, r1), A, int(pref[r1] - pref[r0])


def tile_groups(offsets, n_groups: int):
    """Consecutive column-tile ranges [(g0, g1)] for the pipelined values broadcast: about
    equal VALUE counts per group (cut on the tile-major offsets), at most n_groups, every
    group non-empty in tiles."""
    offs = np.asarray(offsets, dtype=np.int64)
    G = len(offs) - 1
    k = max(1, min(int(n_groups), G))
    cuts = [0]
    for i in range(1, k):
        c = int(np.searchsorted(offs, (int(offs[-1]) * i) // k, side="left"))
        cuts.append(min(max(c, cuts[-1] + 1), G - (k - i)))
    cuts.append(G)
    return [(cuts[i], cuts[i + 1]) for i in range(k)]


class StepFailed(RuntimeError):
    """A rank of the step failed before the ranks agreed on how B's values travel; every
    rank raises this (or the failing rank its own error) instead of blocking in a collective
    its peers never enter."""


# agreement codes (the first word of agree_tiles' all_gather)
_AGREE_TILES, _AGREE_ROWMAJOR, _AGREE_FAILED = 1, 0, -1


def agree_tiles(geom, device, group=None, failed: bool = False) -> bool:
    """The one agreement of a pipelined step, reached by every rank exactly once (one 4-int64
    all_gather): True when every rank's plan runs by tiles with the same tile width, tile
    count and value type; False when some rank cannot (``geom`` None: not the tile path, ALG1,
    several row chunks, an A block that promotes B) -- the values then go row-major to all.
    A rank that failed locally before this point reports ``failed=True``; every rank then
    raises StepFailed, so no rank is left in a collective its peers skip."""
    world = dist.get_world_size(group)
    if dist.get_backend(group) != "nccl":
        device = "cpu"   # gloo (the rehearsal on one GPU) gathers host tensors
    if failed:
        words = [_AGREE_FAILED, 0, 0, -1]
    elif geom is None:
        words = [_AGREE_ROWMAJOR, 0, 0, -1]
    else:
        words = [_AGREE_TILES, geom["tile_width"], geom["tiles"], _DT_CODE[geom["dtype"]]]
    mine = torch.tensor(words, dtype=torch.int64, device=device)
    out = [torch.zeros(4, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(out, mine, group=group)
    rows = [tuple(int(v) for v in t.tolist()) for t in out]
    bad = [r for r, w in enumerate(rows) if w[0] == _AGREE_FAILED]
    if bad:
        raise StepFailed(f"rank(s) {bad} failed before the values broadcast; the step is abandoned on every rank")
    return rows[0][0] == _AGREE_TILES and all(r == rows[0] for r in rows)


class TileValueBroadcast:
    """The `by_tiles` protocol of cusparse._spgemm for one row-block step (see module doc):
    agree on the tile geometry, then `src` permutes B's values tile-major and every group
    goes out as its own async broadcast; receivers yield a group once its work is waited
    on (the current stream is ordered after it).  On disagreement the row-major values go
    out in one broadcast and spg_numeric runs.  After the product, `overlap` holds
    (groups, values bytes) for the report; `finish()` orders the current stream after
    every broadcast (the source's numeric tiles do not wait for its own sends).

    Every rank calls it (or `fail`) exactly once per step: `agreed` records that it did."""

    def __init__(self, B: csr_matrix, src: int, device, group=None, n_groups: int = 8):
        self.B, self.src, self.device, self.group, self.n_groups = B, src, device, group, n_groups
        self.works = []
        self.pipelined = False
        self.agreed = False
        self.groups = []

    def __call__(self, geom):
        if self.agreed:
            raise RuntimeError("TileValueBroadcast called twice in one step")
        rank = dist.get_rank(self.group)
        self.agreed = True
        if not agree_tiles(geom, self.device, self.group):
            if self.B.nnz:
                dist.broadcast(_bytes_of(self.B.data), self.src, group=self.group)
            return None
        self.pipelined = True
        offs = geom["offsets"]
        if rank == self.src:
            tm = geom["tile_values"]()
        else:
            # the plan's value type, which every rank agreed on (agree_tiles), not the buffer's
            tm = torch.empty(self.B.nnz, dtype=geom["dtype"], device=self.device)
        self.groups = tile_groups(offs, self.n_groups)
        works = []
        for g0, g1 in self.groups:
            a, b = int(offs[g0]), int(offs[g1])
            works.append(dist.broadcast(_bytes_of(tm[a:b]), self.src, group=self.group, async_op=True)
                         if b > a else None)
        self.works = works
        return tm, self._release(rank)

    def fail(self):
        """This rank failed before reaching the agreement: tell the others (they raise
        StepFailed); the caller re-raises its own error.  A no-op once the rank has agreed."""
        if not self.agreed:
            self.agreed = True
            try:
                agree_tiles(None, self.device, self.group, failed=True)
            except StepFailed:
                pass   # (this rank raises its own error)

    def _release(self, rank):
        for (g0, g1), w in zip(self.groups, self.works):
            if w is not None and rank != self.src:
                w.wait()
            yield g0, g1

    def finish(self):
        """Order the current stream after every outstanding broadcast (also after a failed
        multiply: peers must not be left blocked in a group broadcast) and drop the
        references to B and its values."""
        works, self.works = self.works, []
        for w in works:
            if w is not None:
                w.wait()
        self.B = None

    def report(self):
        """(pipelined, groups) of the step, for the bench line (no tensors kept alive)."""
        return StepReport(self.pipelined, list(self.groups))


class StepReport:
    """What the last rowblock_step did (rowblock_step.last): only report fields."""

    def __init__(self, pipelined: bool, groups):
        self.pipelined, self.groups = pipelined, groups


def _device_multiply_tiles(A_block, B, alg, chunk_fraction, by_tiles, values_first):
    """The pipelined step's device multiply (rowblock_step's `multiply_tiles` default)."""
    if by_tiles is None:
        return spgemm_rowblock(A_block, B, alg, chunk_fraction)
    from . import cusparse
    return cusparse._spgemm(A_block, B, alg=alg, chunk_fraction=chunk_fraction, by_tiles=by_tiles,
                            values_first=values_first)


def rowblock_step(A_block: csr_matrix, B_src: csr_matrix | None, src: int, device, alg: int = 2,
                  chunk_fraction: float = 0.2, multiply=None, group=None, pipeline: bool | None = None,
                  n_groups: int = 8, values_first: bool = True, multiply_tiles=None):
    """One C = A.B step of the row-block scheme on this rank: B arrives from `src` (its
    structure first; the values stay in flight through the symbolic pass and, pipelined,
    the numeric tiles), then this
    rank's slab A_block . B.  `multiply(A_block, B, wait_values)` replaces the device
    multiply (the gloo tests run the CPU oracle there).  `pipeline` (default: on a GPU
    device): the values travel tile-major in `n_groups` async broadcasts, each group's
    numeric tiles starting as its slice lands (TileValueBroadcast); `values_first` (default)
    sends them before the symbolic pass, False after it (round 4's order, for comparison).

    Returns (C slab, B).  After a pipelined step B's values exist row-major on `src` only,
    so the other ranks get None for B (their B never held row-major values).  A_block is
    cast to B's value type when that type is the common one; otherwise (B would have to be
    promoted after its values arrive) this rank votes for the row-major values broadcast in
    the one agreement every rank reaches (agree_tiles), and every rank takes it.

    Failure before the agreement (planning, the tile layout, the symbolic pass of the
    values-after order, ...) on any rank makes every rank raise (StepFailed on the others)
    instead of leaving them in a collective; failure after it leaves the peers' step intact
    (the failing rank still waits for its outstanding broadcasts).

    `multiply_tiles(A_block, B, alg, chunk_fraction, by_tiles, values_first)` replaces the
    pipelined device multiply (cusparse._spgemm with `by_tiles`; ``by_tiles=None``: B's
    values are complete row-major) -- the gloo tests drive the protocol through a CPU one."""
    if pipeline is None:
        pipeline = multiply is None and torch.device(device).type == "cuda"
    if pipeline and multiply is None:
        B, _ = broadcast_csr(B_src, src, device, group, async_values=True, values=False)
        tv = TileValueBroadcast(B, src, device, group, n_groups)
        mul = multiply_tiles or _device_multiply_tiles
        try:
            if A_block.data.dtype != B.data.dtype:
                common = np.promote_types(A_block.dtype, B.dtype)
                if common == B.dtype:
                    A_block = A_block.astype(common)
            if A_block.data.dtype == B.data.dtype:
                C = mul(A_block, B, alg, chunk_fraction, tv, values_first)
            else:
                # B must be promoted after its values arrive: vote for the row-major values
                tv(None)
                C = mul(A_block, B, alg, chunk_fraction, None, values_first)
        except StepFailed:
            raise
        except BaseException:
            tv.fail()   # (a no-op after the agreement)
            raise
        finally:
            tv.finish()
        rowblock_step.last = tv.report()
        rank = dist.get_rank(group)
        return C, (B if (rank == src or not tv.pipelined) else None)
    B, work = broadcast_csr(B_src, src, device, group, async_values=True)
    wait = work.wait if work is not None else (lambda: None)
    rowblock_step.last = StepReport(False, [])
    if multiply is not None:
        return multiply(A_block, B, wait), B
    return spgemm_rowblock(A_block, B, alg, chunk_fraction, before_numeric=wait), B


rowblock_step.last = None


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
