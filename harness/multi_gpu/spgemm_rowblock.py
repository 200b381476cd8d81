#!/usr/bin/env python3
"""Multi-GPU C = A.B, 1-D row blocks of A, B broadcast over RCCL/xGMI (BASELINE config 5:
N = 262144, density 1e-3, 8 x MI355X).

Launch:  python -m torch.distributed.run --nproc-per-node G --master-addr 127.0.0.1 \\
             harness/multi_gpu/spgemm_rowblock.py --n 262144 --density 1e-3

* strong scaling: the global N x N problem is fixed; every rank draws the whole A (the same
  seed everywhere), rank 0 draws B; one broadcast of B gives every rank B's row lengths,
  and rank r keeps the rows [r0, r1) cut on the product-count prefix (equal products per
  rank, spmm_amd.distributed.rowblock_setup);
* a timed step is spmm_amd.distributed.rowblock_step: B broadcast from rank 0 (metadata, one
  packed structure buffer, then the values in tile-major groups, each group's numeric tiles
  launched as it lands -- or, if a plan cannot run by tiles, one values broadcast left in
  flight through the symbolic pass) and this rank's slab; GFLOPS = sum_r 2 P_r / max_r t_r; the broadcast alone is timed beside it;
  allgather of the per-rank nnz gives the global row-pointer offsets;
* --check S: S sampled rows per rank are recomputed on the host with the CPU oracle
  (tests/ oracle, parity check only) and compared bit for bit.
Prints one JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--density", type=float, default=1e-3)
    ap.add_argument("--alg", type=int, default=2)
    ap.add_argument("--chunk-fraction", type=float, default=0.2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--check", type=int, default=16, help="sampled rows per rank checked on the host")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from spmm_amd import cusparse, distributed, gen

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_dev = local % max(1, torch.cuda.device_count())   # (a gloo rehearsal may share a GPU)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        backend = os.environ.get("SPG_DIST_BACKEND", "nccl")   # nccl = RCCL on ROCm
        dist.init_process_group(backend, **({"device_id": dev} if backend == "nccl" else {}))

    n = args.n
    A = gen.random_csr(n, n, args.density, seed=args.seed, device=dev)
    B0 = gen.random_csr(n, n, args.density, seed=args.seed + 1, device=dev) if rank == 0 or world == 1 else None
    bcast_ms = 0.0
    if world > 1:
        Bw = distributed.broadcast_csr(B0, 0, dev)
        (r0, r1), A, P = distributed.rowblock_setup(A, Bw.indptr, world, rank)
        del Bw
        ts = []
        for _ in range(2):
            torch.cuda.synchronize(); dist.barrier()
            t0 = time.perf_counter()
            Bt = distributed.broadcast_csr(B0, 0, dev)
            torch.cuda.synchronize(); dist.barrier()
            ts.append(time.perf_counter() - t0)
            del Bt
        bcast_ms = float(np.median(ts)) * 1e3

        def step():
            return distributed.rowblock_step(A, B0, 0, dev, args.alg, args.chunk_fraction)
    else:
        r0, r1 = 0, n
        P = cusparse.num_products(A, B0)

        def step():
            return distributed.spgemm_rowblock(A, B0, args.alg, args.chunk_fraction), B0
    C = None
    for _ in range(args.warmup):
        C, B = step()
        del C
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        C = None   # (the previous slab is freed before the next one is built)
        C, B = step()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    peak = cusparse.last_stats.peak_bytes
    nnzs = distributed.allgather_nnz(C.nnz, dev) if world > 1 else [C.nnz]

    # sampled-row parity against the CPU oracle
    bad = 0
    if args.check > 0:
        from oracle import oracle
        import scipy.sparse as sp
        rng = np.random.default_rng(rank)
        rows = np.sort(rng.choice(r1 - r0, size=min(args.check, r1 - r0), replace=False))
        Ah = A.get()[rows]
        # (after a pipelined step B's values are row-major on rank 0 only: fetch them whole)
        Bh = (distributed.broadcast_csr(B0 if rank == 0 else None, 0, dev) if world > 1 else B).get()
        ref = oracle.spgemm(sp.csr_matrix(Ah), Bh, keep_zeros=True, sort=True)
        cp = C.indptr.cpu().numpy().astype(np.int64)
        for q, i in enumerate(rows):
            s, e = cp[i], cp[i + 1]
            rs, re = ref[0][q], ref[0][q + 1]
            if not (np.array_equal(C.indices[s:e].cpu().numpy(), ref[1][rs:re]) and
                    np.array_equal(C.data[s:e].cpu().numpy().view(np.uint8), ref[2][rs:re].view(np.uint8))):
                bad += 1

    vals = torch.tensor([t, float(P), float(C.nnz), float(peak), float(bad)], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = vals[:1].clone(); dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        sums = vals[1:3].clone(); dist.all_reduce(sums)
        pk = vals[3:4].clone(); dist.all_reduce(pk, op=dist.ReduceOp.MAX)
        bd = vals[4:5].clone(); dist.all_reduce(bd)
        t, P_all, nnz_all, peak, bad = float(tmax[0]), float(sums[0]), float(sums[1]), float(pk[0]), float(bd[0])
    else:
        P_all, nnz_all = float(P), float(C.nnz)
    if rank == 0:
        print(json.dumps({
            "metric": "CSR×CSR SpGEMM GFLOPS (row-block shards, B broadcast)",
            "n_gpus": world, "N": n, "density": args.density, "alg": args.alg,
            "gflops": round(2.0 * P_all * args.steps / t / 1e9, 3),
            "ms_per_step": round(t / args.steps * 1e3, 3), "num_products": int(P_all),
            "nnzC": int(nnz_all), "nnz_per_rank": nnzs, "peak_hbm_bytes_per_gpu": int(peak),
            "b_broadcast_ms": round(bcast_ms, 3), "sampled_rows_checked": args.check * world,
            "sampled_rows_bad": int(bad)}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if bad:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
