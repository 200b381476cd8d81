#!/usr/bin/env python3
"""CSR x CSR SpGEMM benchmark on MI355X (BASELINE.json metric: GFLOPS + peak HBM bytes).

Step = one complete ``C = A.B`` through the drop-in shim (``spmm_amd.cusparse.spgemm``:
plan, symbolic with its nnz(C) host sync, C allocation, numeric), inputs resident in HBM.

Workloads (``--config``; ``auto`` = 2 on one GPU, 5 on several):

* ``2`` (N=1 default, BASELINE configs[1]): random 16384 x 16384, density 1e-3, fp64, A then
  B from one ``default_rng(42)`` stream via scipy.sparse.random (nnz(C) = 4,366,124,
  P = 4,402,284), ALG1 single pass.
* ``4``: N = 65536, density 5e-3, fp64, ALG3 chunked (chunk_fraction 0.2): nnz(C) = 3.46e9,
  int64 row pointer.  Inputs generated on the device (spmm_amd.gen.random_csr).
* ``5``: N = 262144, density 1e-3, fp64, ALG2, strong scaling over the ranks: rank r owns
  the rows [r0, r1) cut on the product-count prefix, B (826 MB) is broadcast from rank 0
  over RCCL/xGMI INSIDE every step -- structure first, values in flight while the
  symbolic pass runs (spmm_amd.distributed.rowblock_step) -- and every rank writes its own
  C slab: no reduction.  value = sum_r 2 P_r per step / max-over-ranks step time.  At
  ``--gpus 1`` it is the whole problem on one GPU (200 GB of C and workspace fit in 288 GB).

Also reported: ``roofline`` for the numeric-phase kernel (compulsory bytes of the product,
SURVEY 8d, / the phase's device time from HIP events on the library's stream, per launch),
``cpu_baseline`` = scipy's ``A @ B`` -- the reference's CPU comparator
(SpGEMM_vs_SpMV/profiler.py:408) -- timed in forked children with their RSS growth, on
rank 0 at N=1 (the whole product for config 2, a bounded row sample beyond), with the
oracle's single-thread and OpenMP restatements beside it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CSR×CSR SpGEMM GFLOPS + peak HBM bytes, random N×N at stated density"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    "2": dict(n=16384, density=1e-3, alg=1, gen="scipy", steps=200, warmup=20,
              name="BASELINE config 2 (configs[1])"),
    "4": dict(n=65536, density=5e-3, alg=3, gen="device", steps=5, warmup=2,
              name="BASELINE config 4 (ALG3 chunked, HBM-capped)"),
    "5": dict(n=262144, density=1e-3, alg=2, gen="device", steps=5, warmup=2,
              name="BASELINE config 5 (row blocks, B broadcast)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default per config)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default per config)")
    ap.add_argument("--config", default="auto", choices=["auto", "2", "4", "5"])
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--density", type=float, default=None)
    ap.add_argument("--alg", type=int, default=None)
    ap.add_argument("--chunk-fraction", type=float, default=0.2)
    ap.add_argument("--dtype", default="float64", choices=["float32", "float64"])
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="budget of the CPU-baseline sample (0 disables it)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="PMC traffic summary written by profiles/pmc_to_json.py")
    return ap.parse_args()


def compulsory_bytes(n_rows, n_cols, nnzA, nnzB, nnzC, vb, ib_c=4):
    """SURVEY 8d compulsory bytes: A and B read once (int32 row pointers), C written once
    (its row pointer ib_c bytes per entry: 8 once nnz(C) >= 2^31)."""
    return 4 * (n_rows + 1) + 4 * (n_cols + 1) + ib_c * (n_rows + 1) + (4 + vb) * (nnzA + nnzB + nnzC)


def cpu_baseline(A_h, B_h, rows_sample, budget_s):
    """scipy A @ B (the reference's comparator) in forked children: median time and RSS
    growth; the oracle port (single thread) and its OpenMP form beside it.  On a row sample
    of A when `rows_sample` is given (configs 4/5: C does not fit a host sample budget)."""
    import scipy.sparse as sp
    from oracle import oracle
    from spmm_amd import profiling
    A_s = A_h if rows_sample is None else sp.csr_matrix(A_h[rows_sample])
    P = oracle.num_products(A_s, B_h)
    runs, t_start = [], time.perf_counter()
    while len(runs) < 30 and (len(runs) < 3 or time.perf_counter() - t_start < budget_s):
        runs.append(profiling.profile_op_cpu("scipy A@B", lambda: A_s @ B_h))
    t = float(np.median([r.time_ms for r in runs])) / 1e3
    rss = int(np.median([r.peak_ram or 0 for r in runs]))
    oracle.build()
    pt = []
    t_start = time.perf_counter()
    while len(pt) < 20 and (len(pt) < 2 or time.perf_counter() - t_start < budget_s / 2):
        t0 = time.perf_counter()
        oracle.spgemm(A_s, B_h, keep_zeros=True, sort=True)
        pt.append(time.perf_counter() - t0)
    nthr = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    om = []
    t_start = time.perf_counter()
    while len(om) < 20 and (len(om) < 2 or time.perf_counter() - t_start < budget_s / 2):
        t0 = time.perf_counter()
        oracle.spgemm(A_s, B_h, keep_zeros=True, sort=True, threads=nthr)
        om.append(time.perf_counter() - t0)
    t_port, t_omp = float(np.median(pt)), float(np.median(om))
    what = ("the whole product (same A, B)" if rows_sample is None
            else f"{len(rows_sample)} sampled rows of A times all of B ({P} products)")
    return {"value": round(2.0 * P / t / 1e9, 4), "unit": "GFLOPS", "cores": 1, "kind": "reference",
            "sample": f"scipy.sparse A@B (csr_matmat, single thread; the reference's CPU comparator, "
                      f"SpGEMM_vs_SpMV/profiler.py:408) on {what}, median of {len(runs)} forked runs",
            "ms_per_run": round(t * 1e3, 3), "rss_growth_bytes": rss,
            "port": {"gflops": round(2.0 * P / t_port / 1e9, 4), "ms_per_run": round(t_port * 1e3, 3),
                     "threads": 1, "what": "oracle/gustavson.c (scipy's rule restated in C)"},
            "omp": {"gflops": round(2.0 * P / t_omp / 1e9, 4), "ms_per_run": round(t_omp * 1e3, 3),
                    "threads": nthr, "what": "oracle/gustavson.c, OpenMP over rows"},
            "host_cpus": os.cpu_count()}


def traffic_for(pmc_path, key, build_id, source_id=None):
    """HBM bytes per launch from the committed PMC summary -- only when it was collected on
    this very build of the library, or on a build of the same sources (else None: the
    number would be stale)."""
    if not os.path.exists(pmc_path):
        return None, None
    try:
        with open(pmc_path) as f:
            e = json.load(f).get(key, {})
    except Exception:
        return None, None
    if e.get("build_id") != build_id and (source_id is None or e.get("source_id") != source_id):
        return None, e.get("build_id")
    return e.get("hbm_bytes_per_launch"), e.get("build_id")


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # one process per GPU; a rehearsal with more ranks than GPUs (SPG_DIST_BACKEND=gloo on a
    # one-GPU box) puts several ranks on one device
    local_dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        backend = os.environ.get("SPG_DIST_BACKEND", "nccl")   # nccl = RCCL on ROCm
        dist.init_process_group(backend, **({"device_id": dev} if backend == "nccl" else {}))

    from spmm_amd import _lib, cusparse, distributed, gen
    from spmm_amd.sparse import csr_matrix

    cfg_name = args.config if args.config != "auto" else ("2" if world == 1 else "5")
    cfg = dict(CONFIGS[cfg_name])
    n = args.n or cfg["n"]
    dens = args.density or cfg["density"]
    alg = args.alg or cfg["alg"]
    steps = args.steps if args.steps is not None else cfg["steps"]
    warmup = args.warmup if args.warmup is not None else cfg["warmup"]
    cf = args.chunk_fraction
    if world > 1 and cfg_name != "5":
        raise SystemExit("several GPUs run the row-block workload (config 5)")
    npdt = np.float64 if args.dtype == "float64" else np.float32
    tdt = torch.float64 if args.dtype == "float64" else torch.float32
    vb = 8 if npdt == np.float64 else 4

    # ---- inputs in HBM (not timed)
    A_h = B_h = None
    if cfg["gen"] == "scipy":
        A_h, B_h = gen.scipy_pair(n, dens, seed=args.seed, dtype=npdt)
        A, B = csr_matrix(A_h, device=dev), csr_matrix(B_h, device=dev)
    else:
        A = gen.random_csr(n, n, dens, seed=args.seed, dtype=tdt, device=dev)
        B = gen.random_csr(n, n, dens, seed=args.seed + 1, dtype=tdt, device=dev) if rank == 0 or world == 1 else None

    bcast_ms = None
    rows = (0, n)
    if world > 1:
        # the row cut needs B's row lengths: one broadcast ahead of the timed steps (it also
        # warms RCCL up), then this rank's block of A
        Bw = distributed.broadcast_csr(B, 0, dev)
        nnzB = Bw.nnz
        rows, A, P_r = distributed.rowblock_setup(A, Bw.indptr, world, rank)
        del Bw
        torch.cuda.empty_cache()
        ts = []
        for _ in range(3):   # the broadcast alone (reported beside the step)
            torch.cuda.synchronize(); dist.barrier()
            t0 = time.perf_counter()
            Bt = distributed.broadcast_csr(B, 0, dev)
            torch.cuda.synchronize(); dist.barrier()
            ts.append(time.perf_counter() - t0)
            del Bt
        bcast_ms = float(np.median(ts)) * 1e3

        def step():
            C, _ = distributed.rowblock_step(A, B, 0, dev, alg=alg, chunk_fraction=cf)
            return C
        P = P_r
    else:
        def step():
            return cusparse.spgemm(A, B, alg=alg, chunk_fraction=cf)
        P = cusparse.num_products(A, B)
        nnzB = B.nnz

    # ---- warmup, then exactly K timed steps between barrier + synchronize
    C = None
    for _ in range(warmup):
        C = step()
        del C
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        C = step()
        if i < steps - 1:
            del C
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    nnzC = C.nnz
    ib_c = C.indptr.element_size()
    peak_bytes = cusparse.last_stats.peak_bytes
    del C
    torch.cuda.empty_cache()

    tot = torch.tensor([elapsed, float(P), float(nnzC), float(peak_bytes)], dtype=torch.float64, device=dev)
    if world > 1:
        mx = tot[:1].clone(); dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tot[1:3].clone(); dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        pk = tot[3:].clone(); dist.all_reduce(pk, op=dist.ReduceOp.MAX)
        elapsed, P_all, nnz_all, peak_max = float(mx[0]), float(sm[0]), float(sm[1]), float(pk[0])
    else:
        P_all, nnz_all, peak_max = float(P), float(nnzC), float(peak_bytes)
    ms_per_step = elapsed / steps * 1e3
    gflops = 2.0 * P_all * steps / elapsed / 1e9

    # ---- the other algorithms on the same inputs (config 2; after the timed region)
    other = {}
    if world == 1 and cfg_name == "2":
        for a2 in (1, 2, 3):
            if a2 == alg:
                continue
            for _ in range(3):
                cusparse.spgemm(A, B, alg=a2, chunk_fraction=cf)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reps_o = max(5, steps // 2)
            for _ in range(reps_o):
                cusparse.spgemm(A, B, alg=a2, chunk_fraction=cf)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps_o
            other[f"alg{a2}"] = {"gflops": round(2.0 * P / dt / 1e9, 3), "ms_per_step": round(dt * 1e3, 5),
                                 "peak_hbm_bytes": int(cusparse.last_stats.peak_bytes)}

    # ---- per-phase device times (separate, instrumented pass after the timed region): HIP
    # events on the library's stream, which is torch's current stream
    h = _lib.get_handle(local_dev)
    h.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    h.set_timing(True)
    reps = 10 if cfg_name == "2" else 2
    for _ in range(reps):
        C = step()
        del C
    phases = h.get_timing()
    h.set_timing(False)
    tile = cfg_name != "2"
    num_kernel = "k_tile" if tile else "k_row"
    num_ms, num_launches = phases["numeric"]
    launches_per_product = max(1, num_launches // reps)
    avg_num_ms = num_ms / max(num_launches, 1)
    # this rank's product (its slab at N>1): algorithmic bytes, split over the numeric launches
    bytes_product = compulsory_bytes(A.shape[0], n, A.nnz, nnzB, nnzC, vb, ib_c)
    bytes_launch = bytes_product / launches_per_product
    achieved = bytes_launch / (avg_num_ms * 1e-3) / 1e9
    key = f"c{cfg_name}_n{n}_d{dens:g}_{args.dtype}_alg{alg}_w{world}"
    traffic, traffic_build = traffic_for(args.pmc, key, _lib.build_id(), _lib.source_id())

    # ---- CPU baseline (rank 0 at N=1): scipy A@B, the reference's comparator
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        if A_h is None:   # configs 4/5: a bounded row sample of the same A, all of B
            A_h, B_h = A.get(), B.get()
            sample = np.sort(np.random.default_rng(0).choice(n, size=min(n, 1024), replace=False))
        else:
            sample = None
        cpu = cpu_baseline(A_h, B_h, sample, args.cpu_seconds)

    if rank == 0:
        step_desc = {"2": "ALG1 single-pass numeric", "4": f"ALG{alg} chunked, chunk_fraction {cf}",
                     "5": f"ALG{alg}"}[cfg_name]
        line = {
            "metric": METRIC, "value": round(gflops, 3), "unit": "GFLOPS", "n_gpus": world,
            "steps": steps, "warmup": warmup, "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True, "scaling": "strong" if cfg_name == "5" else "weak",
            "vs_baseline": None, "dtype": "f64" if vb == 8 else "f32", "data": "synthetic",
            "config": {
                "workload": (f"{cfg['name']}: random CSR {n}x{n} density={dens:g} {args.dtype} "
                             + ("(scipy.sparse.random, default_rng(42); A then B), " if cfg["gen"] == "scipy"
                                else f"(spmm_amd.gen.random_csr on the device, seeds {args.seed}/{args.seed + 1}), ")
                             + step_desc
                             + ("" if world == 1 else
                                f"; {world} row blocks cut on the product prefix, B broadcast over RCCL inside every step")),
                "N": n, "density": dens, "alg": alg, "nnzB": int(nnzB),
                ("nnzA" if world == 1 else "nnzA_rank0"): int(A.nnz),
                "nnzC": int(nnz_all), "num_products": int(P_all),
                "parallelism": "single GPU" if world == 1 else f"row-block x{world}, B broadcast over RCCL",
            },
            "peak_hbm_bytes": int(peak_max),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_build_id": traffic_build,
                         "kernel": num_kernel + " (numeric phase)",
                         "bytes_per_launch": int(bytes_launch), "launches_per_product": launches_per_product,
                         "avg_launch_ms": round(avg_num_ms, 5),
                         "step_frac": round(bytes_product / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                         if world == 1 else None},
            "phases_ms_per_step": {k: round(v[0] / reps, 5) for k, v in phases.items() if v[1]},
            "b_broadcast_ms": None if bcast_ms is None else round(bcast_ms, 3),
            "rows_rank0": list(rows),
            "cpu_baseline": cpu,
            "other_algs": other or None,
            "lib_build_id": _lib.build_id(),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
