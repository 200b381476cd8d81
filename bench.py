#!/usr/bin/env python3
"""CSR x CSR SpGEMM benchmark on MI355X (BASELINE.json metric: GFLOPS + peak HBM bytes).

Step = one complete ``C = A.B`` through the drop-in shim (``spmm_amd.cusparse.spgemm``:
plan, symbolic with its nnz(C) host sync, C allocation, numeric), inputs resident in HBM.

* N=1: BASELINE config 2 -- random 16384 x 16384, density 1e-3, fp64, A then B from one
  ``default_rng(42)`` stream via scipy.sparse.random (nnz(C) = 4,366,124, P = 4,402,284),
  ALG1-style single pass (``--alg``).
* N>1 (torchrun, one process per GPU, RCCL): weak scaling -- rank r owns a 16384-row block
  of A (rank 0's block is config 2's A, rank r>0 draws its own with seed 42+r), B is built
  on rank 0 and broadcast over RCCL/xGMI once (timed and reported separately, not inside
  the step), every rank computes its C slab; no collective inside the step.
  value = sum over ranks of 2*P_r per step / max-over-ranks step time.

Also reported: ``roofline`` for the numeric-phase kernel (k_row here; algorithmic bytes per
launch / its average device time from HIP events on the library's stream, SURVEY 8d
compulsory-bytes model) and ``cpu_baseline`` (the oracle's C restatement of scipy's
csr_matmat, single thread, on the same A and B, rank 0 at N=1), plus scipy itself.
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--density", type=float, default=1e-3)
    ap.add_argument("--alg", type=int, default=1)
    ap.add_argument("--chunk-fraction", type=float, default=0.2)
    ap.add_argument("--dtype", default="float64", choices=["float32", "float64"])
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="budget of the CPU-baseline sample (0 disables it)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="PMC traffic summary written by profiles/collect_pmc.py")
    return ap.parse_args()


def compulsory_bytes(n_rows, n_cols, nnzA, nnzB, nnzC, vb, ib=4):
    """SURVEY 8d compulsory bytes: three row pointers, A and B read once, C written once."""
    return ib * (n_rows + 1) * 2 + ib * (n_cols + 1) + (4 + vb) * (nnzA + nnzB + nnzC)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from spmm_amd import _lib, cusparse, distributed, gen
    from spmm_amd.sparse import csr_matrix

    npdt = np.float64 if args.dtype == "float64" else np.float32
    vb = 8 if npdt == np.float64 else 4
    n, dens = args.n, args.density

    # ---- inputs (host -> HBM once; not timed)
    if rank == 0:
        A_h, B_h = gen.scipy_pair(n, dens, seed=args.seed, dtype=npdt)
    else:
        A_h = gen.scipy_random(n, n, dens, np.random.default_rng(args.seed + rank), npdt)
        B_h = None
    A = csr_matrix(A_h, device=dev)
    bcast_ms = None
    if world > 1:
        B0 = csr_matrix(B_h, device=dev) if rank == 0 else None
        torch.cuda.synchronize(); dist.barrier()
        t0 = time.perf_counter()
        B = distributed.broadcast_csr(B0, 0, dev)
        torch.cuda.synchronize(); dist.barrier()
        bcast_ms = (time.perf_counter() - t0) * 1e3
    else:
        B = csr_matrix(B_h, device=dev)

    P = cusparse.num_products(A, B)

    def step():
        return cusparse.spgemm(A, B, alg=args.alg, chunk_fraction=args.chunk_fraction)

    # ---- warmup, then exactly K timed steps between barrier + synchronize
    C = None
    for _ in range(args.warmup):
        C = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        C = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    nnzC = C.nnz
    peak_bytes = cusparse.last_stats.peak_bytes

    tot = torch.tensor([elapsed, float(P), float(nnzC), float(peak_bytes)], dtype=torch.float64, device=dev)
    if world > 1:
        mx = tot[:1].clone(); dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tot[1:3].clone(); dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        pk = tot[3:].clone(); dist.all_reduce(pk, op=dist.ReduceOp.MAX)
        elapsed, P_all, nnz_all, peak_max = float(mx[0]), float(sm[0]), float(sm[1]), float(pk[0])
    else:
        P_all, nnz_all, peak_max = float(P), float(nnzC), float(peak_bytes)
    ms_per_step = elapsed / args.steps * 1e3
    gflops = 2.0 * P_all * args.steps / elapsed / 1e9

    # ---- the other algorithms on the same inputs (after the timed region; reported beside)
    other = {}
    if world == 1:
        for alg in (1, 2, 3):
            if alg == args.alg:
                continue
            for _ in range(3):
                cusparse.spgemm(A, B, alg=alg, chunk_fraction=args.chunk_fraction)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reps_o = max(5, args.steps // 2)
            for _ in range(reps_o):
                cusparse.spgemm(A, B, alg=alg, chunk_fraction=args.chunk_fraction)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps_o
            other[f"alg{alg}"] = {"gflops": round(2.0 * P / dt / 1e9, 3), "ms_per_step": round(dt * 1e3, 5),
                                  "peak_hbm_bytes": int(cusparse.last_stats.peak_bytes)}

    # ---- per-kernel device times (separate, instrumented pass after the timed region)
    h = _lib.get_handle(local)
    h.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    h.set_timing(True)
    reps = 10
    for _ in range(reps):
        step()
    phases = h.get_timing()
    h.set_timing(False)
    dom = max(phases.items(), key=lambda kv: kv[1][0])
    avgA, avgB = A.nnz / max(A.shape[0], 1), B.nnz / max(B.shape[0], 1)
    # which kernel the numeric phase launches (the library's own dispatch rule, want_short)
    num_kernel = ("k_row" if B.shape[1] <= 16384 and avgA <= 48 and avgA * avgB <= 400
                  else "k_tile / k_numeric")
    dom_name, (dom_ms, dom_launches) = dom
    num_ms, num_launches = phases["numeric"]
    avg_num_ms = num_ms / max(num_launches, 1)
    bytes_launch = compulsory_bytes(A.shape[0], B.shape[1], A.nnz, B.nnz, nnzC, vb)
    achieved = bytes_launch / (avg_num_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.pmc):
        try:
            with open(args.pmc) as f:
                pm = json.load(f)
            key = f"n{n}_d{dens:g}_{args.dtype}_alg{args.alg}"
            traffic = pm.get(key, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    # ---- CPU baseline (rank 0 at N=1): oracle port, single thread, same A and B
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        from oracle import oracle
        oracle.build()
        times = []
        t_start = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            oracle.spgemm(A_h, B_h, keep_zeros=True, sort=True)
            times.append(time.perf_counter() - t0)
            if time.perf_counter() - t_start > args.cpu_seconds or len(times) >= 200:
                break
        t_port = float(np.median(times))
        st = []
        for _ in range(min(5, max(1, len(times)))):
            t0 = time.perf_counter()
            _ = A_h @ B_h
            st.append(time.perf_counter() - t0)
        t_scipy = float(np.median(st))
        # multi-core point: the same restatement with OpenMP over rows on the host cores
        # (OMP_NUM_THREADS when set -- 16 on the GPU box -- else every visible core)
        nthr = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        om = []
        t_start = time.perf_counter()
        while len(om) < 20 and (len(om) < 3 or time.perf_counter() - t_start < args.cpu_seconds / 2):
            t0 = time.perf_counter()
            oracle.spgemm(A_h, B_h, keep_zeros=True, sort=True, threads=nthr)
            om.append(time.perf_counter() - t0)
        t_omp = float(np.median(om))
        cpu = {"value": round(2.0 * P / t_port / 1e9, 4), "unit": "GFLOPS", "cores": 1,
               "kind": "port",
               "sample": f"full config product (same A,B), median of {len(times)} runs, "
                         f"{t_port * 1e3:.1f} ms/run, oracle/gustavson.c single thread",
               "ms_per_step": round(t_port * 1e3, 3),
               "scipy_ms": round(t_scipy * 1e3, 3),
               "scipy_gflops": round(2.0 * P / t_scipy / 1e9, 4),
               "omp": {"threads": nthr, "ms_per_step": round(t_omp * 1e3, 3),
                       "gflops": round(2.0 * P / t_omp / 1e9, 4),
                       "sample": f"oracle/gustavson.c OpenMP over rows, median of {len(om)} runs"},
               "host_cpus": os.cpu_count()}

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(gflops, 3), "unit": "GFLOPS", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64" if vb == 8 else "f32", "data": "synthetic",
            "config": {
                "workload": (f"random CSR {n}x{n} density={dens:g} {args.dtype} "
                             f"(scipy.sparse.random, default_rng({args.seed}); A then B), "
                             f"ALG{args.alg}" + (" single-pass numeric" if args.alg == 1 else "")
                             + ("" if world == 1 else f"; {world} row blocks of {n} rows, B broadcast")),
                "N": n, "density": dens, "alg": args.alg, "nnzA": A.nnz, "nnzB": B.nnz,
                "nnzC": int(nnz_all), "num_products": int(P_all),
                "parallelism": "single GPU" if world == 1 else f"row-block x{world}, B broadcast over RCCL",
            },
            "peak_hbm_bytes": int(peak_max),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "kernel": num_kernel + " (numeric phase, one launch)",
                         "bytes_per_launch": int(bytes_launch),
                         "avg_launch_ms": round(avg_num_ms, 5)},
            "phases_ms_per_step": {k: round(v[0] / reps, 5) for k, v in phases.items() if v[1]},
            "dominant_phase": dom_name,
            "b_broadcast_ms": None if bcast_ms is None else round(bcast_ms, 3),
            "cpu_baseline": cpu,
            "other_algs": other or None,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
