#!/usr/bin/env python3
"""scipy CPU SpGEMM and SpMV vs spmm_amd GPU SpGEMM and SpMV, end to end (port of
SpGEMM_vs_SpMV/profiler.py :380-528; the figure SPGEMM-gpu-speedup.png).

CPU: scipy ``A @ B`` for CSR/CSC/COO operand combinations, each run in a forked child
(time + ΔRSS, profiler.py:116-178), median of --runs.  GPU: the same products with the host
matrices converted and uploaded inside the timed region (H2D included, as the reference
times ``to_gpu_sparse`` + ``@`` together, profiler.py:485-498); CSC/COO operands go through
CSR conversion on the device.  SpMV rows (profiler.py:410-411, 500-501): ``A @ C`` with C a
dense vector of n entries (seed+2), A in each format, on the CPU (scipy) and the GPU
(spmm_amd.cusparse.spmv through ``__matmul__``, x uploaded inside the timed region as the
reference's ``cp.asarray(C)``).  Deliberate fix: B uses seed+1 (the reference reuses the
seed, so A == B, profiler.py:397-398).
"""
import argparse
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from spmm_amd.profiling import human_bytes, repeat_cpu, repeat_gpu  # noqa: E402
from spmm_amd.sparse import coo_matrix, csc_matrix, csr_matrix  # noqa: E402

try:
    from threadpoolctl import threadpool_limits
except Exception:   # noqa: BLE001
    threadpool_limits = None

TO_GPU = {"csr": lambda M: csr_matrix(M, device="cuda"), "csc": lambda M: csc_matrix(M, device="cuda"),
          "coo": lambda M: coo_matrix(M, device="cuda")}


def make(m, n, density, fmt, dtype, seed):
    rng = np.random.default_rng(seed)
    M = sp.random(m, n, density=density, format="csr", dtype=dtype, random_state=rng,
                  data_rvs=rng.standard_normal)
    M.eliminate_zeros()
    M.sort_indices()
    return M.asformat(fmt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1024)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--p", type=int, default=1024)
    ap.add_argument("--densityA", type=float, default=0.1)
    ap.add_argument("--densityB", type=float, default=0.1)
    ap.add_argument("--dtype", default="float32", choices=["float32", "float64"])
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--formats", nargs="+", default=["csr", "csc", "coo"])
    args = ap.parse_args()
    dtype = np.float32 if args.dtype == "float32" else np.float64
    A = {f: make(args.m, args.n, args.densityA, f, dtype, args.seed) for f in args.formats}
    B = {f: make(args.n, args.p, args.densityB, f, dtype, args.seed + 1) for f in args.formats}
    C = np.random.default_rng(args.seed + 2).standard_normal(args.n).astype(dtype)
    ctx = threadpool_limits(limits=args.threads) if threadpool_limits and args.threads > 0 else None

    cpu = []
    if ctx:
        ctx.__enter__()
    for fa in args.formats:
        for fb in args.formats:
            cpu.append(repeat_cpu(f"A_{fa} @ B_{fb} (SpGEMM)", lambda a=A[fa], b=B[fb]: a @ b, args.runs))
    for fa in args.formats:
        cpu.append(repeat_cpu(f"A_{fa} @ C (SpMV, dense vec)", lambda a=A[fa]: a @ C, args.runs))
    if ctx:
        ctx.__exit__(None, None, None)
    print("\n=== Results (CPU/SciPy) ===")
    header = f"{'name':36}  {'time(ms)':>10}  {'ΔPeak RAM':>12}  {'out_shape':>16}  {'dtype':>10}"
    print(header)
    print("-" * len(header))
    for r in cpu:
        print(f"{r.name:36}  {r.time_ms:10.6f}  {human_bytes(r.peak_ram or 0):>12}  "
              f"{str(r.out_shape):>16}  {str(r.out_dtype):>10}")

    import torch
    print("\n\n", "*" * 91)
    print("\n\n=== Config (GPU/spmm_amd) ===")
    print(f"GPU Name     : {torch.cuda.get_device_name()}")
    print(f"A shape      : ({args.m}, {args.n}) density={args.densityA}")
    print(f"B shape      : ({args.n}, {args.p}) density={args.densityB}")
    print(f"dtype        : {args.dtype}")
    print(f"runs         : {args.runs}")
    gpu = []
    for fa in args.formats:
        for fb in args.formats:
            fn = (lambda a=A[fa], b=B[fb], fa=fa, fb=fb: TO_GPU[fa](a) @ TO_GPU[fb](b))
            gpu.append(repeat_gpu(f"A_{fa} @ B_{fb} (SpGEMM)", fn, args.runs))
    for fa in args.formats:
        fn = (lambda a=A[fa], fa=fa: TO_GPU[fa](a) @ torch.from_numpy(C).cuda())
        gpu.append(repeat_gpu(f"A_{fa} @ C (SpMV, dense vec)", fn, args.runs))
    print("\n=== Results ===")
    header = f"{'name':36}  {'time(ms)':>10}  {'ΔPeak VRAM':>12}  {'out_shape':>16}  {'speedup':>8}"
    print(header)
    print("-" * len(header))
    for rc, rg in zip(cpu, gpu):
        if rg is None:
            print(f"{rc.name:36}  SKIPPED (OOM)")
            continue
        print(f"{rg.name:36}  {rg.time_ms:10.6f}  {human_bytes(rg.peak_vram):>12}  "
              f"{str(tuple(rg.out_shape)):>16}  {rc.time_ms / rg.time_ms:8.2f}x")


if __name__ == "__main__":
    main()
