#!/usr/bin/env python3
"""ALG1 / ALG2 / ALG3 comparison: time and ΔPeak VRAM per algorithm.

Port of SpGEMM_alg_comparison/profiler.py (:210-287) over spmm_amd.cusparse.spgemm.  Same CLI
(--size/--density lists, --dtype, --runs, --seed, --threads, --no-warmup) and the same
table.  As in the reference, each timed run includes building the device CSR operands
from the host scipy matrices (H2D) -- SpGEMM(...) at profiler.py:210-213.  Deliberate fix:
B is drawn with seed+1 (the reference draws A and B with the same seed, profiler.py:
176-177, so A == B).  Extra columns: GFLOPS (2P/t) and the library's exact peak bytes
(workspace + C) next to the sampled ΔPeak.
"""
import argparse
import itertools
import os
import sys

import numpy as np
import scipy.sparse as sp_cpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from spmm_amd import cusparse  # noqa: E402
from spmm_amd.profiling import human_bytes, repeat_gpu  # noqa: E402
from spmm_amd.sparse import csr_matrix  # noqa: E402

try:
    from threadpoolctl import threadpool_limits
except Exception:   # noqa: BLE001
    threadpool_limits = None


def make_sparse_matrix(m, n, density, dtype=np.float32, seed=0):
    rng = np.random.default_rng(seed)
    M = sp_cpu.random(m, n, density=density, format="csr", dtype=dtype, random_state=rng,
                      data_rvs=rng.standard_normal)
    M.eliminate_zeros()
    M.sort_indices()
    return M


def run_all(m, n, p, densityA, densityB, dtype, dtype_str, runs, seed, do_warmup=True):
    import torch
    A = make_sparse_matrix(m, n, densityA, dtype=dtype, seed=seed)
    B = make_sparse_matrix(n, p, densityB, dtype=dtype, seed=seed + 1)
    dA, dB = csr_matrix(A, device="cuda"), csr_matrix(B, device="cuda")
    P = cusparse.num_products(dA, dB)
    del dA, dB
    print("\n\n", "*" * 91)
    print("\n\n=== Config (GPU/spmm_amd) ===")
    print(f"GPU Name     : {torch.cuda.get_device_name()}")
    print(f"A shape      : ({m}, {n}) CSR density={densityA}")
    print(f"B shape      : ({n}, {p}) CSR density={densityB}")
    print(f"dtype        : {dtype_str}")
    print(f"runs         : {runs}")
    print(f"products     : {P}")

    def SpGEMM(alg):
        a = csr_matrix(A, device="cuda")
        b = csr_matrix(B, device="cuda")
        return cusparse.spgemm(a, b, alg=alg)

    results = []
    for alg in [1, 2, 3]:
        name = f"A_csr @ B_csr (alg={alg})"
        results.append(repeat_gpu(name, lambda alg=alg: SpGEMM(alg), runs, do_warmup))

    print("\n=== Results (alg comparison) ===")
    header = (f"{'name':40}  {'time(ms)':>10}  {'ΔPeak VRAM':>12}  {'lib peak':>12}  "
              f"{'GFLOPS':>9}  {'out_shape':>16}  {'dtype':>10}")
    print(header)
    print("-" * len(header))
    for r in results:
        if r is None:
            print(f"{'SKIPPED (OOM)':40}")
            continue
        gf = 2.0 * P / (r.time_ms * 1e-3) / 1e9
        print(f"{r.name:40}  {r.time_ms:10.6f}  {human_bytes(r.peak_vram):>12}  "
              f"{human_bytes(r.lib_peak_bytes):>12}  {gf:9.3f}  {str(r.out_shape):>16}  "
              f"{str(r.out_dtype):>10}")


def main():
    ap = argparse.ArgumentParser(description="spmm_amd SpGEMM ALG1/2/3 benchmark (A,B)")
    ap.add_argument("--size", type=int, nargs="+", default=[1024])
    ap.add_argument("--density", type=float, nargs="+", default=[1e-1])
    ap.add_argument("--dtype", type=str, default="float32", choices=["float32", "float64"])
    ap.add_argument("--runs", type=int, default=1)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--no-warmup", action="store_true")
    args = ap.parse_args()
    dtype = {"float32": np.float32, "float64": np.float64}[args.dtype]
    ctx = threadpool_limits(limits=args.threads) if args.threads > 0 and threadpool_limits else None
    for size, density in itertools.product(args.size, args.density):
        kw = dict(m=size, n=size, p=size, densityA=density, densityB=density, dtype=dtype,
                  dtype_str=args.dtype, runs=args.runs, seed=args.seed, do_warmup=not args.no_warmup)
        if ctx is None:
            run_all(**kw)
        else:
            with ctx:
                run_all(**kw)


if __name__ == "__main__":
    main()
