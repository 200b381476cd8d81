#!/usr/bin/env python3
"""Run the BASELINE.json configurations on one GPU and print one JSON line each:
GFLOPS (2P/t), ms per C = A.B, peak HBM bytes (workspace + C), per-phase device times,
compulsory-bytes GB/s, and (config 3) the rocBLAS dense GEMM comparator.

  config 2: N=16384  density 1e-3          fp64  ALG1
  config 3: N=8192   density 1e-4..1e-1    fp64  ALG2  (+ dense torch.matmul = rocBLAS dgemm)
  config 4: N=65536  density 5e-3          fp64  ALG3, chunk_fraction 0.2
  config 5: N=262144 density 1e-3          fp64  (1-GPU point; the 8-GPU run is
            harness/multi_gpu/spgemm_rowblock.py)
Inputs: scipy_pair (seed 42) up to N=16384, spmm_amd.gen.random_csr beyond.  --check S
compares S sampled rows with the CPU oracle.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)

CONFIGS = {
    "2": [(16384, 1e-3, 1)],
    "3": [(8192, 1e-4, 2), (8192, 1e-3, 2), (8192, 1e-2, 2), (8192, 1e-1, 2)],
    "4": [(65536, 5e-3, 3)],
    "5": [(262144, 1e-3, 2)],
}


def run_case(n, density, alg, steps, check, dense, cf):
    import torch
    from spmm_amd import _lib, cusparse, gen
    from spmm_amd.sparse import csr_matrix
    dev = torch.device("cuda", 0)
    if n <= 16384:
        Ah, Bh = gen.scipy_pair(n, density, seed=42)
        A, B = csr_matrix(Ah, device=dev), csr_matrix(Bh, device=dev)
    else:
        A = gen.random_csr(n, n, density, seed=42, device=dev)
        B = gen.random_csr(n, n, density, seed=43, device=dev)
    P = cusparse.num_products(A, B)
    C = cusparse.spgemm(A, B, alg=alg, chunk_fraction=cf)   # warmup
    nnz = C.nnz
    del C
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        C = cusparse.spgemm(A, B, alg=alg, chunk_fraction=cf)
        if _ < steps - 1:
            del C
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    peak = cusparse.last_stats.peak_bytes
    h = _lib.get_handle(0)
    h.set_stream(torch.cuda.current_stream().cuda_stream)
    del C
    h.set_timing(True)
    C = cusparse.spgemm(A, B, alg=alg, chunk_fraction=cf)
    ph = {k: round(v[0], 4) for k, v in h.get_timing().items() if v[1]}
    h.set_timing(False)
    comp = 4 * (n + 1) * 3 + 12 * (A.nnz + B.nnz + nnz)
    out = {"N": n, "density": density, "alg": alg, "nnzA": A.nnz, "nnzC": nnz, "num_products": P,
           "ms": round(t * 1e3, 4), "gflops": round(2 * P / t / 1e9, 3), "peak_hbm_bytes": peak,
           "compulsory_GBps": round(comp / t / 1e9, 1), "phases_ms": ph}
    if dense:
        Ad = torch.from_numpy(A.get().toarray()).to(dev) if n <= 16384 else None
        if Ad is not None:
            Bd = torch.from_numpy(B.get().toarray()).to(dev)
            Ad @ Bd
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                Ad @ Bd
            torch.cuda.synchronize()
            out["dense_ms"] = round((time.perf_counter() - t0) / 3 * 1e3, 4)
            del Ad, Bd
    if check > 0:
        import scipy.sparse as sp
        from oracle import oracle
        rng = np.random.default_rng(0)
        rows = np.sort(rng.choice(n, size=min(check, n), replace=False))
        Ah = A.get()
        Bh = B.get()
        rp, rj, rx = oracle.spgemm(sp.csr_matrix(Ah[rows]), Bh, keep_zeros=True, sort=True)
        cp = C.indptr.cpu().numpy().astype(np.int64)
        bad = 0
        for q, i in enumerate(rows):
            s, e = cp[i], cp[i + 1]
            if not (np.array_equal(C.indices[s:e].cpu().numpy(), rj[rp[q]:rp[q + 1]]) and
                    np.array_equal(C.data[s:e].cpu().numpy().view(np.uint64), rx[rp[q]:rp[q + 1]].view(np.uint64))):
                bad += 1
        out["checked_rows"] = int(len(rows))
        out["bad_rows"] = bad
    del C
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["2", "3", "4"])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--check", type=int, default=32)
    ap.add_argument("--cf", type=float, default=0.2)
    ap.add_argument("--alg", type=int, default=0, help="override the config's algorithm")
    args = ap.parse_args()
    for c in args.configs:
        for (n, d, alg) in CONFIGS[c]:
            r = run_case(n, d, args.alg or alg, args.steps, args.check, c == "3", args.cf)
            r["config"] = c
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
