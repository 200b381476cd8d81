#!/usr/bin/env python3
"""Port of dense_vs_sparseGEMM/main.py (:17-112): CLI --size/--density lists (required),
--dtype, --runs (3), --seed (42), --threads, --no-warmup."""
import argparse
import itertools
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from utils import run_spmm_case  # noqa: E402

try:
    from threadpoolctl import threadpool_limits
except Exception:   # noqa: BLE001
    threadpool_limits = None


def main() -> None:
    ap = argparse.ArgumentParser(description="spmm_amd SpGEMM (CSR @ CSR) vs dense GEMM benchmark")
    ap.add_argument("--size", type=int, nargs="+", required=True)
    ap.add_argument("--density", type=float, nargs="+", required=True)
    ap.add_argument("--dtype", type=str, default="float32", choices=["float32", "float64"])
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--no-warmup", action="store_true")
    args = ap.parse_args()
    dtype = {"float32": np.float32, "float64": np.float64}[args.dtype]
    ctx = threadpool_limits(limits=args.threads) if args.threads > 0 and threadpool_limits else None
    for size, density in itertools.product(args.size, args.density):
        kw = dict(m=size, n=size, p=size, density=density, dtype=dtype, dtype_str=args.dtype,
                  runs=args.runs, seed=args.seed, do_warmup=not args.no_warmup)
        if ctx is None:
            run_spmm_case(**kw)
        else:
            with ctx:
                run_spmm_case(**kw)


if __name__ == "__main__":
    main()
