#!/usr/bin/env python3
"""Per-phase device times (HIP events on the library's stream) and wall time per call for
every algorithm on one configuration -- the breakdown behind DESIGN.md's kernel table.

    python profiles/phases.py [--n 16384] [--density 1e-3] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--density", type=float, default=1e-3)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dtype", default="float64")
    args = ap.parse_args()
    import torch
    from spmm_amd import _lib, cusparse, gen
    from spmm_amd.sparse import csr_matrix
    dev = torch.device("cuda", 0)
    npdt = np.float64 if args.dtype == "float64" else np.float32
    A_h, B_h = gen.scipy_pair(args.n, args.density, seed=42, dtype=npdt)
    A, B = csr_matrix(A_h, device=dev), csr_matrix(B_h, device=dev)
    P = cusparse.num_products(A, B)
    h = _lib.get_handle(0)
    h.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    out = {"n": args.n, "density": args.density, "P": P, "short_kernel": os.environ.get("SPG_SHORT_KERNEL", "row")}
    for alg in (1, 2, 3):
        for _ in range(3):
            cusparse.spgemm(A, B, alg=alg)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            cusparse.spgemm(A, B, alg=alg)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.reps * 1e3
        h.set_timing(True)
        for _ in range(args.reps):
            cusparse.spgemm(A, B, alg=alg)
        ph = h.get_timing()
        h.set_timing(False)
        out[f"alg{alg}"] = {"wall_ms": round(wall, 4), "gflops": round(2 * P / wall / 1e6, 2),
                            "phases_ms": {k: round(v[0] / args.reps, 4) for k, v in ph.items() if v[1]},
                            "launches": {k: v[1] // args.reps for k, v in ph.items() if v[1]}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
