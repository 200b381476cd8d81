#!/usr/bin/env python3
"""Per-phase device times (HIP events on the library's stream) and wall time per call for
every algorithm on one configuration -- the breakdown behind DESIGN.md's kernel table.

    python profiles/phases.py [--n 16384] [--density 1e-3] [--reps 20] [--trace out.bin]

--trace sets SPG_LB_TRACE for one extra ALG1 call: per-row wall-clock stamps of the
single-pass kernel (start, count published, value work done, base known), summarised here.
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
    ap.add_argument("--trace", default="")
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
    if args.trace:
        os.environ["SPG_LB_TRACE"] = args.trace
        cusparse.spgemm(A, B, alg=1)
        torch.cuda.synchronize()
        del os.environ["SPG_LB_TRACE"]
    if args.trace and os.path.exists(args.trace):
        t = np.fromfile(args.trace, dtype=np.uint64).reshape(-1, 4).astype(np.int64)
        ok = (t > 0).all(axis=1)
        t = t[ok]
        t0 = t[:, 0].min()
        us = (t - t0) / 100.0   # 100 MHz wall clock
        rows = np.arange(len(us))
        q = lambda a: [round(float(np.percentile(a, x)), 2) for x in (5, 50, 95, 100)]
        out["trace_us"] = {
            "rows": int(ok.sum()),
            "start": q(us[:, 0]), "published": q(us[:, 1]), "values_done": q(us[:, 2]),
            "base_known": q(us[:, 3]),
            "pass1": q(us[:, 1] - us[:, 0]), "value_work": q(us[:, 2] - us[:, 1]),
            "wait_base": q(us[:, 3] - us[:, 2]),
            "start_by_row_decile": [round(float(us[rows[len(rows) * k // 10], 0]), 2) for k in range(10)],
            "end_by_row_decile": [round(float(us[rows[len(rows) * k // 10], 3]), 2) for k in range(10)],
        }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
