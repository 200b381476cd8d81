#!/usr/bin/env python3
"""Host-side cost of one ``cusparse.spgemm`` call, step by step (GPU box).

Times the shim's stages with perf_counter around each (the device work of the same call is
reported by profiles/phases.py), for ALG1 and ALG2 on BASELINE config 2:

    python profiles/host_overhead.py [--alg 1] [--reps 200]
"""
from __future__ import annotations

import argparse
import ctypes
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
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    import torch
    from spmm_amd import _lib, cusparse, gen
    from spmm_amd.sparse import csr_matrix
    dev = torch.device("cuda", 0)
    A_h, B_h = gen.scipy_pair(args.n, args.density, seed=42)
    A, B = csr_matrix(A_h, device=dev), csr_matrix(B_h, device=dev)
    h = cusparse._handle_for(A)
    lib = h.lib
    out = {}
    for alg in (1, 2):
        stages = {}

        def tick(name, t0):
            t1 = time.perf_counter()
            stages[name] = stages.get(name, 0.0) + (t1 - t0)
            return t1

        for rep in range(args.reps + 10):
            if rep == 10:
                stages.clear()
            t = time.perf_counter()
            a, b = cusparse._cast_common_type(A, B)
            va, vb = cusparse._csr_view(a), cusparse._csr_view(b)
            t = tick("checks+views", t)
            ws_bytes = ctypes.c_size_t(0)
            lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), alg, 0.2, ctypes.byref(ws_bytes), None, None)
            t = tick("plan(size)", t)
            ws = torch.empty(max(ws_bytes.value, 1), dtype=torch.uint8, device=dev)
            t = tick("alloc ws", t)
            plan = ctypes.c_void_p()
            lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), alg, 0.2, ctypes.byref(ws_bytes),
                         ctypes.c_void_p(ws.data_ptr()), ctypes.byref(plan))
            t = tick("plan(build)", t)
            indptr = torch.empty(A.shape[0] + 1, dtype=torch.int32, device=dev)
            t = tick("alloc indptr", t)
            nnz = ctypes.c_int64(0)
            lib.spg_symbolic(h.ptr, plan, ctypes.c_void_p(indptr.data_ptr()), _lib.SPG_INDEX_32I, ctypes.byref(nnz))
            t = tick("symbolic(+sync)", t)
            n = int(nnz.value)
            pj, px = ctypes.c_void_p(), ctypes.c_void_p()
            lib.spg_result_in_workspace(plan, ctypes.byref(pj), ctypes.byref(px))
            if pj.value:
                base = ws.data_ptr()
                indices = ws[pj.value - base:pj.value - base + 4 * n].view(torch.int32)
                data = ws[px.value - base:px.value - base + 8 * n].view(torch.float64)
            else:
                indices = torch.empty(n, dtype=torch.int32, device=dev)
                data = torch.empty(n, dtype=torch.float64, device=dev)
            t = tick("C arrays", t)
            c = csr_matrix._from_parts(data, indices, indptr, (A.shape[0], B.shape[1]), canonical=True)
            vc = _lib.SpgCsr(A.shape[0], B.shape[1], n, indptr.data_ptr(), indices.data_ptr(), data.data_ptr(),
                             _lib.SPG_INDEX_32I, _lib.SPG_R_64F)
            al = ctypes.c_double(1.0)
            t = tick("C object", t)
            lib.spg_numeric(h.ptr, plan, ctypes.byref(al), ctypes.byref(vc))
            t = tick("numeric", t)
            ws.record_stream(torch.cuda.current_stream(dev))
            lib.spg_plan_destroy(plan)
            t = tick("finish", t)
        torch.cuda.synchronize()
        tot = sum(stages.values())
        out[f"alg{alg}"] = {"us_per_call": round(tot / args.reps * 1e6, 2),
                            "stages_us": {k: round(v / args.reps * 1e6, 2) for k, v in stages.items()}}
        # the shim itself, for comparison
        for _ in range(10):
            cusparse.spgemm(A, B, alg=alg)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            cusparse.spgemm(A, B, alg=alg)
        torch.cuda.synchronize()
        out[f"alg{alg}"]["shim_us_per_call"] = round((time.perf_counter() - t0) / args.reps * 1e6, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
