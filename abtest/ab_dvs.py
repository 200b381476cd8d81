#!/usr/bin/env python3
"""Per-phase device times of one product per (N, density, dtype) for the library in SPG_LIB
(A/B of tile kernels on the dense_vs_sparseGEMM grid).  One JSON line per case."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from spmm_amd import _lib, cusparse, gen  # noqa: E402
from spmm_amd.sparse import csr_matrix  # noqa: E402

cases = [(int(a), float(b), c) for a, b, c in (x.split(":") for x in sys.argv[1:])]
h = _lib.get_handle(0)
for n, d, dt in cases:
    A, B = gen.scipy_pair(n, d, seed=42, dtype=np.float32 if dt == "f32" else np.float64)
    dA, dB = csr_matrix(A, device="cuda:0"), csr_matrix(B, device="cuda:0")
    for _ in range(2):
        cusparse.spgemm(dA, dB, alg=2)
    torch.cuda.synchronize()
    h.set_stream(torch.cuda.current_stream().cuda_stream)
    h.set_timing(True)
    for _ in range(5):
        cusparse.spgemm(dA, dB, alg=2)
    ph = h.get_timing()
    h.set_timing(False)
    info = cusparse.plan_info(dA, dB, alg=2)
    print(json.dumps({"n": n, "density": d, "dtype": dt, "tw": info["tile_width"], "dense": info["dense_tiles"],
                      "path": info["path"], **{k: round(v[0] / 5, 4) for k, v in ph.items() if v[1]}}), flush=True)
