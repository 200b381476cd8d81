"""Small fp32 products of the reference's grid (N = 1024): plan and per-call time of A @ B at
densities 0.001 / 0.01 / 0.05 / 0.1 (the grid showed 0.01 slower than 0.05)."""
import sys
import time

import numpy as np
import scipy.sparse as sp
import torch

sys.path.insert(0, ".")
from spmm_amd import cusparse  # noqa: E402
from spmm_amd.sparse import csr_matrix  # noqa: E402

for d in (0.001, 0.01, 0.05, 0.1):
    rng = np.random.default_rng(42)
    A = sp.random(1024, 1024, density=d, format="csr", random_state=rng, dtype=np.float32)
    B = sp.random(1024, 1024, density=d, format="csr", random_state=rng, dtype=np.float32)
    dA, dB = csr_matrix(A, device="cuda:0"), csr_matrix(B, device="cuda:0")
    for _ in range(5):
        C = dA @ dB
    torch.cuda.synchronize()
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        C = dA @ dB
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(d, cusparse.plan_info(dA, dB, alg=0), f"{np.median(ts) * 1e3:.3f} ms", C.nnz, flush=True)
