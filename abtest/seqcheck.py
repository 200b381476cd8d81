"""Bit-identity of an A/B library against the shipped one on a dense-tile product (run once
per library: SPG_LIB=... python abtest/seqcheck.py; prints the plan and a digest of C)."""
import hashlib
import sys

import numpy as np
import scipy.sparse as sp
import torch

sys.path.insert(0, ".")
from spmm_amd import cusparse  # noqa: E402
from spmm_amd.sparse import csr_matrix  # noqa: E402

rng = np.random.default_rng(7)
for n, d in ((20000, 0.01), (40000, 0.004)):
    A = sp.random(n, n, density=d, format="csr", random_state=rng)
    B = sp.random(n, n, density=d, format="csr", random_state=rng)
    dA, dB = csr_matrix(A, device="cuda:0"), csr_matrix(B, device="cuda:0")
    C = cusparse.spgemm(dA, dB, alg=2)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in (C.indptr, C.indices, C.data):
        h.update(t.cpu().numpy().tobytes())
    print(n, d, cusparse.plan_info(dA, dB, alg=2), h.hexdigest()[:16])
