"""Per-rank multiply hook for bench.py's CPU rehearsal (`--device cpu --multiply-hook
tests.bench_hooks:oracle_multiply`): the CPU oracle stands in for the device multiply so the
launcher, the row blocks, the B broadcast and the timing/reduction logic of bench.py run on
gloo without a GPU.  Test infrastructure only: bench.py never imports the oracle itself."""
import os

import numpy as np
import torch

from oracle import oracle
from spmm_amd.sparse import csr_matrix


def oracle_multiply(A_block, B, wait_values):
    wait_values()
    p, j, x = oracle.spgemm(A_block.get(), B.get(), keep_zeros=True, sort=True)
    ip = torch.from_numpy(p.astype(np.int64))
    C = csr_matrix._from_parts(torch.from_numpy(x), torch.from_numpy(j.astype(np.int32)), ip,
                               (A_block.shape[0], B.shape[1]), canonical=True)
    out = os.environ.get("SPG_BENCH_HOOK_DUMP")
    if out:   # each rank's slab, for the test to compare with the oracle on the global A
        np.savez(f"{out}.n{B.shape[1]}.rank{os.environ.get('RANK', '0')}.npz", p=p, j=j, x=x)
    return C
