"""Sparse-vs-dense break-even case (port of dense_vs_sparseGEMM/utils.py:226-329).

Inputs are placed on the device before timing ("inputs_on_gpu", utils.py:243-250): the
sparse path times ``A_sparse @ B_sparse`` through spmm_amd (CSR @ CSR -> sum_duplicates ->
spgemm), the dense path times ``A_dense @ B_dense`` through torch (rocBLAS / hipBLASLt GEMM,
the reference's cuBLAS comparator).  Out-of-memory in either path prints [SKIP] and the
row reads SKIPPED (OOM) (utils.py:156-173).
"""
from __future__ import annotations

import os
import sys
from typing import Optional

import numpy as np
import scipy.sparse as sp_cpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from spmm_amd.profiling import BenchResult, human_bytes, repeat_gpu  # noqa: E402,F401
from spmm_amd.sparse import csr_matrix  # noqa: E402


def make_sparse_matrix(m, n, density, dtype, rng):
    M = sp_cpu.random(m, n, density=density, format="csr", dtype=dtype, random_state=rng)
    M.sort_indices()
    return M


def run_spmm_case(m, n, p, density, dtype, dtype_str, runs, seed, do_warmup=True) -> None:
    import torch
    rng = np.random.default_rng(seed)
    A = make_sparse_matrix(m, n, density, dtype, rng)
    B = make_sparse_matrix(n, p, density, dtype, rng)
    A_sparse = csr_matrix(A, device="cuda")
    B_sparse = csr_matrix(B, device="cuda")
    A_dense = torch.from_numpy(A.toarray()).cuda()
    B_dense = torch.from_numpy(B.toarray()).cuda()

    print("\n" + "*" * 80)
    print("=== spmm_amd SpGEMM (CSR @ CSR) vs dense GEMM: A @ B ===")
    print(f"A / B shape (CSR) : A=({m}, {n}), B=({n}, {p}), target_density={density}")
    print(f"actual_density    : {A.nnz / (m * n):.6f}")
    print(f"dtype             : {dtype_str}")
    print(f"runs              : {runs}\n")

    op = "A @ B"
    rs = repeat_gpu(op + " [sparse, inputs_on_gpu]", lambda: A_sparse @ B_sparse, runs, do_warmup)
    rd = repeat_gpu(op + " [dense, inputs_on_gpu]", lambda: A_dense @ B_dense, runs, do_warmup)

    header = f"{'name':40}  {'time(ms)':>10}  {'ΔPeak Mem':>16}  {'out_shape':>16}  {'dtype':>10}  {'lib peak':>12}"
    print(header)
    print("-" * len(header))

    def show(r: Optional[BenchResult]):
        if r is None:
            print(f"{'SKIPPED (OOM)':40}  {'-':>10}  {'-':>16}  {'-':>16}  {'-':>10}  {'-':>12}")
            return
        print(f"{r.name:40}  {r.time_ms:10.6f}  {human_bytes(r.peak_vram):>16}  "
              f"{str(tuple(r.out_shape)):>16}  {str(r.out_dtype):>10}  {human_bytes(r.lib_peak_bytes):>12}")

    show(rs)
    show(rd)
