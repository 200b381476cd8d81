#!/usr/bin/env python3
"""Generate A, B and C_py = spgemm(A, B, alg=k) as text CSR files.

Port of cupy_cusparse/gen_and_save_alg{1,2,3}_txt.py (:16-44 / :20-58): A and B are random
n x n fp32 CSR matrices (seed, seed + 1), indices sorted; C_py comes from the Python shim
(spmm_amd.cusparse.spgemm) instead of cupyx.cusparse.spgemm.  Tags and file names are the
reference's: {A,B,C_py}_n{N}_dens{d with . -> p}_alg{k}[_cf{cf}]_{indptr,indices,data}.txt.
Inputs come from scipy.sparse.random with numpy RandomState(seed) (CuPy's generator is not
available here); everything downstream only needs the same A and B on both sides.
"""
import argparse
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from spmm_amd import cusparse  # noqa: E402
from spmm_amd.sparse import csr_matrix  # noqa: E402
from spmm_amd.txtio import save_csr_txt  # noqa: E402


def gen_rand_csr(n, d, seed, dtype=np.float32):
    M = sp.random(n, n, density=d, format="csr", dtype=dtype, random_state=np.random.RandomState(seed))
    M.sort_indices()
    return M


def run_once(n, d, outdir, alg, chunk_fraction=0.2, seed=0, include_cf_in_tag=False, dtype=np.float32):
    os.makedirs(outdir, exist_ok=True)
    A = gen_rand_csr(n, d, seed, dtype)
    B = gen_rand_csr(n, d, seed + 1, dtype)
    C = cusparse.spgemm(csr_matrix(A, device="cuda"), csr_matrix(B, device="cuda"), alg=alg,
                        chunk_fraction=chunk_fraction)
    cf_tag = f"_cf{str(chunk_fraction).replace('.', 'p')}" if include_cf_in_tag else ""
    tag = f"n{n}_dens{str(d).replace('.', 'p')}_alg{alg}{cf_tag}"
    save_csr_txt(os.path.join(outdir, f"A_{tag}"), A.indptr, A.indices, A.data)
    save_csr_txt(os.path.join(outdir, f"B_{tag}"), B.indptr, B.indices, B.data)
    save_csr_txt(os.path.join(outdir, f"C_py_{tag}"), C.indptr.cpu().numpy(), C.indices.cpu().numpy(),
                 C.data.cpu().numpy())
    print(f"[PY] saved A/B/C txt to {outdir} ({tag}, chunk_fraction={chunk_fraction})")


def main(alg=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", nargs="+", type=int, default=[32, 64, 128, 256, 512, 1024])
    ap.add_argument("--densities", nargs="+", type=float, default=[0.01, 0.1, 0.3, 0.5])
    ap.add_argument("--outdir", default=None)
    ap.add_argument("--seed", type=int, default=123)
    ap.add_argument("--alg", type=int, default=alg if alg is not None else 1, choices=[1, 2, 3])
    ap.add_argument("--chunk-fraction", type=float, default=0.2,
                    help="ALG3 chunk_fraction in (0,1], default=0.2")
    ap.add_argument("--include-cf-in-tag", action="store_true")
    ap.add_argument("--dtype", default="float32", choices=["float32", "float64"])
    args = ap.parse_args()
    if not (0.0 < args.chunk_fraction <= 1.0):
        raise SystemExit(f"chunk_fraction must be in (0,1], got {args.chunk_fraction}")
    outdir = args.outdir or f"dump_alg{args.alg}_txt"
    dt = np.float32 if args.dtype == "float32" else np.float64
    for n in args.sizes:
        for d in args.densities:
            run_once(n, d, outdir, args.alg, args.chunk_fraction, args.seed, args.include_cf_in_tag, dt)


if __name__ == "__main__":
    main()
