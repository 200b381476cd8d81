"""The run-time guard of the ordered-LDS property.

fp64 / complex128 tile kernels (k_tile_dn, k_tile_sp) get scipy's summation order from two
properties of gfx950's LDS: the lanes of one ds_add_f64 that hit the same address apply in
ascending lane order, and a wave's DS instructions apply in issue order (spgemm_tile_dn.hpp).
spg_create checks both on the device (k_lds_order_check: 64 trials of two 64-lane
instructions into 4 slots, replayed on the host bit for bit); a failed check sends fp64 tiles
to k_tile's owner rounds, which rely on neither.  SPG_LDS_ORDERED=0 forces that fallback
(read when a handle is created), so these tests run the fallback in a fresh process on the
shapes of the lean kernels -- config 3 (N=8192, density 1e-2, dense tiles), the 2048-column
dense shape (config 4's) and the 8192-column sparse shape (config 5's) -- and check every
result bit for bit against the oracle.  The same fresh-process runner also takes a tile-path
product through SPG_LB_SPIN_TICKS=0 (every bounded look-back wait of an out-of-place scan on
its direct path; in-place scans never take it).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bits(x):
    return x.view(np.uint32 if x.dtype == np.float32 else np.uint64)


def _cases():
    """(name, A, B, alpha) on the lean kernels' shapes (fixed seeds, scipy inputs)."""
    from spmm_amd import gen
    out = []
    A, B = gen.scipy_pair(8192, 1e-2, seed=42)
    out.append(("config3_d1e-2", A, B, 1.0))
    rng = np.random.default_rng(33)
    A = sp.random(257, 17000, density=0.01, format="csr", random_state=rng, dtype=np.float64)
    B = sp.random(17000, 17000, density=0.01, format="csr", random_state=rng, dtype=np.float64)
    out.append(("dense2048_shape", A, B, 1.0))
    rng = np.random.default_rng(34)
    A = sp.random(300, 40000, density=0.0075, format="csr", random_state=rng)
    B = sp.random(40000, 40000, density=0.00075, format="csr", random_state=rng)
    out.append(("sparse8192_shape", A, B, 0.5))
    for _, X, Y, _ in out:
        for M in (X, Y):
            M.sum_duplicates()
            M.sort_indices()
    return out


def _run_fresh(env, tmp_path, algs=(2, 3)):
    """Every case under every alg in a fresh process with `env`; returns {(name, alg): (p, j, x)}
    and the plan infos."""
    code = f"""
import json, sys, numpy as np, torch
sys.path.insert(0, {ROOT!r})
from tests.test_gpu_lds_guard import _cases
from spmm_amd import cusparse
from spmm_amd.sparse import csr_matrix
infos = {{}}
arrs = {{}}
for name, A, B, alpha in _cases():
    dA, dB = csr_matrix(A, device="cuda:0"), csr_matrix(B, device="cuda:0")
    infos[name] = cusparse.plan_info(dA, dB, alg=2)
    for alg in {list(algs)!r}:
        C = cusparse.spgemm(dA, dB, alpha=alpha, alg=alg, chunk_fraction=0.05)
        torch.cuda.synchronize()
        arrs[f"{{name}}|{{alg}}|p"] = C.indptr.cpu().numpy().astype(np.int64)
        arrs[f"{{name}}|{{alg}}|j"] = C.indices.cpu().numpy()
        arrs[f"{{name}}|{{alg}}|x"] = C.data.cpu().numpy()
np.savez({str(tmp_path / "out.npz")!r}, **arrs)
json.dump(infos, open({str(tmp_path / "info.json")!r}, "w"))
"""
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    got = np.load(tmp_path / "out.npz")
    return got, json.load(open(tmp_path / "info.json"))


def _check_all(got, algs=(2, 3)):
    for name, A, B, alpha in _cases():
        rp, rj, rx = oracle.spgemm(A, B, alpha=alpha, keep_zeros=True, sort=True, threads=16)
        for alg in algs:
            key = f"{name}|{alg}"
            assert np.array_equal(got[key + "|p"], rp), f"{key}: row pointer"
            assert np.array_equal(got[key + "|j"], rj), f"{key}: columns"
            assert np.array_equal(_bits(got[key + "|x"]), _bits(rx)), f"{key}: values"


def test_device_check_finds_ordered_lds():
    """On MI355X the check passes: fp64 tile plans run the ordered-LDS kernels, and the shapes
    keep their lean geometries (2048-column dense tiles, 8192-column sparse tiles)."""
    from spmm_amd import cusparse
    from spmm_amd.sparse import csr_matrix
    cases = {name: (A, B) for name, A, B, _ in _cases()}
    widths = {"dense2048_shape": (2048, True), "sparse8192_shape": (8192, False)}
    for name, (A, B) in cases.items():
        info = cusparse.plan_info(csr_matrix(A, device="cuda:0"), csr_matrix(B, device="cuda:0"), alg=2)
        assert info["path"] == "tile" and info["lds_ordered"], (name, info)
        if name in widths:
            assert (info["tile_width"], info["dense_tiles"]) == widths[name], (name, info)


def test_owner_round_fallback_bitexact(tmp_path):
    """SPG_LDS_ORDERED=0: every lean shape on k_tile's owner rounds (plan_info says so, and the
    geometry falls back to <= 4096-column tiles), bit-exact against the oracle under ALG2 and
    chunked ALG3."""
    got, infos = _run_fresh({"SPG_LDS_ORDERED": "0"}, tmp_path)
    for name, info in infos.items():
        assert info["path"] == "tile" and not info["lds_ordered"], (name, info)
        assert info["tile_width"] <= 4096, (name, info)
    _check_all(got)


def test_tile_path_with_every_scan_wait_direct(tmp_path):
    """SPG_LB_SPIN_TICKS=0 on the tile path: the segment-table and item scans run in place and
    must keep waiting (their inputs are overwritten by earlier tiles); results bit-exact."""
    got, _ = _run_fresh({"SPG_LB_SPIN_TICKS": "0"}, tmp_path, algs=(2,))
    _check_all(got, algs=(2,))
