"""bench.py's host logic (no GPU): the PMC traffic figure is reported only for the library
build -- or a build of the same sources -- it was measured on."""
import json

import bench


def _db(tmp_path, entry):
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"c2_key": entry}))
    return str(p)


def test_traffic_for_matching_build(tmp_path):
    p = _db(tmp_path, {"hbm_bytes_per_launch": 123, "build_id": "b1", "source_id": "s1"})
    assert bench.traffic_for(p, "c2_key", "b1", "other") == (123, "b1")
    # a rebuild of the same sources (hipcc output differs byte for byte)
    assert bench.traffic_for(p, "c2_key", "b2", "s1") == (123, "b1")


def test_traffic_for_stale_or_missing(tmp_path):
    p = _db(tmp_path, {"hbm_bytes_per_launch": 123, "build_id": "b1", "source_id": "s1"})
    assert bench.traffic_for(p, "c2_key", "b2", "s2") == (None, "b1")
    assert bench.traffic_for(p, "other_key", "b1", "s1") == (None, None)
    assert bench.traffic_for(str(tmp_path / "absent.json"), "c2_key", "b1", "s1") == (None, None)


def test_committed_traffic_is_stamped():
    """Every committed entry names the build and sources it was measured on."""
    with open(bench.os.path.join(bench.ROOT, "profiles", "pmc_traffic.json")) as f:
        db = json.load(f)
    for key in ("c2_n16384_d0.001_float64_alg1_w1", "c4_n65536_d0.005_float64_alg3_w1",
                "c5_n262144_d0.001_float64_alg2_w1"):
        assert db[key]["build_id"] and db[key]["source_id"], key
        assert db[key]["hbm_bytes_per_launch"] > 0


import pytest


@pytest.mark.parametrize("world", [2, 4])
def test_bench_spawns_ranks_without_launcher(tmp_path, world):
    """`python3 bench.py --gpus N` with no WORLD_SIZE (the driver's SCALE command), N = 2 and 4:
    the parent starts N worker ranks itself (gloo here, --device cpu, the oracle as the per-rank
    multiply hook) and rank 0 prints ONE JSON line.  Both workloads are checked against the
    oracle on the global matrices: config 4 weak-scaled (rank r owns rows [r*n, (r+1)*n) of an
    N*n x n A) and config 5 strong-scaled (one n5 x n5 A cut on the product prefix, each rank
    drawing only its block)."""
    import os
    import subprocess
    import sys

    import numpy as np
    import torch

    from oracle import oracle
    from spmm_amd import gen

    n, n5 = 1500, 2500
    dump = str(tmp_path / "slab")
    env = dict(os.environ, SPG_BENCH_HOOK_DUMP=dump, PYTHONPATH=bench.ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(bench.ROOT, "bench.py"), "--gpus", str(world), "--device", "cpu",
           "--multiply-hook", "tests.bench_hooks:oracle_multiply", "--n", str(n), "--config5-n", str(n5),
           "--steps", "2", "--warmup", "1", "--cpu-seconds", "0"]
    r = subprocess.run(cmd, env=env, cwd=bench.ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["steps"] == 2 and line["warmup"] == 1
    # the pipelined-broadcast report is a GPU figure: present, and None on the CPU hook path
    assert "b_values_pipeline" in line and line["b_values_pipeline"] is None
    assert "b_values_pipeline" in line["config5"] and line["config5"]["b_values_pipeline"] is None
    assert line["scaling"] == "weak" and line["config"]["rows_per_rank"] == n
    assert line["config5"]["scaling"] == "strong"

    def stitched(nn):
        parts = [np.load(f"{dump}.n{nn}.rank{k}.npz") for k in range(world)]
        base, ps = 0, [np.zeros(1, np.int64)]
        for q in parts:
            ps.append(q["p"][1:].astype(np.int64) + base)
            base += int(q["p"][-1])
        return (np.concatenate(ps), np.concatenate([q["j"] for q in parts]),
                np.concatenate([q["x"] for q in parts]))

    cpu = torch.device("cpu")
    # config 4, weak: the global A is (world * n) x n
    A = gen.random_csr(world * n, n, 5e-3, seed=42, device=cpu).get()
    B = gen.random_csr(n, n, 5e-3, seed=43, device=cpu).get()
    rp, rj, rx = oracle.spgemm(A, B, keep_zeros=True, sort=True)
    p, j, x = stitched(n)
    assert np.array_equal(p, rp) and np.array_equal(j, rj) and np.array_equal(x.view(np.uint64), rx.view(np.uint64))
    assert line["config"]["nnzC"] == len(rj)
    assert line["config"]["num_products"] == oracle.num_products(A, B)
    # config 5, strong: one n5 x n5 A over both ranks
    A5 = gen.random_csr(n5, n5, 1e-3, seed=42, device=cpu).get()
    B5 = gen.random_csr(n5, n5, 1e-3, seed=43, device=cpu).get()
    rp, rj, rx = oracle.spgemm(A5, B5, keep_zeros=True, sort=True)
    p, j, x = stitched(n5)
    assert np.array_equal(p, rp) and np.array_equal(j, rj) and np.array_equal(x.view(np.uint64), rx.view(np.uint64))
    assert line["config5"]["num_products"] == oracle.num_products(A5, B5)
    r0, r1 = line["config5"]["rows_rank0"]
    assert r0 == 0 and 0 < r1 < n5


def test_pick_keeps_explicit_zero():
    assert bench.pick(0, 3) == 0 and bench.pick(None, 3) == 3
    a = bench.parse(["--alg", "0"])
    assert bench.pick(a.alg, 3) == 0
