#!/usr/bin/env python3
"""CSR x CSR SpGEMM benchmark on MI355X (BASELINE.json metric: GFLOPS + peak HBM bytes).

Step = one complete ``C = A.B`` through the drop-in shim (``spmm_amd.cusparse.spgemm``:
plan, symbolic with its nnz(C) host sync, C allocation, numeric), inputs resident in HBM.

Workloads (``--config``; ``auto`` = 4 at every N):

* ``4`` (the N=1 headline: the largest single-GPU configuration of BASELINE.json, configs[3]):
  N = 65536, density 5e-3, fp64, ALG3 at chunk_fraction 0.2 -- the reference's ALG3 path,
  estimateMemory then the compute (cupy_cusparse/spgemm_from_txt_alg3.cu:194-208).  The plan
  chunks only when the unchunked workspace exceeds the cap (chunk_fraction x P entries of C);
  config 4's dense tiles keep 0.35 GB of workspace against a 17 GB cap, so it runs ONE chunk
  and the line says so (``config.n_chunks``, ``config.alg3_cap``).  The chunked schedule's cost
  at scale is the ``alg3_chunked`` key: config 5 under ALG2 and under ALG3 at chunk_fraction
  0.02 (>= 50 chunks), time and peak side by side (the reference's time / peak trade,
  BASELINE.md 1a).  nnz(C) = 3.46e9: int64 row pointer.  Inputs generated on the device
  (spmm_amd.gen.random_csr).
  At N > 1 it scales WEAK: rank r owns rows [r*65536, (r+1)*65536) of an (N*65536) x 65536
  A of the same density (rank 0's block is the N=1 A), B (258 MB) is broadcast from rank 0
  over RCCL/xGMI inside every step -- structure first, values in flight while the symbolic
  pass runs (spmm_amd.distributed.rowblock_step) -- and every rank writes its own C slab: no
  reduction.  value = sum_r 2 P_r / max-over-ranks time.
* ``2`` (BASELINE configs[1]): random 16384 x 16384, density 1e-3, fp64, A then B from one
  ``default_rng(42)`` stream via scipy.sparse.random (nnz(C) = 4,366,124, P = 4,402,284), ALG1
  single pass.  Reported as the ``config2`` key of the N=1 line.
* ``5``: N = 262144, density 1e-3, fp64, ALG2, STRONG scaling over the ranks (north_star's
  8-GPU configuration): rank r owns the rows [r0, r1) cut on the product-count prefix, B
  (826 MB) broadcast inside every step.  At N > 1 it is also reported as the ``config5`` key
  of the line (``--config5-n 0`` skips it).

``python3 bench.py --gpus N`` (N > 1) without a launcher spawns N worker processes itself
(before anything touches the GPU) with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, exactly
as ``torch.distributed.run`` would; under a launcher (WORLD_SIZE set) it is one rank.

Also reported: ``roofline`` for the numeric-phase kernel (compulsory bytes of the product,
SURVEY 8d, / the phase's device time from HIP events on the library's stream, per launch),
``cpu_baseline`` = scipy's ``A @ B`` -- the reference's CPU comparator
(SpGEMM_vs_SpMV/profiler.py:408) -- timed in forked children with their RSS growth, on
rank 0 at N=1 (a bounded row sample of config 4), with the oracle's single-thread and OpenMP
restatements beside it.

``--device cpu --multiply-hook MOD:FN`` (tests only) runs the same multi-rank step logic on
CPU tensors over gloo with the hook as the per-rank multiply (tests/test_bench_cpu.py).
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CSR×CSR SpGEMM GFLOPS + peak HBM bytes, random N×N at stated density"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    "2": dict(n=16384, density=1e-3, alg=1, gen="scipy", steps=200, warmup=20,
              name="BASELINE config 2 (configs[1])"),
    "4": dict(n=65536, density=5e-3, alg=3, gen="device", steps=5, warmup=2,
              name="BASELINE config 4 (configs[3], ALG3 with its HBM cap)"),
    "5": dict(n=262144, density=1e-3, alg=2, gen="device", steps=5, warmup=2,
              name="BASELINE config 5 (configs[4], row blocks, B broadcast)"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default per config)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default per config)")
    ap.add_argument("--config", default="auto", choices=["auto", "2", "4", "5"])
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--density", type=float, default=None)
    ap.add_argument("--alg", type=int, default=None)
    ap.add_argument("--chunk-fraction", type=float, default=0.2)
    ap.add_argument("--dtype", default="float64", choices=["float32", "float64"])
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="budget of the CPU-baseline sample (0 disables it)")
    ap.add_argument("--no-config2", action="store_true", help="N=1: skip the config2 key")
    ap.add_argument("--no-alg3-chunked", action="store_true", help="N=1: skip the alg3_chunked key")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="N>1: B's values in one broadcast (overlapping the symbolic pass only) instead of "
                         "tile-major groups overlapping the numeric pass")
    ap.add_argument("--value-groups", type=int, default=8, help="N>1: column-tile groups of the values broadcast")
    ap.add_argument("--config5-n", type=int, default=262144,
                    help="N>1: size of the strong-scaled config5 key (0 skips it)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="PMC traffic summary written by profiles/pmc_to_json.py")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: tests only (gloo, --multiply-hook as the per-rank multiply)")
    ap.add_argument("--multiply-hook", default=None,
                    help="MOD:FN called as FN(A_block, B, wait_values) -> C (tests only)")
    return ap.parse_args(argv)


def pick(value, default):
    """An explicit flag wins, including 0 (`args.alg or cfg` dropped --alg 0)."""
    return default if value is None else value


def compulsory_bytes(n_rows, n_cols, nnzA, nnzB, nnzC, vb, ib_c=4):
    """SURVEY 8d compulsory bytes: A and B read once (int32 row pointers), C written once
    (its row pointer ib_c bytes per entry: 8 once nnz(C) >= 2^31)."""
    return 4 * (n_rows + 1) + 4 * (n_cols + 1) + ib_c * (n_rows + 1) + (4 + vb) * (nnzA + nnzB + nnzC)


# ------------------------------------------------------------------ launcher (no torchrun)

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _forward(pipe, rank):
    """A worker's stdout: rank 0's JSON line to our stdout, everything else (the collective
    libraries' banners) to stderr, so the parent prints exactly ONE JSON line."""
    for raw in iter(pipe.readline, b""):
        line = raw.decode(errors="replace")
        out = sys.stdout if rank == 0 and line.lstrip().startswith("{") else sys.stderr
        out.write(line)
        out.flush()
    pipe.close()


def spawn_workers(n, argv):
    """`--gpus N` without a launcher: start N fresh worker processes of this script (rank r
    on GPU r), wait for all of them and return the worst exit status.  Runs before anything
    touches the GPU and never re-execs this process.  Rank 0's JSON line is the output."""
    import threading
    port = _free_port()
    procs, readers = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE))
        readers.append(threading.Thread(target=_forward, args=(procs[-1].stdout, r), daemon=True))
        readers[-1].start()
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):   # one rank failed: end the others
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        time.sleep(0.05)
    for t in readers:
        t.join(timeout=30)
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


# ------------------------------------------------------------------ measurement pieces

def cpu_baseline(A_h, B_h, rows_sample, budget_s):
    """scipy A @ B (the reference's comparator) in forked children: median time and RSS
    growth; the oracle port (single thread) and its OpenMP form beside it.  On a row sample
    of A when `rows_sample` is given (configs 4/5: C does not fit a host sample budget)."""
    import scipy.sparse as sp
    from oracle import oracle
    from spmm_amd import profiling
    A_s = A_h if rows_sample is None else sp.csr_matrix(A_h[rows_sample])
    P = oracle.num_products(A_s, B_h)
    runs, t_start = [], time.perf_counter()
    while len(runs) < 30 and (len(runs) < 3 or time.perf_counter() - t_start < budget_s):
        runs.append(profiling.profile_op_cpu("scipy A@B", lambda: A_s @ B_h))
    t = float(np.median([r.time_ms for r in runs])) / 1e3
    rss = int(np.median([r.peak_ram or 0 for r in runs]))
    oracle.build()
    pt = []
    t_start = time.perf_counter()
    while len(pt) < 20 and (len(pt) < 2 or time.perf_counter() - t_start < budget_s / 2):
        t0 = time.perf_counter()
        oracle.spgemm(A_s, B_h, keep_zeros=True, sort=True)
        pt.append(time.perf_counter() - t0)
    nthr = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    om = []
    t_start = time.perf_counter()
    while len(om) < 20 and (len(om) < 2 or time.perf_counter() - t_start < budget_s / 2):
        t0 = time.perf_counter()
        oracle.spgemm(A_s, B_h, keep_zeros=True, sort=True, threads=nthr)
        om.append(time.perf_counter() - t0)
    t_port, t_omp = float(np.median(pt)), float(np.median(om))
    what = ("the whole product (same A, B)" if rows_sample is None
            else f"{len(rows_sample)} sampled rows of A times all of B ({P} products)")
    return {"value": round(2.0 * P / t / 1e9, 4), "unit": "GFLOPS", "cores": 1, "kind": "reference",
            "sample": f"scipy.sparse A@B (csr_matmat, single thread; the reference's CPU comparator, "
                      f"SpGEMM_vs_SpMV/profiler.py:408) on {what}, median of {len(runs)} forked runs",
            "ms_per_run": round(t * 1e3, 3), "rss_growth_bytes": rss,
            "port": {"gflops": round(2.0 * P / t_port / 1e9, 4), "ms_per_run": round(t_port * 1e3, 3),
                     "threads": 1, "what": "oracle/gustavson.c (scipy's rule restated in C)"},
            "omp": {"gflops": round(2.0 * P / t_omp / 1e9, 4), "ms_per_run": round(t_omp * 1e3, 3),
                    "threads": nthr, "what": "oracle/gustavson.c, OpenMP over rows",
                    "thread_cap": (f"OMP_NUM_THREADS={os.environ['OMP_NUM_THREADS']}: the CPU share this job gets "
                                   f"on the GPU box (os.cpu_count()={os.cpu_count()} counts the whole host)")
                    if os.environ.get("OMP_NUM_THREADS") else "all host CPUs"},
            "host_cpus": os.cpu_count()}


def traffic_for(pmc_path, key, build_id, source_id=None):
    """HBM bytes per launch from the committed PMC summary -- only when it was collected on
    this very build of the library, or on a build of the same sources (else None: the
    number would be stale)."""
    if not os.path.exists(pmc_path):
        return None, None
    try:
        with open(pmc_path) as f:
            e = json.load(f).get(key, {})
    except Exception:
        return None, None
    if e.get("build_id") != build_id and (source_id is None or e.get("source_id") != source_id):
        return None, e.get("build_id")
    return e.get("hbm_bytes_per_launch"), e.get("build_id")


class Ctx:
    """Device, rank and the collectives of one bench process."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={self.world}")
        self.gpu = args.device == "cuda"
        if self.gpu:
            # one process per GPU; a rehearsal with more ranks than GPUs (SPG_DIST_BACKEND=gloo
            # on a one-GPU box) puts several ranks on one device
            self.local_dev = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(self.local_dev)
            self.dev = torch.device("cuda", self.local_dev)
        else:
            self.local_dev, self.dev = None, torch.device("cpu")
        self.backend = None
        if self.world > 1:
            backend = os.environ.get("SPG_DIST_BACKEND", "nccl" if self.gpu else "gloo")   # nccl = RCCL
            dist.init_process_group(backend, **({"device_id": self.dev} if backend == "nccl" else {}))
            self.backend = backend

    def collective_name(self):
        """The collective library the broadcasts actually ran on (the line must not claim RCCL
        for a gloo rehearsal)."""
        return {"nccl": "RCCL", "gloo": "gloo (host-staged; a rehearsal, not xGMI)"}.get(self.backend, self.backend)

    def sync(self):
        if self.gpu:
            self.torch.cuda.synchronize()

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def reduce(self, vals, op):
        """vals (floats) reduced over the ranks with `op` ("max" / "sum")."""
        if self.world == 1:
            return list(vals)
        t = self.torch.tensor(list(vals), dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return [float(x) for x in t.tolist()]


def timed(ctx, step, steps, warmup):
    """W untimed steps, then exactly K timed steps between barrier + synchronize on both
    sides.  Returns (seconds, the last step's result)."""
    for _ in range(warmup):
        C = step()
        del C
    ctx.sync()
    ctx.barrier()
    t0 = time.perf_counter()
    C = None
    for i in range(steps):
        C = step()
        if i < steps - 1:
            del C
    ctx.sync()
    ctx.barrier()
    return time.perf_counter() - t0, C


def phase_times(ctx, step, reps):
    """Per-phase device times of `reps` extra steps (HIP events on the library's stream,
    which is torch's current stream).  {} on CPU."""
    if not ctx.gpu:
        for _ in range(reps):
            C = step()
            del C
        return {}
    from spmm_amd import _lib
    h = _lib.get_handle(ctx.local_dev)
    h.set_stream(ctx.torch.cuda.current_stream(ctx.dev).cuda_stream)
    h.set_timing(True)
    for _ in range(reps):
        C = step()
        del C
    ph = h.get_timing()
    h.set_timing(False)
    return ph


def roofline(phases, reps, kernel, bytes_product, ms_per_step, traffic, traffic_build, step_frac=True):
    """`roofline` object of the numeric-phase kernel: algorithmic (compulsory) bytes of the
    product split over its numeric launches / the average launch time from HIP events."""
    num_ms, num_launches = phases.get("numeric", (0.0, 0))
    if not num_launches:
        return None
    per = max(1, num_launches // reps)
    avg = num_ms / num_launches
    b_launch = bytes_product / per
    achieved = b_launch / (avg * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_build_id": traffic_build,
            "kernel": kernel + " (numeric phase)", "bytes_per_launch": int(b_launch),
            "launches_per_product": per, "avg_launch_ms": round(avg, 5),
            "step_frac": round(bytes_product / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if step_frac else None}


def lib_ids(ctx):
    if not ctx.gpu:
        return None, None
    from spmm_amd import _lib
    return _lib.build_id(), _lib.source_id()


def load_hook(spec):
    if not spec:
        return None
    mod, fn = spec.split(":")
    return getattr(importlib.import_module(mod), fn)


def tile_kernel(ctx, A, B, alg, cf):
    """(name of the numeric tile kernel the product runs, its number of row chunks)."""
    if not ctx.gpu or B is None:
        return "k_tile", 1
    from spmm_amd import cusparse
    info = cusparse.plan_info(A, B, alg=alg, chunk_fraction=cf)
    nch = len(info["chunk_rows"]) - 1
    if info["path"] != "tile":
        return info["path"], nch
    rg = info.get("record_group", 1)
    return (("k_tile_dn" if info["dense_tiles"] else "k_tile_sp") + f" (TW={info['tile_width']}"
            + (f", cooperative record groups of {rg} tiles" if rg > 1 else "") + f", {nch} chunk(s))"), nch


def alg3_label(alg, nch):
    if alg != 3:
        return f"ALG{alg}"
    return (f"ALG3, {nch} chunks (cap binding)" if nch > 1
            else "ALG3, 1 chunk (cap not binding: the unchunked workspace is within chunk_fraction x P entries)")


def gen_device(ctx, n, dens, seed, tdt, rows=None, row_offset=0):
    from spmm_amd import gen
    return gen.random_csr(n if rows is None else rows, n, dens, seed=seed, dtype=tdt, device=ctx.dev,
                          row_offset=row_offset)


# ------------------------------------------------------------------ workloads

def run_config4(ctx, args, cfg, tdt, vb, hook):
    """Config 4 at N=1, weak-scaled row blocks at N > 1.  Returns the JSON line's fields."""
    from spmm_amd import cusparse, distributed
    n = pick(args.n, cfg["n"])
    dens = pick(args.density, cfg["density"])
    alg = pick(args.alg, cfg["alg"])
    steps, warmup, cf = pick(args.steps, cfg["steps"]), pick(args.warmup, cfg["warmup"]), args.chunk_fraction
    w, r = ctx.world, ctx.rank
    # rank r's block of the (w*n) x n global A: rows [r*n, (r+1)*n); rank 0's is the N=1 A
    A = gen_device(ctx, n, dens, args.seed, tdt, rows=n, row_offset=r * n)
    B = gen_device(ctx, n, dens, args.seed + 1, tdt) if (r == 0 or w == 1) else None
    bcast_ms = None
    if w > 1:
        Bw = distributed.broadcast_csr(B, 0, ctx.dev)   # warms RCCL up; B's row lengths
        P = int(distributed.product_prefix(A, Bw.indptr)[-1])
        nnzB = Bw.nnz
        del Bw
        bcast_ms = broadcast_ms(ctx, B)

        def step():
            C, _ = distributed.rowblock_step(A, B, 0, ctx.dev, alg=alg, chunk_fraction=cf, multiply=hook,
                                             pipeline=None if not args.no_pipeline else False,
                                             n_groups=args.value_groups)
            return C
    else:
        P, nnzB = cusparse.num_products(A, B), B.nnz

        def step():
            return cusparse.spgemm(A, B, alg=alg, chunk_fraction=cf)
    elapsed, C = timed(ctx, step, steps, warmup)
    nnzC, ib_c = C.nnz, C.indptr.element_size()
    peak = last_peak(ctx)
    del C
    if ctx.gpu:
        ctx.torch.cuda.empty_cache()
    (elapsed,) = ctx.reduce([elapsed], "max")
    P_all, nnz_all = ctx.reduce([float(P), float(nnzC)], "sum")
    (peak_max,) = ctx.reduce([float(peak)], "max")
    ms = elapsed / steps * 1e3
    reps = 2
    ph = phase_times(ctx, step, reps)
    bid, sid = lib_ids(ctx)
    key = f"c4_n{n}_d{dens:g}_{args.dtype}_alg{alg}_w1"   # per-rank work = the N=1 product
    traffic, tb = traffic_for(args.pmc, key, bid, sid) if ctx.gpu else (None, None)
    kname, nch = tile_kernel(ctx, A, B, alg, cf)
    rf = roofline(ph, reps, kname, compulsory_bytes(A.shape[0], n, A.nnz, nnzB, nnzC, vb, ib_c), ms, traffic, tb,
                  step_frac=(w == 1))
    cpu = None
    if r == 0 and w == 1 and args.cpu_seconds > 0 and ctx.gpu:
        A_h, B_h = A.get(), B.get()
        sample = np.sort(np.random.default_rng(0).choice(n, size=min(n, 1024), replace=False))
        cpu = cpu_baseline(A_h, B_h, sample, args.cpu_seconds)
    desc = (f"{cfg['name']}: random CSR {n}x{n} density={dens:g} {args.dtype} "
            f"(spmm_amd.gen.random_csr on the device, seeds {args.seed}/{args.seed + 1}), "
            f"{alg3_label(alg, nch)}, chunk_fraction {cf}")
    if w > 1:
        desc += (f"; weak scaling: rank r owns rows [r*{n}, (r+1)*{n}) of a {w * n}x{n} A "
                 f"(rank 0's block is the N=1 A), B broadcast over {ctx.collective_name()} inside every step, "
                 "no reduction")
    out = {
        "value": round(2.0 * P_all * steps / elapsed / 1e9, 3), "steps": steps, "warmup": warmup,
        "ms_per_step": round(ms, 5), "scaling": "weak",
        "config": {"workload": desc, "N": n, "rows_per_rank": n, "density": dens, "alg": alg,
                   "chunk_fraction": cf, "n_chunks": nch,
                   "alg3_cap": None if alg != 3 else ("binding" if nch > 1 else "not binding"),
                   "nnzB": int(nnzB), "nnzA_rank0" if w > 1 else "nnzA": int(A.nnz),
                   "nnzC": int(nnz_all), "num_products": int(P_all),
                   "parallelism": "single GPU" if w == 1 else
                   f"row-block x{w} (weak), B broadcast over {ctx.collective_name()}"},
        "peak_hbm_bytes": int(peak_max), "roofline": rf,
        "phases_ms_per_step": {k: round(v[0] / reps, 5) for k, v in ph.items() if v[1]},
        "b_broadcast_ms": None if bcast_ms is None else round(bcast_ms, 3),
        "b_values_pipeline": None if w == 1 else pipeline_report(ctx, args, A, B, alg, cf, hook, ms),
        "cpu_baseline": cpu,
    }
    del A, B
    return out


def broadcast_ms(ctx, B):
    """The B broadcast alone (median of 3), reported beside the step."""
    from spmm_amd import distributed
    ts = []
    for _ in range(3):
        ctx.sync()
        ctx.barrier()
        t0 = time.perf_counter()
        Bt = distributed.broadcast_csr(B, 0, ctx.dev)
        ctx.sync()
        ctx.barrier()
        ts.append(time.perf_counter() - t0)
        del Bt
    return float(np.median(ts)) * 1e3


def pipeline_report(ctx, args, A, B, alg, cf, hook, ms):
    """How much of B's values broadcast the step hides (N > 1): the values broadcast alone
    and B's structure broadcast alone (median of 3 each; the structure is what every
    rank waits for before its layout and symbolic pass), the step with the values in one
    broadcast that overlaps only the symbolic pass (2 steps), and the step as measured
    (tile-major value groups in flight from before the symbolic pass through the numeric
    tiles), and the pipelined step with the values sent after the symbolic pass (round 4's
    order).  hidden_ms = unpipelined - measured; overlap_frac = hidden_ms /
    values_broadcast_ms; symbolic_hidden_ms = values-after-symbolic - measured.  None on the
    CPU test path."""
    if not ctx.gpu or hook is not None:
        return None
    from spmm_amd import distributed
    torch = ctx.torch
    # the values alone (rank 0's B; the others receive into a buffer of its size)
    meta = torch.tensor([B.nnz, B.data.element_size()] if B is not None else [0, 0], dtype=torch.int64,
                        device=ctx.dev)
    ctx.dist.broadcast(meta, 0)
    nnzB, esz = (int(x) for x in meta.tolist())
    buf = B.data.view(torch.uint8) if B is not None else torch.empty(nnzB * esz, dtype=torch.uint8, device=ctx.dev)
    ts = []
    for _ in range(3):
        ctx.sync()
        ctx.barrier()
        t0 = time.perf_counter()
        ctx.dist.broadcast(buf, 0)
        ctx.sync()
        ctx.barrier()
        ts.append(time.perf_counter() - t0)
    vms = float(np.median(ts)) * 1e3
    ts = []
    for _ in range(3):
        ctx.sync()
        ctx.barrier()
        t0 = time.perf_counter()
        distributed.broadcast_csr(B, 0, ctx.dev, values=False)
        ctx.sync()
        ctx.barrier()
        ts.append(time.perf_counter() - t0)
    sms = float(np.median(ts)) * 1e3
    sbytes = None
    if B is not None:   # (rank 0 prints the line)
        nb1 = distributed.cols16_layout(B.shape[0], B.shape[1], B.nnz)
        sbytes = B.indptr.element_size() * (B.shape[0] + 1) + (4 * B.nnz if nb1 < 0 else 4 * B.shape[0] * nb1 + 2 * B.nnz)
    pipelined = not args.no_pipeline
    last = distributed.rowblock_step.last

    def other():
        C, _ = distributed.rowblock_step(A, B, 0, ctx.dev, alg=alg, chunk_fraction=cf, pipeline=not pipelined,
                                         n_groups=args.value_groups)
        return C
    el, C = timed(ctx, other, 2, 1)
    del C
    (el,) = ctx.reduce([el], "max")
    oms = el / 2 * 1e3
    ums, pms = (oms, ms) if pipelined else (ms, oms)
    lms = None
    if pipelined:   # the values after the symbolic pass (round 4's order): what sending them first hides
        def late():
            C, _ = distributed.rowblock_step(A, B, 0, ctx.dev, alg=alg, chunk_fraction=cf, pipeline=True,
                                             n_groups=args.value_groups, values_first=False)
            return C
        el, C = timed(ctx, late, 2, 1)
        del C
        (el,) = ctx.reduce([el], "max")
        lms = el / 2 * 1e3
    groups = len(last.groups) if (pipelined and last is not None and last.pipelined) else None
    return {"pipelined": pipelined and groups is not None, "groups": groups,
            "values_broadcast_ms": round(vms, 3), "structure_broadcast_ms": round(sms, 3),
            "structure_bytes": sbytes, "values_bytes": nnzB * esz,
            "step_ms_unpipelined": round(ums, 4),
            "step_ms_pipelined": round(pms, 4), "hidden_ms": round(ums - pms, 4),
            "step_ms_values_after_symbolic": None if lms is None else round(lms, 4),
            "symbolic_hidden_ms": None if lms is None else round(lms - pms, 4),
            "overlap_frac": round((ums - pms) / vms, 4) if vms > 0 else None}


def last_peak(ctx):
    if not ctx.gpu:
        return 0
    from spmm_amd import cusparse
    return cusparse.last_stats.peak_bytes


def run_config5(ctx, args, cfg, n, tdt, vb, hook, steps, warmup):
    """Config 5 strong-scaled: the rows of one n x n A cut on the product prefix over the
    ranks (each rank draws only its own block), B broadcast inside every step."""
    from spmm_amd import cusparse, distributed
    dens, alg, cf = cfg["density"], cfg["alg"], args.chunk_fraction
    w, r = ctx.world, ctx.rank
    B = gen_device(ctx, n, dens, args.seed + 1, tdt) if (r == 0 or w == 1) else None
    if w > 1:
        Bw = distributed.broadcast_csr(B, 0, ctx.dev)
        nnzB = Bw.nnz

        def draw(rows, off):
            return gen_device(ctx, n, dens, args.seed, tdt, rows=rows, row_offset=off)
        rows, A, P = distributed.rowblock_setup_drawn(draw, n, Bw.indptr, w, r)
        del Bw
        if ctx.gpu:
            ctx.torch.cuda.empty_cache()
        bcast_ms = broadcast_ms(ctx, B)

        def step():
            C, _ = distributed.rowblock_step(A, B, 0, ctx.dev, alg=alg, chunk_fraction=cf, multiply=hook,
                                             pipeline=None if not args.no_pipeline else False,
                                             n_groups=args.value_groups)
            return C
    else:
        A = gen_device(ctx, n, dens, args.seed, tdt)
        rows, P, nnzB, bcast_ms = (0, n), cusparse.num_products(A, B), B.nnz, None

        def step():
            return cusparse.spgemm(A, B, alg=alg, chunk_fraction=cf)
    elapsed, C = timed(ctx, step, steps, warmup)
    nnzC, ib_c = C.nnz, C.indptr.element_size()
    peak = last_peak(ctx)
    del C
    if ctx.gpu:
        ctx.torch.cuda.empty_cache()
    (elapsed,) = ctx.reduce([elapsed], "max")
    P_all, nnz_all = ctx.reduce([float(P), float(nnzC)], "sum")
    (peak_max,) = ctx.reduce([float(peak)], "max")
    ms = elapsed / steps * 1e3
    reps = 1
    ph = phase_times(ctx, step, reps)
    kname, nch = tile_kernel(ctx, A, B, alg, cf)
    rf = roofline(ph, reps, kname, compulsory_bytes(A.shape[0], n, A.nnz, nnzB, nnzC, vb, ib_c),
                  ms, None, None, step_frac=False)
    out = {"gflops": round(2.0 * P_all * steps / elapsed / 1e9, 3), "ms_per_step": round(ms, 5),
           "steps": steps, "warmup": warmup, "scaling": "strong", "N": n, "density": dens, "alg": alg,
           "num_products": int(P_all), "nnzC": int(nnz_all), "rows_rank0": list(rows), "n_chunks": nch,
           "peak_hbm_bytes_max_rank": int(peak_max), "b_broadcast_ms": None if bcast_ms is None else round(bcast_ms, 3),
           "b_values_pipeline": None if w == 1 else pipeline_report(ctx, args, A, B, alg, cf, hook, ms),
           "roofline_rank0": rf, "phases_ms_per_step": {k: round(v[0] / reps, 5) for k, v in ph.items() if v[1]},
           "workload": (f"{cfg['name']}: random CSR {n}x{n} density={dens:g} {args.dtype}, ALG{alg}; "
                        f"{w} row blocks cut on the product prefix (each rank draws its own block), "
                        f"{alg3_label(alg, nch)}, "
                        + ("one GPU" if w == 1 else f"B broadcast over {ctx.collective_name()} inside every step"))}
    del A, B
    return out


def _device_sig(torch, x, piece=1 << 27):
    """Position-weighted wrapping int64 sum of a 1-D integer tensor, computed in pieces."""
    acc = torch.zeros((), dtype=torch.int64, device=x.device)
    for s in range(0, x.numel(), piece):
        v = x[s:s + piece].to(torch.int64)
        w = torch.arange(s, s + v.numel(), device=x.device, dtype=torch.int64) % 1000003 + 1
        acc += torch.sum(v * w)
    return int(acc)


def run_alg3_chunked(ctx, args, tdt, n=262144, dens=1e-3, cf=0.02, steps=2, warmup=1):
    """ALG3's time / peak trade where its cap binds: config 5 on one GPU under ALG2
    and under ALG3 at chunk_fraction `cf` (>= 50 equal-product row chunks), same inputs, the
    results compared bit for bit on device (row pointer, columns, value bits)."""
    from spmm_amd import cusparse
    A = gen_device(ctx, n, dens, args.seed, tdt)
    B = gen_device(ctx, n, dens, args.seed + 1, tdt)
    P = cusparse.num_products(A, B)
    out = {"N": n, "density": dens, "num_products": int(P),
           "workload": f"BASELINE config 5 shape (N={n}, density {dens:g}) on one GPU: ALG2 vs ALG3 at chunk_fraction {cf}"}
    ref = None
    for alg, c in ((2, 0.2), (3, cf)):
        elapsed, C = timed(ctx, lambda: cusparse.spgemm(A, B, alg=alg, chunk_fraction=c), steps, warmup)
        _, nch = tile_kernel(ctx, A, B, alg, c)
        key = "alg2" if alg == 2 else "alg3"
        out[key] = {"chunk_fraction": c, "n_chunks": nch, "ms_per_step": round(elapsed / steps * 1e3, 3),
                    "gflops": round(2.0 * P * steps / elapsed / 1e9, 3),
                    "peak_hbm_bytes": int(cusparse.last_stats.peak_bytes),
                    # the working set ALG3 caps (peak minus C's own arrays): the figure comparable
                    # to the reference's ALG1 -> ALG3 trade (6.03 -> 2.44 GB)
                    "workspace_bytes": int(cusparse.last_stats.workspace_bytes)}
        # the same C under both schedules: position-weighted sums of the arrays on the device,
        # in pieces (no 190 GB copy to the host, no int64 copy of all of C)
        torch = ctx.torch
        sig = (_device_sig(torch, C.indptr.to(torch.int64)), _device_sig(torch, C.indices),
               _device_sig(torch, C.data.view(torch.int64)))
        ref = sig if ref is None else ref
        out[key]["same_result_as_alg2"] = sig == ref
        del C
        torch.cuda.empty_cache()
    out["alg3_over_alg2_time"] = round(out["alg3"]["ms_per_step"] / out["alg2"]["ms_per_step"], 3)
    out["alg3_over_alg2_peak"] = round(out["alg3"]["peak_hbm_bytes"] / out["alg2"]["peak_hbm_bytes"], 3)
    out["alg3_over_alg2_workspace"] = round(out["alg3"]["workspace_bytes"] / max(1, out["alg2"]["workspace_bytes"]), 4)
    del A, B
    return out


def dense_matmul_ms(torch, A, B, reps=10, warmup=3) -> float:
    """ms per dense torch.matmul of A and B densified (same dtype, same device): the dense GEMM
    the reference's dense_vs_sparseGEMM compares SpGEMM with, timed with events."""
    def dense(M):
        D = torch.zeros(M.shape, dtype=M.data.dtype, device=M.data.device)
        rows = torch.repeat_interleave(torch.arange(M.shape[0], device=M.data.device),
                                       (M.indptr[1:] - M.indptr[:-1]).to(torch.int64))
        D[rows, M.indices.to(torch.int64)] = M.data
        return D
    Ad, Bd = dense(A), dense(B)
    for _ in range(warmup):
        torch.matmul(Ad, Bd)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.matmul(Ad, Bd)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del Ad, Bd
    return ms


def run_config3_fp32(ctx, args, n=8192, dens=0.1, steps=10, warmup=2):
    """BASELINE config 3's densest point in fp32, the dtype of every published reference figure
    (SpGEMM_alg_comparison/profiler.py:215-222, dense_vs_sparseGEMM/utils.py:278-289): one
    C = A.B at N=8192, density 0.1 (ALG2), with its phases, and the dense fp32 GEMM of the same
    matrices (torch.matmul: rocBLAS/hipBLASLt sgemm) timed in the same process, as the
    reference's dense_vs_sparseGEMM/utils.py:278-289 times its torch.matmul -- the break-even
    that sweep looks for."""
    from spmm_amd import cusparse
    torch = ctx.torch
    A = gen_device(ctx, n, dens, args.seed, torch.float32)
    B = gen_device(ctx, n, dens, args.seed + 1, torch.float32)
    P = cusparse.num_products(A, B)
    elapsed, C = timed(ctx, lambda: cusparse.spgemm(A, B, alg=2), steps, warmup)
    del C
    ph = phase_times(ctx, lambda: cusparse.spgemm(A, B, alg=2), 2)
    kname, _ = tile_kernel(ctx, A, B, 2, 0.2)
    out = {"N": n, "density": dens, "dtype": "f32", "alg": 2, "num_products": int(P),
           "ms_per_step": round(elapsed / steps * 1e3, 4), "gflops": round(2.0 * P * steps / elapsed / 1e9, 3),
           "kernel": kname, "phases_ms_per_step": {k: round(v[0] / 2, 5) for k, v in ph.items() if v[1]},
           "sgemm_ms_same_n": round(dense_matmul_ms(torch, A, B), 4)}
    del A, B
    torch.cuda.empty_cache()
    return out


def run_config2(ctx, args, cfg, npdt, vb, with_cpu):
    """Config 2 (ALG1, N=16384) on one GPU: GFLOPS, its k_row roofline and the other ALGs."""
    from spmm_amd import _lib, cusparse, gen
    from spmm_amd.sparse import csr_matrix
    n, dens, alg, cf = cfg["n"], cfg["density"], cfg["alg"], args.chunk_fraction
    A_h, B_h = gen.scipy_pair(n, dens, seed=args.seed, dtype=npdt)
    A, B = csr_matrix(A_h, device=ctx.dev), csr_matrix(B_h, device=ctx.dev)
    P = cusparse.num_products(A, B)
    steps, warmup = cfg["steps"], cfg["warmup"]

    def step():
        return cusparse.spgemm(A, B, alg=alg, chunk_fraction=cf)
    elapsed, C = timed(ctx, step, steps, warmup)
    nnzC, ib_c = C.nnz, C.indptr.element_size()
    peak = cusparse.last_stats.peak_bytes
    del C
    ms = elapsed / steps * 1e3
    other = {}
    for a2 in (2, 3):
        t, _ = timed(ctx, lambda: cusparse.spgemm(A, B, alg=a2, chunk_fraction=cf), max(5, steps // 2), 3)
        dt = t / max(5, steps // 2)
        other[f"alg{a2}"] = {"gflops": round(2.0 * P / dt / 1e9, 3), "ms_per_step": round(dt * 1e3, 5),
                             "peak_hbm_bytes": int(cusparse.last_stats.peak_bytes)}
    reps = 10
    ph = phase_times(ctx, step, reps)
    key = f"c2_n{n}_d{dens:g}_{args.dtype}_alg{alg}_w1"
    traffic, tb = traffic_for(args.pmc, key, _lib.build_id(), _lib.source_id())
    rf = roofline(ph, reps, "k_row", compulsory_bytes(n, n, A.nnz, B.nnz, nnzC, vb, ib_c), ms, traffic, tb)
    out = {"gflops": round(2.0 * P * steps / elapsed / 1e9, 3), "ms_per_step": round(ms, 5),
           "steps": steps, "warmup": warmup, "N": n, "density": dens, "alg": alg, "nnzC": int(nnzC),
           "num_products": int(P), "peak_hbm_bytes": int(peak), "roofline": rf,
           "phases_ms_per_step": {k: round(v[0] / reps, 5) for k, v in ph.items() if v[1]},
           "other_algs": other,
           "workload": (f"{cfg['name']}: random CSR {n}x{n} density={dens:g} {args.dtype} "
                        "(scipy.sparse.random, default_rng(42); A then B), ALG1 single-pass numeric")}
    if with_cpu and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(A_h, B_h, None, args.cpu_seconds)
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_workers(args.gpus, argv)   # before any GPU call; no re-exec
    ctx = Ctx(args)
    hook = load_hook(args.multiply_hook)
    if hook is None and not ctx.gpu:
        raise SystemExit("--device cpu needs --multiply-hook (the product path runs on the GPU only)")
    torch = ctx.torch
    npdt = np.float64 if args.dtype == "float64" else np.float32
    tdt = torch.float64 if args.dtype == "float64" else torch.float32
    vb = 8 if npdt == np.float64 else 4
    name = args.config if args.config != "auto" else "4"
    if ctx.world > 1 and name == "2":
        raise SystemExit("several GPUs run the row-block workloads (config 4 weak, config 5 strong)")

    line = {"metric": METRIC, "unit": "GFLOPS", "n_gpus": ctx.world, "higher_is_better": True,
            "vs_baseline": None, "dtype": "f64" if vb == 8 else "f32", "data": "synthetic"}
    if name == "4":
        res = run_config4(ctx, args, CONFIGS["4"], tdt, vb, hook)
        line.update(res)
        if ctx.world == 1 and ctx.gpu and not args.no_config2:
            line["config2"] = run_config2(ctx, args, CONFIGS["2"], npdt, vb, with_cpu=False)
        if ctx.world == 1 and ctx.gpu and not args.no_alg3_chunked:
            line["alg3_chunked"] = run_alg3_chunked(ctx, args, tdt)
        if ctx.world == 1 and ctx.gpu and not args.no_config2:
            line["config3_fp32"] = run_config3_fp32(ctx, args)
        if ctx.world > 1 and args.config5_n > 0:
            line["config5"] = run_config5(ctx, args, CONFIGS["5"], args.config5_n, tdt, vb, hook,
                                          steps=3, warmup=1)
    elif name == "5":
        cfg = CONFIGS["5"]
        res = run_config5(ctx, args, cfg, pick(args.n, cfg["n"]), tdt, vb, hook,
                          pick(args.steps, cfg["steps"]), pick(args.warmup, cfg["warmup"]))
        line.update({"value": res.pop("gflops"), "steps": res.pop("steps"), "warmup": res.pop("warmup"),
                     "ms_per_step": res.pop("ms_per_step"), "scaling": res.pop("scaling"),
                     "config": res, "peak_hbm_bytes": res.pop("peak_hbm_bytes_max_rank"),
                     "roofline": res.pop("roofline_rank0")})
    else:   # config 2 as the line (one GPU)
        res = run_config2(ctx, args, CONFIGS["2"], npdt, vb, with_cpu=ctx.rank == 0)
        line.update({"value": res.pop("gflops"), "steps": res.pop("steps"), "warmup": res.pop("warmup"),
                     "ms_per_step": res.pop("ms_per_step"), "scaling": "weak",
                     "peak_hbm_bytes": res.pop("peak_hbm_bytes"), "roofline": res.pop("roofline"),
                     "cpu_baseline": res.pop("cpu_baseline", None), "config": res})
    line["lib_build_id"], line["lib_source_id"] = lib_ids(ctx)
    if ctx.rank == 0:
        print(json.dumps(line), flush=True)
    if ctx.world > 1:
        ctx.barrier()
        ctx.dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
