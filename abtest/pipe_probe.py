"""Per-step timing of rowblock_step (pipelined and not) with gloo ranks on one GPU: where a
slow pipelined step spends its time (a rehearsal diagnostic, not a benchmark)."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spmm_amd import distributed, gen  # noqa: E402

n, dens = int(os.environ.get("PN", "131072")), 1e-3
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
dev = torch.device("cuda:0")
B = gen.random_csr(n, n, dens, seed=43, dtype=torch.float64, device=dev) if rank == 0 else None
Bw = distributed.broadcast_csr(B, 0, dev)
(r0, r1), A, _ = distributed.rowblock_setup_drawn(
    lambda rows, off: gen.random_csr(rows, n, dens, seed=42, dtype=torch.float64, device=dev, row_offset=off),
    n, Bw.indptr, world, rank)
del Bw
orig = distributed.TileValueBroadcast.__call__
orig_agree = distributed.agree_tiles
marks = {}


def agree(*a, **k):
    t0 = time.perf_counter()
    r = orig_agree(*a, **k)
    marks["agree"] = time.perf_counter() - t0
    return r


def traced(self, geom):
    t0 = time.perf_counter()
    out = orig(self, geom)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    self.t_call = time.perf_counter() - t0
    self.t_parts = (marks.get("agree", 0.0), t1 - t0, time.perf_counter() - t1)
    return out


distributed.agree_tiles = agree
distributed.TileValueBroadcast.__call__ = traced
for pipe in (True, False, True):
    for i in range(3):
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        C, _ = distributed.rowblock_step(A, B, 0, dev, alg=2, pipeline=pipe, n_groups=8)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        dist.barrier()
        t2 = time.perf_counter()
        tv = distributed.rowblock_step.last if pipe else None
        print(f"rank {rank} pipe {pipe} step {i}: {1e3 * (t1 - t0):.1f} ms (+barrier {1e3 * (t2 - t1):.1f}); "
              f"by_tiles call {1e3 * getattr(tv, 't_call', 0):.1f} ms "
              f"(agree / call / sync {'/'.join(f'{1e3 * x:.1f}' for x in getattr(tv, 't_parts', ()))})\n",
              end="", flush=True)
        del C
dist.destroy_process_group()
