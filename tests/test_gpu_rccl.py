"""The row-block step on its real collective backend: RCCL (torch.distributed "nccl").

Every earlier multi-rank run used gloo (host-staged broadcasts).  Several code paths of
spmm_amd.distributed run only under "nccl": ``init_process_group(device_id=...)``, the
device-tensor all_gather of ``agree_tiles``, the async broadcasts of tile-major value slices
on RCCL's own stream and the ``work.wait()`` ordering of the numeric tiles after them
(the reference's protocol: modify_src/cupy-src/cupyx/distributed/_nccl_comm.py:651-674).
RCCL takes one rank per GPU, so on a one-GPU box this is a world of size 1: every
collective runs through RCCL's kernels and streams, with rank 0 as the broadcast source.
Run in a child process (a fresh process group, bounded by a timeout); the C slabs of
``pipeline=True`` (values before the symbolic pass, and after it: ``values_first=False``) and
``pipeline=False`` are checked bit for bit against the oracle.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import os, sys, json
import numpy as np, torch, torch.distributed as dist
sys.path.insert(0, ROOT)
from tests.test_gpu_tiles import _cases
from spmm_amd import distributed
from spmm_amd.sparse import csr_matrix
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
assert dist.get_backend() == "nccl"
cases = {c[0]: c for c in _cases()}
report = {}
for name in ("dense2048_f64", "sparse8192_f64"):
    _, A, B, alpha = cases[name]
    dA = csr_matrix(A, device=dev)
    for pipe in (True, False, "late"):   # late: the values after the symbolic pass
        B_src = csr_matrix(B, device=dev)
        (r0, r1), A_blk, _ = distributed.rowblock_setup(dA, B_src.indptr, 1, 0)
        for rep in range(2):   # a second step reuses RCCL's communicator and buffers
            C, Bo = distributed.rowblock_step(A_blk, B_src, 0, dev, alg=2, pipeline=bool(pipe), n_groups=3,
                                              values_first=pipe != "late")
        torch.cuda.synchronize()
        last = distributed.rowblock_step.last
        from spmm_amd import cusparse
        info = cusparse.plan_info(A_blk, B_src, alg=2)
        vt = -(-info["tiles_per_row"] // info["record_group"])   # value tiles (record groups)
        key = pipe if pipe == "late" else int(pipe)
        report[f"{name}_{key}"] = {"pipelined": bool(last.pipelined), "groups": len(last.groups),
                                         "b_returned": Bo is not None, "value_tiles": vt}
        np.savez(os.path.join(OUT, f"{name}_{key}.npz"), p=C.indptr.cpu().numpy().astype(np.int64),
                 j=C.indices.cpu().numpy(), x=C.data.cpu().numpy())
    # agree_tiles on device tensors: a plan off the tile path disagrees, a tile plan agrees
    assert distributed.agree_tiles(None, dev) is False
    g = {"tile_width": 2048, "tiles": 9, "dtype": torch.float64}
    assert distributed.agree_tiles(g, dev) is True
with open(os.path.join(OUT, "report.json"), "w") as f:
    json.dump(report, f)
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bits(x):
    return x.view({4: np.uint32, 8: np.uint64, 16: np.uint64}[x.dtype.itemsize])


def test_rowblock_step_over_rccl_world1(tmp_path):
    import json
    from tests.test_gpu_tiles import _cases
    code = _CHILD.replace("ROOT", repr(ROOT)).replace("OUT", repr(str(tmp_path)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-5000:])
    report = json.loads((tmp_path / "report.json").read_text())
    cases = {c[0]: c for c in _cases()}
    for name in ("dense2048_f64", "sparse8192_f64"):
        _, A, B, _ = cases[name]
        rp, rj, rx = oracle.spgemm(A, B, keep_zeros=True, sort=True, threads=16)
        for pipe in (1, 0, "late"):
            r = report[f"{name}_{pipe}"]
            assert r["pipelined"] == bool(pipe), (name, r)
            assert r["groups"] == (min(3, r["value_tiles"]) if pipe else 0), (name, r)
            assert r["b_returned"], (name, r)   # rank 0 is the source: its B is whole
            q = np.load(tmp_path / f"{name}_{pipe}.npz")
            assert np.array_equal(q["p"], rp), (name, pipe)
            assert np.array_equal(q["j"], rj), (name, pipe)
            assert np.array_equal(_bits(q["x"]), _bits(rx)), (name, pipe)
