"""Overlap probe (round 6): can config 4's symbolic pass run under its numeric pass?

Two handles on two HIP streams, two plans of the same config-4 product.  Times (HIP events /
host clock around a full sync): plan 1's numeric pass alone, plan 2's symbolic pass alone, and
both issued together (numeric on stream 1, then the symbolic on stream 2 while it runs).  If the
together time is well under the sum, a chunked schedule that runs chunk c+1's symbolic under
chunk c's numeric pays.  usage: SPG_LIB=... python abtest/overlap_probe.py [N] [density]"""
import ctypes
import sys
import time

import torch

sys.path.insert(0, ".")
from spmm_amd import _lib, gen  # noqa: E402
from spmm_amd._lib import SpgCsr, check  # noqa: E402
from spmm_amd.cusparse import _IT, _VT, _csr_view  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dens = float(sys.argv[2]) if len(sys.argv) > 2 else 5e-3
dev = torch.device("cuda:0")
A = gen.random_csr(n, n, dens, seed=0, dtype=torch.float64, device=dev)
B = gen.random_csr(n, n, dens, seed=1, dtype=torch.float64, device=dev)
lib = _lib.load()
va, vb = _csr_view(A), _csr_view(B)
streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
hs, plans, wss, cs = [], [], [], []
for s in streams:
    h = _lib.Handle(0)
    h.set_stream(s.cuda_stream)
    hs.append(h)


def new_plan(i):
    h, s = hs[i], streams[i]
    wsb = ctypes.c_size_t(0)
    check(lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), _lib.SPG_ALG3, ctypes.c_float(0.2), ctypes.byref(wsb), None, None))
    with torch.cuda.stream(s):
        ws = torch.empty(wsb.value, dtype=torch.uint8, device=dev)
    p = ctypes.c_void_p()
    check(lib.spg_plan(h.ptr, ctypes.byref(va), ctypes.byref(vb), _lib.SPG_ALG3, ctypes.c_float(0.2), ctypes.byref(wsb),
                       ctypes.c_void_p(ws.data_ptr()), ctypes.byref(p)))
    wss.append(ws)
    return p


plans = [new_plan(0), new_plan(1)]
one = ctypes.c_double(1.0)


def symbolic(i, fresh=False):
    if fresh:   # (a plan's repeated symbolic call reuses its counts: a new plan each time)
        plans[i] = new_plan(i)
        torch.cuda.synchronize()
    indptr = torch.empty(n + 1, dtype=torch.int64, device=dev)
    nnz = ctypes.c_int64(0)
    check(lib.spg_symbolic(hs[i].ptr, plans[i], ctypes.c_void_p(indptr.data_ptr()), _IT[torch.int64],
                           ctypes.byref(nnz)), "spg_symbolic")
    return indptr, int(nnz.value)


# plan 1: symbolic once, C allocated; plan 2 symbolic warm-up
ip1, nnz1 = symbolic(0)
with torch.cuda.stream(streams[0]):
    cj = torch.empty(nnz1, dtype=torch.int32, device=dev)
    cx = torch.empty(nnz1, dtype=torch.float64, device=dev)
vc = SpgCsr(n, n, nnz1, ip1.data_ptr(), cj.data_ptr(), cx.data_ptr(), _IT[torch.int64], _VT[torch.float64])
symbolic(1)


def numeric():
    check(lib.spg_numeric(hs[0].ptr, plans[0], ctypes.byref(one), ctypes.byref(vc)), "spg_numeric")


def timed(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best * 1e3


numeric()
t_num = timed(numeric)
def sym_only():
    plans[1] = new_plan(1)
    torch.cuda.synchronize()
    t = time.perf_counter()
    symbolic(1)
    torch.cuda.synchronize()
    return time.perf_counter() - t


t_sym = min(sym_only() for _ in range(3)) * 1e3


def both():
    plans[1] = new_plan(1)
    torch.cuda.synchronize()
    t = time.perf_counter()
    numeric()
    symbolic(1)
    torch.cuda.synchronize()
    return time.perf_counter() - t


t_both = min(both() for _ in range(3)) * 1e3
print(f"N={n} density={dens}: numeric {t_num:.3f} ms, symbolic {t_sym:.3f} ms, "
      f"sum {t_num + t_sym:.3f} ms, together {t_both:.3f} ms, hidden {t_num + t_sym - t_both:.3f} ms")
for p in plans:
    lib.spg_plan_destroy(p)
