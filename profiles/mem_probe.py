#!/usr/bin/env python3
"""hipMemGetInfo as torch sees it around allocations, and the harness ΔPeak sampler on the
dense-vs-sparse N=8192 density 1e-2 product (diagnostic for the free-memory sampler)."""
import torch, time, sys
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..'))
torch.cuda.init()
f0, t = torch.cuda.mem_get_info(); print("free0", f0, "total", t)
x = torch.empty(1 << 30, dtype=torch.uint8, device="cuda"); torch.cuda.synchronize()
f1, _ = torch.cuda.mem_get_info(); print("after empty 1GiB", f0 - f1)
x.fill_(1); torch.cuda.synchronize()
f2, _ = torch.cuda.mem_get_info(); print("after touch", f0 - f2)
del x; torch.cuda.empty_cache()
f3, _ = torch.cuda.mem_get_info(); print("after free", f0 - f3)
from spmm_amd import gen, profiling
from spmm_amd.sparse import csr_matrix
Ah, Bh = gen.scipy_pair(8192, 1e-2, seed=42)
A, B = csr_matrix(Ah, device="cuda"), csr_matrix(Bh, device="cuda")
r = profiling.profile_op_gpu("sp", lambda: A @ B)
print("dpeak", r.peak_vram, "lib", r.lib_peak_bytes, "torch", r.torch_peak_bytes, "ms", r.time_ms)
