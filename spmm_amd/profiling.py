"""Measurement helpers shared by the harness ports (harness/*).

Restates the reference's measurement loop:

* ``profile_op_gpu`` -- SpGEMM_alg_comparison/profiler.py:108-143 and
  dense_vs_sparseGEMM/utils.py:93-139: synchronize, start a background sampler of device
  free memory, time ``fn()`` + synchronize with ``time.perf_counter``, report
  ΔPeak = free0 - min(free) (the reference's ``live_peak_from_free``).  CuPy's fresh
  ``MemoryPool`` per op becomes ``torch.cuda.empty_cache()`` before and after, so the caching
  allocator's blocks are returned and ``mem_get_info`` sees real allocations.  The exact
  figure the library reports (workspace + C, ``spg_peak_bytes``) and torch's own peak
  counter are recorded beside it.
* ``repeat_gpu`` -- dense_vs_sparseGEMM/utils.py:144-191: optional warmup, N runs, result
  of the median-by-time run; an out-of-memory error prints ``[SKIP]`` and returns None.
* ``profile_op_cpu`` -- SpGEMM_vs_SpMV/profiler.py:94-178: run in a forked child, report
  time and ΔRSS peak through a pipe.
* ``human_bytes`` -- SpGEMM_alg_comparison/profiler.py:70-79 (1024 units).
"""
from __future__ import annotations

import gc
import json
import os
import resource
import sys
import threading
import time
from dataclasses import dataclass
from typing import Any, Callable, Optional

import numpy as np


@dataclass
class BenchResult:
    name: str
    time_ms: float
    peak_vram: Optional[int]
    peak_ram: Optional[int]
    out_shape: Optional[tuple]
    out_dtype: Optional[str]
    lib_peak_bytes: Optional[int] = None     # spg_peak_bytes of the last spgemm in fn
    torch_peak_bytes: Optional[int] = None   # torch.cuda.max_memory_allocated delta


def human_bytes(x: Optional[int]) -> str:
    if x is None:
        return "-"
    units = ["B", "KB", "MB", "GB", "TB"]
    i = 0
    val = float(x)
    while val >= 1024.0 and i < len(units) - 1:
        val /= 1024.0
        i += 1
    return f"{val:.2f} {units[i]}"


def synchronize() -> None:
    import torch
    torch.cuda.synchronize()


def _sample_gpu(stop_evt: threading.Event, out: dict, period_s: float) -> None:
    import torch
    min_free = None
    while not stop_evt.is_set():
        free, _ = torch.cuda.mem_get_info()
        if min_free is None or free < min_free:
            min_free = free
        time.sleep(period_s)
    free, _ = torch.cuda.mem_get_info()
    if min_free is None or free < min_free:
        min_free = free
    out["min_free"] = min_free


def _is_oom(e: BaseException) -> bool:
    import torch
    if isinstance(e, (torch.cuda.OutOfMemoryError, MemoryError)):
        return True
    from ._lib import STATUS_ALLOC_FAILED, SpgError
    if isinstance(e, SpgError) and e.status == STATUS_ALLOC_FAILED:
        return True
    return isinstance(e, RuntimeError) and "out of memory" in str(e).lower()


def cleanup_gpu() -> None:
    """Best-effort cleanup after a failure (dense_vs_sparseGEMM/utils.py:17-28)."""
    import torch
    try:
        synchronize()
    except Exception:
        pass
    gc.collect()
    torch.cuda.empty_cache()


def profile_op_gpu(name: str, fn: Callable[[], Any], period_s: float = 1e-4) -> BenchResult:
    import torch
    from . import cusparse
    synchronize()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()
    base_alloc = torch.cuda.memory_allocated()
    free0, _ = torch.cuda.mem_get_info()
    stats: dict = {}
    stop = threading.Event()
    th = threading.Thread(target=_sample_gpu, args=(stop, stats, period_s), daemon=True)
    th.start()
    cusparse.last_stats.peak_bytes = 0
    t0 = time.perf_counter()
    try:
        out = fn()
        synchronize()
    finally:
        t1 = time.perf_counter()
        stop.set()
        th.join()
    torch_peak = torch.cuda.max_memory_allocated() - base_alloc
    res = BenchResult(
        name=name, time_ms=(t1 - t0) * 1e3,
        peak_vram=int(free0 - stats["min_free"]) if "min_free" in stats else None,
        peak_ram=None, out_shape=getattr(out, "shape", None),
        out_dtype=str(getattr(out, "dtype", "")) if hasattr(out, "dtype") else None,
        lib_peak_bytes=cusparse.last_stats.peak_bytes or None, torch_peak_bytes=int(torch_peak))
    del out
    torch.cuda.empty_cache()
    return res


def repeat_gpu(name: str, fn: Callable[[], Any], runs: int, do_warmup: bool = True) -> Optional[BenchResult]:
    """Median-by-time of `runs` runs; None (after printing [SKIP]) on out-of-memory."""
    if do_warmup:
        try:
            profile_op_gpu(name + " [warmup]", fn)
        except Exception as e:   # noqa: BLE001 -- mirror the reference's SKIP on OOM
            if not _is_oom(e):
                raise
            print(f"[SKIP] {name}: warmup failed ({type(e).__name__}: {e})")
            cleanup_gpu()
            return None
    results = []
    for i in range(runs):
        try:
            results.append(profile_op_gpu(name, fn))
        except Exception as e:   # noqa: BLE001
            if not _is_oom(e):
                raise
            print(f"[SKIP] {name}: run {i + 1}/{runs} failed ({type(e).__name__}: {e})")
            cleanup_gpu()
            return None
    times = np.asarray([r.time_ms for r in results])
    return results[int(np.argsort(times)[runs // 2])]


def _rss_bytes() -> int:
    with open("/proc/self/statm") as f:
        return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")


def _ru_maxrss_bytes() -> int:
    ru = resource.getrusage(resource.RUSAGE_SELF)
    return ru.ru_maxrss * (1024 if sys.platform != "darwin" else 1)


def profile_op_cpu(name: str, func: Callable[[], Any]) -> BenchResult:
    """Time `func` in a fresh forked child; ΔRSS peak (SpGEMM_vs_SpMV/profiler.py:116-178)."""
    r_fd, w_fd = os.pipe()
    pid = os.fork()
    if pid == 0:
        try:
            os.close(r_fd)
            gc.collect()
            rss0 = _rss_bytes()
            t0 = time.perf_counter()
            out = func()
            t1 = time.perf_counter()
            payload = {"time_ms": (t1 - t0) * 1e3, "rss_peak_delta": _ru_maxrss_bytes() - rss0,
                       "out_shape": list(getattr(out, "shape", ()) or ()),
                       "out_dtype": str(getattr(out, "dtype", ""))}
            os.write(w_fd, json.dumps(payload).encode())
        except Exception as e:   # noqa: BLE001
            os.write(w_fd, json.dumps({"error": repr(e)}).encode())
        finally:
            os.close(w_fd)
            os._exit(0)
    os.close(w_fd)
    chunks = []
    while True:
        b = os.read(r_fd, 65536)
        if not b:
            break
        chunks.append(b)
    os.close(r_fd)
    os.waitpid(pid, 0)
    data = json.loads(b"".join(chunks).decode() or "{}")
    if "error" in data:
        raise RuntimeError(f"Child error: {data['error']}")
    return BenchResult(name=name, time_ms=data.get("time_ms", 0.0), peak_vram=None,
                       peak_ram=data.get("rss_peak_delta"),
                       out_shape=tuple(data.get("out_shape") or ()) or None,
                       out_dtype=data.get("out_dtype"))


def repeat_cpu(name: str, fn: Callable[[], Any], runs: int) -> BenchResult:
    results = [profile_op_cpu(name, fn) for _ in range(runs)]
    times = np.asarray([r.time_ms for r in results])
    return results[int(np.argsort(times)[runs // 2])]
