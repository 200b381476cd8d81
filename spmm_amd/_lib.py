"""ctypes binding of libmi355_spgemm.so (include/spgemm.h).

Plays the role of the reference's Cython layer
(modify_src/cupy-src/cupy_backends/cuda/libs/cusparse.pyx:5063-5152, status handling
:1526-1547): thin wrappers that turn a non-zero status into an exception.

The library is loaded after ``torch`` so that it binds to the HIP runtime torch already
loaded (same SONAME, libamdhip64.so.7) and device pointers from torch's allocator are
valid in it.  There is no CPU fallback: if the library is missing the import of the
product path fails loudly.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be loaded before the HIP library, see module doc)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPG_LIB") or os.path.join(_HERE, "lib", "libmi355_spgemm.so")   # SPG_LIB: an alternative build (A/B timing)

# enums of include/spgemm.h
SPG_INDEX_32I = 32
SPG_INDEX_64I = 64
SPG_R_32F = 0
SPG_R_64F = 1
SPG_C_32F = 4
SPG_C_64F = 5
SPG_ALG_DEFAULT, SPG_ALG1, SPG_ALG2, SPG_ALG3 = 0, 1, 2, 3

STATUS_NAMES = {
    0: "SPG_STATUS_SUCCESS", 1: "SPG_STATUS_NOT_INITIALIZED", 2: "SPG_STATUS_ALLOC_FAILED",
    3: "SPG_STATUS_INVALID_VALUE", 4: "SPG_STATUS_ARCH_MISMATCH",
    6: "SPG_STATUS_EXECUTION_FAILED", 7: "SPG_STATUS_INTERNAL_ERROR",
    10: "SPG_STATUS_NOT_SUPPORTED", 11: "SPG_STATUS_INSUFFICIENT_RESOURCES",
    100: "SPG_STATUS_OVERFLOW", 101: "SPG_STATUS_HIP_ERROR",
}
STATUS_ALLOC_FAILED = 2
STATUS_OVERFLOW = 100
STATUS_NOT_SUPPORTED = 10

# every symbol include/spgemm.h declares (tests/test_abi.py checks the .so exports them)
EXPORTS = ("spg_version", "spg_build_info", "spg_status_string", "spg_create", "spg_destroy", "spg_set_stream",
           "spg_last_hip_error", "spg_plan", "spg_num_products", "spg_symbolic",
           "spg_numeric", "spg_peak_bytes", "spg_validate_csr", "spg_plan_destroy",
           "spg_set_timing", "spg_get_timing", "spg_result_in_workspace", "spg_spmv",
           "spg_spgemm_ws", "spg_plan_info", "spg_tile_value_offsets", "spg_tile_values",
           "spg_numeric_tiles", "spg_cols16_split", "spg_cols16_join")

PHASES = ("products", "scan", "symbolic", "numeric", "compact", "validate", "spill", "spmv", "b_layout")
NUM_PHASES = 9


class SpgCsr(ctypes.Structure):
    """spg_csr_t"""
    _fields_ = [("rows", ctypes.c_int64), ("cols", ctypes.c_int64), ("nnz", ctypes.c_int64),
                ("indptr", ctypes.c_void_p), ("indices", ctypes.c_void_p),
                ("values", ctypes.c_void_p), ("indptr_type", ctypes.c_int),
                ("value_type", ctypes.c_int)]


class SpgPlanInfo(ctypes.Structure):
    """spg_plan_info_t"""
    _fields_ = [("path", ctypes.c_int), ("tile_width", ctypes.c_int), ("tiles_per_row", ctypes.c_int64),
                ("dense_tiles", ctypes.c_int), ("n_chunks", ctypes.c_int64), ("lds_ordered", ctypes.c_int),
                ("record_group", ctypes.c_int)]


class SpgTiming(ctypes.Structure):
    """spg_timing_t"""
    _fields_ = [("ms", ctypes.c_double * NUM_PHASES), ("launches", ctypes.c_int64 * NUM_PHASES)]


class SpgError(RuntimeError):
    """Non-zero spg_status_t (the analogue of CuPy's CuSparseError)."""

    def __init__(self, status: int, where: str = ""):
        self.status = int(status)
        name = STATUS_NAMES.get(self.status, f"SPG_STATUS_{self.status}")
        super().__init__(f"{where}: {name}" if where else name)


_lib = None
_lock = threading.Lock()


def load():
    """Load and prototype the library once.  Raises RuntimeError if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c \"import __graft_entry__ as g; "
                f"g.build()\"` (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(LIB_PATH)
        vp, i64, sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_size_t
        csrp = ctypes.POINTER(SpgCsr)
        proto = {
            "spg_version": (ctypes.c_int, []),
            "spg_build_info": (ctypes.c_char_p, []),
            "spg_status_string": (ctypes.c_char_p, [ctypes.c_int]),
            "spg_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int]),
            "spg_destroy": (ctypes.c_int, [vp]),
            "spg_set_stream": (ctypes.c_int, [vp, vp]),
            "spg_last_hip_error": (ctypes.c_int, [vp]),
            "spg_plan": (ctypes.c_int, [vp, csrp, csrp, ctypes.c_int, ctypes.c_float,
                                        ctypes.POINTER(sz), vp, ctypes.POINTER(vp)]),
            "spg_num_products": (ctypes.c_int, [vp, vp, ctypes.POINTER(i64)]),
            "spg_result_in_workspace": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]),
            "spg_spmv": (ctypes.c_int, [vp, csrp, vp, vp, vp, vp]),
            "spg_symbolic": (ctypes.c_int, [vp, vp, vp, ctypes.c_int, ctypes.POINTER(i64)]),
            "spg_numeric": (ctypes.c_int, [vp, vp, vp, csrp]),
            "spg_peak_bytes": (ctypes.c_int, [vp, ctypes.POINTER(sz)]),
            "spg_validate_csr": (ctypes.c_int, [vp, csrp, ctypes.POINTER(ctypes.c_int)]),
            "spg_plan_destroy": (ctypes.c_int, [vp]),
            "spg_plan_info": (ctypes.c_int, [vp, ctypes.POINTER(SpgPlanInfo), ctypes.POINTER(i64), i64]),
            "spg_spgemm_ws": (ctypes.c_int, [vp, csrp, csrp, ctypes.c_int, ctypes.c_float, vp, vp, sz, vp,
                                             ctypes.c_int, ctypes.POINTER(i64), ctypes.POINTER(vp),
                                             ctypes.POINTER(vp), ctypes.POINTER(sz), ctypes.POINTER(vp)]),
            "spg_tile_value_offsets": (ctypes.c_int, [vp, vp, ctypes.POINTER(i64), i64]),
            "spg_tile_values": (ctypes.c_int, [vp, vp, vp]),
            "spg_numeric_tiles": (ctypes.c_int, [vp, vp, vp, csrp, vp, i64, i64]),
            "spg_cols16_split": (ctypes.c_int, [vp, csrp, vp, vp]),
            "spg_cols16_join": (ctypes.c_int, [vp, csrp, vp, vp]),
            "spg_set_timing": (ctypes.c_int, [vp, ctypes.c_int]),
            "spg_get_timing": (ctypes.c_int, [vp, ctypes.POINTER(SpgTiming)]),
        }
        for name, (res, args) in proto.items():
            fn = getattr(lib, name, None)
            if fn is None:
                if os.environ.get("SPG_LIB"):   # (an older development build: A/B timing only)
                    continue
                raise RuntimeError(f"{LIB_PATH} does not export {name}: rebuild it")
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


_build_id = None


def build_id() -> str:
    """First 16 hex digits of the SHA-256 of the library file in use: stamps measurements
    (PMC traffic summaries) so a number collected on another build is not reused."""
    global _build_id
    if _build_id is None:
        import hashlib
        with open(LIB_PATH, "rb") as f:
            _build_id = hashlib.sha256(f.read()).hexdigest()[:16]
    return _build_id


_source_id = None


def source_id() -> str:
    """The source id compiled INTO the loaded library (spg_build_info; spmm_amd/source_id.py:
    a hash of the sources and the effective HIPFLAGS it was built from).  hipcc's output is
    not byte-identical from one build to the next, so a rebuild of the same sources changes
    build_id() but not this; an A/B build (SPG_LIB), a stale .so or a HIPFLAGS variant
    reports its own id.  Measurements carry both."""
    global _source_id
    if _source_id is None:
        info = (load().spg_build_info() or b"").decode()
        sid = dict(kv.split("=", 1) for kv in info.split() if "=" in kv).get("source_id", "unknown")
        _source_id = sid
    return _source_id


def check(status: int, where: str = "") -> None:
    if status != 0:
        raise SpgError(status, where)


class Handle:
    """spg_handle_t bound to one device (one per host thread per device, like CuPy's
    thread-local cuSPARSE handles, cupy-src/cupy/cuda/device.pyx:228-243)."""

    def __init__(self, device: int):
        self.lib = load()
        self.device = device
        h = ctypes.c_void_p()
        check(self.lib.spg_create(ctypes.byref(h), device), "spg_create")
        self.ptr = h

    def set_stream(self, stream_ptr: int) -> None:
        if stream_ptr == getattr(self, "_stream", None):
            return
        check(self.lib.spg_set_stream(self.ptr, ctypes.c_void_p(stream_ptr)), "spg_set_stream")
        self._stream = stream_ptr

    def set_timing(self, enable: bool) -> None:
        check(self.lib.spg_set_timing(self.ptr, int(enable)), "spg_set_timing")

    def get_timing(self) -> dict:
        """{phase: (total device ms, launches)} accumulated since set_timing(True)."""
        t = SpgTiming()
        check(self.lib.spg_get_timing(self.ptr, ctypes.byref(t)), "spg_get_timing")
        return {name: (t.ms[i], int(t.launches[i])) for i, name in enumerate(PHASES)}

    def __del__(self):
        try:
            if getattr(self, "ptr", None):
                self.lib.spg_destroy(self.ptr)
        except Exception:
            pass


_tls = threading.local()


def get_handle(device: int) -> Handle:
    hs = getattr(_tls, "handles", None)
    if hs is None:
        hs = _tls.handles = {}
    h = hs.get(device)
    if h is None:
        h = hs[device] = Handle(device)
    return h
