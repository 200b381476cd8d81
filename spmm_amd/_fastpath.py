"""The native shim path (csrc/fastpath.cpp): loaded from the prebuilt
lib/fastpath/spmm_fastpath.so, never compiled at import.  None when it is absent or when
SPG_LIB selects another build of the engine (the extension links the default one); the
ctypes path in cusparse.spgemm then runs the same C ABI."""
from __future__ import annotations

import importlib.util
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(_HERE, "lib", "fastpath", "spmm_fastpath.so")
_mod = None
_tried = False


def get():
    global _mod, _tried
    if not _tried:
        _tried = True
        if os.path.exists(PATH) and not os.environ.get("SPG_LIB") and not os.environ.get("SPG_NO_FASTPATH"):
            from . import _lib
            _lib.load()   # the engine first: the extension binds to this loaded copy (soname)
            spec = importlib.util.spec_from_file_location("spmm_fastpath", PATH)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            _mod = mod
    return _mod
