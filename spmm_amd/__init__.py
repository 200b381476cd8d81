"""spmm_amd -- MI355X-native CSR x CSR SpGEMM (drop-in for the reference's
``cupyx.cusparse.spgemm`` / ``csr_matrix.__matmul__`` hot path).

The engine is libmi355_spgemm.so (HIP, gfx950; C ABI in include/spgemm.h).  This package
holds only the host-side mirror of the reference interface: device CSR containers
(``sparse``), ``cusparse.spgemm`` and the synthetic input generator (``gen``).
"""
from . import sparse  # noqa: F401
from . import cusparse  # noqa: F401  (binds the .so lazily, on first use)
from .sparse import csr_matrix, csc_matrix, coo_matrix, isspmatrix_csr  # noqa: F401

__version__ = "0.1.0"

