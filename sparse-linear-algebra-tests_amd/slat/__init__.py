"""slat — MI355X-native SpGEMM engine (Python host mirror over libslat.so's C ABI).

Drop-in for the reference's SpGEMM path (imlvts/sparse-linear-algebra-tests):
CsrMatrix.matmul / matmul_par (src/graph_csr.rs:306-484), MagnusMatrix.matmul / matmul_seq
(src/graph_magnus.rs:224-242), linalg Csr.matmul / matmul_par (linalg/src/csr.rs:308-466).
"""
from ._lib import (DEVICE, F64, FLAG_EXACT_ALLOC, FLAG_F64_ANY_ORDER, FLAG_FAT_BUCKETS, FLAG_IDX64, FLAG_NO_TINY, FLAG_STATS, FLAG_TIMING, HOST, SAT64, U32, SlatError, build,
                   lib)
from .matrix import (Context, Csr, CsrBTreeMatrix, CsrF64, CsrMatrix, CsrU32, CsrU64, DeviceCsr, HostCsr, MagnusMatrix, MagnusMatrixUsize, PreparedB, StdRng,
                     default_context, host_from_coo, host_lattice, host_random, host_rmat, host_thin, load_edges, pinned_empty, spgemm_host,
                     torus_thinned, torus_thinned_device)

__all__ = [
    "Context", "Csr", "CsrBTreeMatrix", "CsrF64", "CsrMatrix", "CsrU32", "CsrU64", "DeviceCsr", "HostCsr", "MagnusMatrix", "MagnusMatrixUsize", "PreparedB", "StdRng",
    "default_context", "host_from_coo", "host_lattice", "host_random", "host_rmat", "host_thin", "load_edges", "pinned_empty", "spgemm_host", "torus_thinned", "torus_thinned_device", "SlatError",
    "build", "lib", "U32", "SAT64", "F64", "DEVICE", "HOST", "FLAG_TIMING", "FLAG_EXACT_ALLOC", "FLAG_STATS", "FLAG_F64_ANY_ORDER", "FLAG_IDX64", "FLAG_NO_TINY", "FLAG_FAT_BUCKETS",
    "set_matmul_progress",
]


def set_matmul_progress(on: bool = True) -> bool:
    """MATMUL_PROGRESS.store(on) (src/graph_csr.rs:10-11): every SpGEMM call then prints the
    reference's symbolic / numeric pass summaries to stderr. Returns the previous setting."""
    return bool(lib().slat_set_matmul_progress(1 if on else 0))
