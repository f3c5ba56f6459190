"""ctypes binding of libslat.so (include/slat.h). The HIP engine is the only compute path: if the
library cannot be loaded, importing the GPU entry points raises — there is no CPU fallback."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# SLAT_LIB_PATH: load another build of the same library (kernel experiments); default in-tree
LIB_PATH = os.environ.get("SLAT_LIB_PATH") or os.path.join(PKG_DIR, "libslat.so")

SLAT_OK, SLAT_EINVAL, SLAT_EDIM, SLAT_EOOM, SLAT_EHIP, SLAT_ENOTSUP, SLAT_ENODEV = range(7)
U32, SAT64, F64 = 0, 1, 2
DEVICE, HOST = 0, 1
FLAG_TIMING, FLAG_EXACT_ALLOC, FLAG_STATS, FLAG_F64_ANY_ORDER, FLAG_IDX64, FLAG_NO_TINY = 0x1, 0x2, 0x4, 0x8, 0x10, 0x20
FLAG_FAT_BUCKETS = 0x40  # fat rows: products bucketed by accumulator chunk (MAGNUS fine-level reordering)

# Every symbol include/slat.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "slat_ctx_create", "slat_ctx_destroy", "slat_ctx_set_stream", "slat_ctx_stream", "slat_status_string",
    "slat_last_error", "slat_get_stats", "slat_sync", "slat_set_matmul_progress", "slat_csr_create", "slat_csr_to_host", "slat_csr_free",
    "slat_csr_view_of", "slat_csr_max_row_nnz", "slat_spgemm", "slat_spgemm_csr_u32", "slat_spgemm_csr_sat64",
    "slat_spgemm_csr_f64", "slat_spgemm_rowblock", "slat_rng_seed", "slat_rng_next_u64", "slat_rng_next_f64",
    "slat_rng_next_u32", "slat_rng_range_u32", "slat_host_random",
    "slat_host_from_coo", "slat_host_lattice", "slat_host_thin", "slat_host_rmat", "slat_host_csr_free",
    "slat_csr_add", "slat_csr_identity", "slat_csr_pattern_equal", "slat_reachability_sum",
    "slat_power_until_stable", "slat_connected_components", "slat_csr_from_coo", "slat_csr_lattice", "slat_csr_thin",
    "slat_load_edges", "slat_edges_free", "slat_csr_from_edges", "slat_rcm_order", "slat_csr_permute",
    "slat_bandwidth_stats", "slat_spgemm_dense", "slat_device_alloc", "slat_device_free", "slat_device_copy",
    "slat_magnus_matmul", "slat_magnus_free", "slat_magnus_to_host", "slat_magnus_view_of",
    "slat_magnus_add", "slat_magnus_reachability_sum", "slat_magnus_power_until_stable",
    "slat_magnus_connected_components",
    "slat_comm_id", "slat_comm_create", "slat_comm_destroy", "slat_rowblock_cuts", "slat_bcast_csr",
    "slat_allgather_rows", "slat_concat_rows", "slat_diameter", "slat_spgemm_btree", "slat_host_alloc",
    "slat_host_free", "slat_bprep_create", "slat_bprep_free", "slat_spgemm_rowblock_prepared",
]


class SlatError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"slat status {status}: {msg}")
        self.status = status


class CsrView(C.Structure):
    _fields_ = [("n_rows", C.c_uint64), ("n_cols", C.c_uint64), ("nnz", C.c_uint64), ("row_ptr", C.c_void_p),
                ("col_idx", C.c_void_p), ("values", C.c_void_p), ("dtype", C.c_int32), ("residency", C.c_int32),
                ("max_row_nnz", C.c_uint64)]


class CsrOwned(C.Structure):
    _fields_ = [("n_rows", C.c_uint64), ("n_cols", C.c_uint64), ("nnz", C.c_uint64), ("capacity", C.c_uint64),
                ("max_row_nnz", C.c_uint64), ("row_ptr", C.c_void_p), ("col_idx", C.c_void_p),
                ("values", C.c_void_p), ("dtype", C.c_int32), ("device", C.c_int32), ("alloc", C.c_int32),
                ("_pad", C.c_int32)]


class MagnusView(C.Structure):
    _fields_ = [("n_rows", C.c_uint64), ("n_cols", C.c_uint64), ("nnz", C.c_uint64), ("row_ptr", C.c_void_p),
                ("col_idx", C.c_void_p), ("values", C.c_void_p), ("residency", C.c_int32), ("_pad", C.c_int32),
                ("max_row_nnz", C.c_uint64)]


class MagnusOwned(C.Structure):
    _fields_ = [("n_rows", C.c_uint64), ("n_cols", C.c_uint64), ("nnz", C.c_uint64), ("capacity", C.c_uint64),
                ("max_row_nnz", C.c_uint64), ("row_ptr", C.c_void_p), ("col_idx", C.c_void_p),
                ("values", C.c_void_p), ("device", C.c_int32), ("_pad", C.c_int32), ("_owner", C.c_uint8 * 96)]


class BTreeView(C.Structure):
    _fields_ = [("n_rows", C.c_uint64), ("n_cols", C.c_uint64), ("nnz", C.c_uint64), ("n_nodes", C.c_uint64),
                ("data_start", C.c_void_p), ("data_off", C.c_void_p), ("nodes", C.c_void_p), ("values", C.c_void_p),
                ("residency", C.c_int32), ("_pad", C.c_int32), ("max_row_nnz", C.c_uint64)]


class Stats(C.Structure):
    _fields_ = [("nnz", C.c_uint64), ("flops", C.c_uint64), ("capacity", C.c_uint64), ("symbolic_ms", C.c_double),
                ("scan_ms", C.c_double), ("numeric_ms", C.c_double), ("compact_ms", C.c_double),
                ("total_ms", C.c_double), ("mode", C.c_uint32), ("window_words", C.c_uint32),
                ("exact_alloc", C.c_uint32), ("dropped_rows", C.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class HostCsr(C.Structure):
    _fields_ = [("n", C.c_uint64), ("nnz", C.c_uint64), ("row_ptr", C.c_void_p), ("col_idx", C.c_void_p),
                ("values", C.c_void_p), ("dtype", C.c_int32), ("_pad", C.c_int32)]


class RngState(C.Structure):
    _fields_ = [("opaque", C.c_uint8 * 512)]


def build() -> str:
    """Compile libslat.so in-tree (hipcc, gfx950)."""
    subprocess.run(["make", "-s", "-C", PKG_DIR], check=True)
    return LIB_PATH


_lib = None


def lib():
    """Load libslat.so (raises OSError if it has not been built: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} not built; run `make -C {PKG_DIR}` or __graft_entry__.build()")
    L = C.CDLL(LIB_PATH)
    P, vp, u64, i32, u32 = C.POINTER, C.c_void_p, C.c_uint64, C.c_int32, C.c_uint32
    sig = {
        "slat_ctx_create": ([C.c_int, P(vp)], C.c_int),
        "slat_ctx_destroy": ([vp], C.c_int),
        "slat_ctx_set_stream": ([vp, vp], C.c_int),
        "slat_ctx_stream": ([vp], vp),
        "slat_status_string": ([C.c_int], C.c_char_p),
        "slat_last_error": ([vp], C.c_char_p),
        "slat_get_stats": ([vp, P(Stats)], C.c_int),
        "slat_set_matmul_progress": ([C.c_int], C.c_int),
        "slat_sync": ([vp], C.c_int),
        "slat_csr_create": ([vp, P(CsrView), P(CsrOwned)], C.c_int),
        "slat_csr_to_host": ([vp, P(CsrView), vp, vp, vp], C.c_int),
        "slat_csr_free": ([vp, P(CsrOwned)], C.c_int),
        "slat_csr_view_of": ([P(CsrOwned)], CsrView),
        "slat_csr_max_row_nnz": ([vp, P(CsrView), P(u64)], C.c_int),
        "slat_spgemm": ([vp, P(CsrView), P(CsrView), P(CsrOwned), u32], C.c_int),
        "slat_spgemm_csr_u32": ([vp, P(CsrView), P(CsrView), P(CsrOwned), u32], C.c_int),
        "slat_spgemm_csr_sat64": ([vp, P(CsrView), P(CsrView), P(CsrOwned), u32], C.c_int),
        "slat_spgemm_csr_f64": ([vp, P(CsrView), P(CsrView), P(CsrOwned), u32], C.c_int),
        "slat_spgemm_rowblock": ([vp, P(CsrView), u64, u64, P(CsrView), P(CsrOwned), u32], C.c_int),
        "slat_rng_seed": ([P(RngState), C.c_char_p], None),
        "slat_rng_next_u64": ([P(RngState)], u64),
        "slat_rng_next_f64": ([P(RngState)], C.c_double),
        "slat_rng_next_u32": ([P(RngState)], u32),
        "slat_rng_range_u32": ([P(RngState), u32, u32], u32),
        "slat_host_random": ([P(RngState), u32, u64, P(HostCsr)], C.c_int),
        "slat_host_from_coo": ([u64, u64, vp, vp, vp, i32, P(HostCsr)], C.c_int),
        "slat_host_lattice": ([P(u64), C.c_int, C.c_int, P(HostCsr)], C.c_int),
        "slat_host_thin": ([P(HostCsr), P(RngState), C.c_double, P(HostCsr)], C.c_int),
        "slat_host_rmat": ([u32, u64, C.c_double, C.c_double, C.c_double, C.c_char_p, P(HostCsr)], C.c_int),
        "slat_host_csr_free": ([P(HostCsr)], None),
        "slat_csr_add": ([vp, P(CsrView), P(CsrView), P(CsrOwned)], C.c_int),
        "slat_csr_identity": ([vp, u64, i32, P(CsrOwned)], C.c_int),
        "slat_csr_pattern_equal": ([vp, P(CsrView), P(CsrView), P(i32)], C.c_int),
        "slat_reachability_sum": ([vp, P(CsrView), P(CsrOwned), P(u64)], C.c_int),
        "slat_power_until_stable": ([vp, P(CsrView), P(CsrOwned), P(u64)], C.c_int),
        "slat_connected_components": ([vp, P(CsrView), vp], C.c_int),
        "slat_csr_from_coo": ([vp, u64, u64, vp, vp, vp, i32, i32, P(CsrOwned)], C.c_int),
        "slat_csr_lattice": ([vp, P(u64), C.c_int, C.c_int, P(CsrOwned)], C.c_int),
        "slat_csr_thin": ([vp, P(CsrView), P(RngState), C.c_double, P(CsrOwned)], C.c_int),
        "slat_load_edges": ([C.c_char_p, P(u64), P(u64), P(vp), P(vp)], C.c_int),
        "slat_edges_free": ([vp, vp], None),
        "slat_csr_from_edges": ([vp, u64, u64, vp, vp, i32, i32, P(CsrOwned)], C.c_int),
        "slat_rcm_order": ([vp, P(CsrView), vp], C.c_int),
        "slat_csr_permute": ([vp, P(CsrView), vp, i32, P(CsrOwned)], C.c_int),
        "slat_bandwidth_stats": ([vp, P(CsrView), P(u64), P(C.c_double)], C.c_int),
        "slat_spgemm_dense": ([vp, P(CsrView), P(CsrView), vp, u64, i32, i32], C.c_int),
        "slat_device_alloc": ([vp, u64, P(vp)], C.c_int),
        "slat_device_free": ([vp, vp], C.c_int),
        "slat_device_copy": ([vp, vp, vp, u64, i32], C.c_int),
        "slat_magnus_matmul": ([vp, P(MagnusView), P(MagnusView), P(MagnusOwned), u32], C.c_int),
        "slat_magnus_free": ([vp, P(MagnusOwned)], C.c_int),
        "slat_magnus_to_host": ([vp, P(MagnusOwned), vp, vp, vp], C.c_int),
        "slat_magnus_view_of": ([P(MagnusOwned)], MagnusView),
        "slat_magnus_add": ([vp, P(MagnusView), P(MagnusView), P(MagnusOwned)], C.c_int),
        "slat_magnus_reachability_sum": ([vp, P(MagnusView), P(MagnusOwned), P(C.c_uint64)], C.c_int),
        "slat_magnus_power_until_stable": ([vp, P(MagnusView), P(MagnusOwned), P(C.c_uint64)], C.c_int),
        "slat_magnus_connected_components": ([vp, P(MagnusView), vp], C.c_int),
        "slat_comm_id": ([vp], C.c_int),
        "slat_comm_create": ([vp, C.c_int, C.c_int, vp, P(vp)], C.c_int),
        "slat_comm_destroy": ([vp], C.c_int),
        "slat_rowblock_cuts": ([vp, P(CsrView), P(CsrView), u32, vp], C.c_int),
        "slat_bcast_csr": ([vp, vp, P(CsrOwned), C.c_int], C.c_int),
        "slat_allgather_rows": ([vp, vp, P(CsrView), P(CsrOwned)], C.c_int),
        "slat_concat_rows": ([vp, P(CsrView), C.c_uint32, P(CsrOwned)], C.c_int),
        "slat_diameter": ([vp, P(CsrView), P(u64), P(u64), P(u64)], C.c_int),
        "slat_spgemm_btree": ([vp, P(BTreeView), P(BTreeView), P(CsrOwned), u32], C.c_int),
        "slat_host_alloc": ([u64, P(vp)], C.c_int),
        "slat_host_free": ([vp], C.c_int),
        "slat_bprep_create": ([vp, P(CsrView), P(vp)], C.c_int),
        "slat_bprep_free": ([vp, vp], C.c_int),
        "slat_spgemm_rowblock_prepared": ([vp, P(CsrView), u64, u64, vp, P(CsrOwned), u32], C.c_int),
    }
    for name, (args, res) in sig.items():
        if os.environ.get("SLAT_LIB_PATH") and not hasattr(L, name):
            continue  # an older variant build (A/B against a previous round's library)
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(status: int, ctx=None):
    if status != SLAT_OK:
        L = lib()
        msg = L.slat_status_string(status).decode()
        if ctx:
            detail = L.slat_last_error(ctx)
            if detail:
                msg += f" ({detail.decode()})"
        raise SlatError(status, msg)
