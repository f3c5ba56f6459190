"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference SpGEMM path (see oracle.h for the reference file:line
map). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product (sparse-linear-algebra-tests_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

U32, SAT64, F64 = 0, 1, 2
_VDT = {U32: np.uint32, SAT64: np.uint64, F64: np.float64}


class _Csr(C.Structure):
    _fields_ = [("n", C.c_uint64), ("nnz", C.c_uint64), ("dtype", C.c_int32), ("_pad", C.c_int32),
                ("row_ptr", C.c_void_p), ("col", C.c_void_p), ("val", C.c_void_p)]


class _Rng(C.Structure):
    _fields_ = [("key", C.c_uint32 * 8), ("counter", C.c_uint64), ("buf", C.c_uint32 * 64),
                ("idx", C.c_uint32)]


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.POINTER
        L.orc_rng_seed.argtypes = [P(_Rng), C.c_char_p]
        L.orc_rng_next_u64.argtypes = [P(_Rng)]
        L.orc_rng_next_u64.restype = C.c_uint64
        L.orc_rng_next_f64.argtypes = [P(_Rng)]
        L.orc_rng_next_f64.restype = C.c_double
        L.orc_rng_next_u32.argtypes = [P(_Rng)]
        L.orc_rng_next_u32.restype = C.c_uint32
        L.orc_rng_range_u32.argtypes = [P(_Rng), C.c_uint32, C.c_uint32]
        L.orc_rng_range_u32.restype = C.c_uint32
        L.orc_random.argtypes = [P(_Rng), C.c_uint32, C.c_uint64, P(_Csr)]
        L.orc_chacha12_block.argtypes = [P(C.c_uint32), C.c_uint64, P(C.c_uint32)]
        L.orc_chacha_block.argtypes = [P(C.c_uint32), C.c_uint64, C.c_int, P(C.c_uint32)]
        L.orc_csr_free.argtypes = [P(_Csr)]
        L.orc_from_coo.argtypes = [C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                   P(_Csr)]
        L.orc_lattice.argtypes = [P(C.c_uint64), C.c_int, C.c_int, P(_Csr)]
        L.orc_thin.argtypes = [P(_Csr), P(_Rng), C.c_double, P(_Csr)]
        L.orc_convert.argtypes = [P(_Csr), C.c_int, P(_Csr)]
        L.orc_matmul_seq.argtypes = [P(_Csr), P(_Csr), P(_Csr)]
        L.orc_matmul_par.argtypes = [P(_Csr), P(_Csr), C.c_int, P(_Csr)]
        L.orc_add.argtypes = [P(_Csr), P(_Csr), P(_Csr)]
        L.orc_flops.argtypes = [P(_Csr), P(_Csr)]
        L.orc_flops.restype = C.c_uint64
        L.orc_identity.argtypes = [C.c_uint64, C.c_int, P(_Csr)]
        L.orc_power_until_stable.argtypes = [P(_Csr), P(C.c_uint64), P(_Csr)]
        L.orc_reachability_sum.argtypes = [P(_Csr), P(C.c_uint64), P(_Csr)]
        L.orc_connected_components.argtypes = [P(_Csr), C.c_void_p]
        L.orc_rcm_order.argtypes = [P(_Csr), C.c_void_p]
        L.orc_einsum_sparse_driven.argtypes = [P(_Csr), P(_Csr), C.c_void_p, C.c_uint64, C.c_int]
        L.orc_permute.argtypes = [P(_Csr), C.c_void_p, P(_Csr)]
        L.orc_bandwidth_stats.argtypes = [P(_Csr), P(C.c_uint64), P(C.c_double)]
        L.orc_load_edges.argtypes = [C.c_char_p, P(C.c_uint64), P(C.c_uint64), P(C.c_void_p), P(C.c_void_p)]
        _lib = L
    return _lib


class Rng:
    """rand 0.9 StdRng (ChaCha12) restatement."""

    def __init__(self, seed: bytes = bytes([42] * 32)):
        assert len(seed) == 32
        self._r = _Rng()
        lib().orc_rng_seed(C.byref(self._r), seed)

    def next_u64(self) -> int:
        return lib().orc_rng_next_u64(C.byref(self._r))

    def next_f64(self) -> float:
        return lib().orc_rng_next_f64(C.byref(self._r))

    def next_u32(self) -> int:
        return lib().orc_rng_next_u32(C.byref(self._r))

    def range_u32(self, lo: int, hi: int) -> int:
        """rand 0.9 `random_range(lo..hi)` for usize / u32 (Canon's method on u32 draws)."""
        return lib().orc_rng_range_u32(C.byref(self._r), lo, hi)


class Csr:
    """Owned host CSR from the oracle (n x n, u64 row_ptr, u32 col, typed values)."""

    def __init__(self, raw: _Csr):
        self._raw = raw

    def __del__(self):
        if getattr(self, "_raw", None) is not None and _lib is not None:
            _lib.orc_csr_free(C.byref(self._raw))
            self._raw = None

    @property
    def n(self) -> int:
        return int(self._raw.n)

    @property
    def nnz(self) -> int:
        return int(self._raw.nnz)

    @property
    def dtype(self) -> int:
        return int(self._raw.dtype)

    def arrays(self):
        """Copies of (row_ptr u64, col u32, values)."""
        n, z = self.n, self.nnz
        rp = np.ctypeslib.as_array(C.cast(self._raw.row_ptr, C.POINTER(C.c_uint64)), (n + 1,)).copy()
        if z:
            col = np.ctypeslib.as_array(C.cast(self._raw.col, C.POINTER(C.c_uint32)), (z,)).copy()
            vt = _VDT[self.dtype]
            ct = {np.uint32: C.c_uint32, np.uint64: C.c_uint64, np.float64: C.c_double}[vt]
            val = np.ctypeslib.as_array(C.cast(self._raw.val, C.POINTER(ct)), (z,)).copy()
        else:
            col = np.zeros(0, np.uint32)
            val = np.zeros(0, _VDT[self.dtype])
        return rp, col, val

    def get(self, r: int, c: int):
        rp, col, val = self.arrays()
        s, e = int(rp[r]), int(rp[r + 1])
        i = int(np.searchsorted(col[s:e], c))
        if i < e - s and col[s + i] == c:
            return val[s + i].item()
        return 0


def _new(fn, *args) -> Csr:
    out = _Csr()
    rc = fn(*args, C.byref(out))
    if rc != 0:
        raise RuntimeError(f"oracle call failed rc={rc}")
    return Csr(out)


def from_coo(n: int, rows, cols, vals, dtype: int = U32) -> Csr:
    rows = np.ascontiguousarray(rows, np.uint32)
    cols = np.ascontiguousarray(cols, np.uint32)
    vals = np.ascontiguousarray(vals, _VDT[dtype])
    return _new(lib().orc_from_coo, n, len(rows), rows.ctypes.data, cols.ctypes.data, vals.ctypes.data, dtype)


def from_edges(n: int, edges, dtype: int = U32) -> Csr:
    e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
    return from_coo(n, e[:, 0], e[:, 1], np.ones(len(e)), dtype)


def from_arrays(row_ptr, col, val, dtype: int) -> Csr:
    rp = np.asarray(row_ptr, np.uint64)
    n = len(rp) - 1
    rows = np.repeat(np.arange(n, dtype=np.uint32), np.diff(rp).astype(np.int64))
    return from_coo(n, rows, col, val, dtype)


def lattice(dims, torus: bool) -> Csr:
    d = (C.c_uint64 * len(dims))(*dims)
    return _new(lib().orc_lattice, d, len(dims), int(torus))


def thin(m: Csr, rng: Rng, density: float) -> Csr:
    return _new(lib().orc_thin, C.byref(m._raw), C.byref(rng._r), density)


def random(rng: Rng, n: int, m: int) -> Csr:
    """CsrMatrix::random (src/graph_csr.rs:163-174)."""
    return _new(lib().orc_random, C.byref(rng._r), n, m)


def convert(m: Csr, dtype: int) -> Csr:
    return _new(lib().orc_convert, C.byref(m._raw), dtype)


def matmul_seq(a: Csr, b: Csr) -> Csr:
    return _new(lib().orc_matmul_seq, C.byref(a._raw), C.byref(b._raw))


def matmul_par(a: Csr, b: Csr, nthreads: int) -> Csr:
    return _new(lib().orc_matmul_par, C.byref(a._raw), C.byref(b._raw), nthreads)


def add(a: Csr, b: Csr) -> Csr:
    return _new(lib().orc_add, C.byref(a._raw), C.byref(b._raw))


def flops(a: Csr, b: Csr) -> int:
    return int(lib().orc_flops(C.byref(a._raw), C.byref(b._raw)))


def identity(n: int, dtype: int = U32) -> Csr:
    """CsrMatrix::identity (src/graph_csr.rs:68-80)."""
    return _new(lib().orc_identity, n, dtype)


def power_until_stable(a: Csr):
    """CsrMatrix::power_until_stable (src/graph_csr.rs:562-577) -> (matrix, squarings)."""
    k = C.c_uint64()
    m = _new(lib().orc_power_until_stable, C.byref(a._raw), C.byref(k))
    return m, int(k.value)


def reachability_sum(a: Csr):
    """CsrMatrix::reachability_sum (src/graph_csr.rs:545-559) -> (sum, last power)."""
    k = C.c_uint64()
    m = _new(lib().orc_reachability_sum, C.byref(a._raw), C.byref(k))
    return m, int(k.value)


def connected_components(a: Csr) -> np.ndarray:
    """CsrMatrix::connected_components (src/graph_csr.rs:580-603) -> component id per node."""
    out = np.empty(max(a.n, 1), np.uint64)
    rc = lib().orc_connected_components(C.byref(a._raw), out.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"oracle call failed rc={rc}")
    return out[:a.n]


def diameter(a: Csr):
    """bench_diameter (src/graph_csr.rs:1228-1319) over the oracle's matmul/add/identity: R0 = A + I;
    repeated squaring until the pattern is stable, then the last power before it times R0 until
    stable -> (diameter, squarings, refinements). Small inputs only (pure-Python loop)."""
    def same(x: Csr, y: Csr):
        xr, xc, _ = x.arrays()
        yr, yc, _ = y.arrays()
        return x.nnz == y.nnz and np.array_equal(xr, yr) and np.array_equal(xc, yc)
    r0 = add(a, identity(a.n, a.dtype))
    current, reach, prev_saved, prev_reach, sq = r0, 1, r0, 0, 0
    while True:
        nxt = matmul_seq(current, current)
        sq += 1
        if same(nxt, current):
            break
        prev_saved, prev_reach, current, reach = current, reach, nxt, reach * 2
    if prev_reach == 0:
        return 1, sq, 0
    refine, d, rf = prev_saved, prev_reach, 0
    while True:
        nxt = matmul_seq(refine, r0)
        d += 1
        rf += 1
        if same(nxt, refine):
            return d - 1, sq, rf
        refine = nxt


def rcm_order(a: Csr) -> np.ndarray:
    """The order CsrMatrix::rcm (src/graph_csr.rs:663-722) permutes by (perm[new] = old)."""
    out = np.empty(max(a.n, 1), np.uint32)
    if lib().orc_rcm_order(C.byref(a._raw), out.ctypes.data) != 0:
        raise ValueError("rcm order is not a permutation (the reference panics in permute)")
    return out[:a.n]


def permute(a: Csr, perm) -> Csr:
    """CsrMatrix::permute (src/graph_csr.rs:726-783), perm[new] = old."""
    p = np.ascontiguousarray(perm, np.uint32)
    assert len(p) == a.n
    return _new(lib().orc_permute, C.byref(a._raw), p.ctypes.data)


def bandwidth_stats(a: Csr):
    """CsrMatrix::bandwidth_stats (src/graph_csr.rs:802-818) -> (max |r-c|, mean |r-c|)."""
    mx, avg = C.c_uint64(), C.c_double()
    lib().orc_bandwidth_stats(C.byref(a._raw), C.byref(mx), C.byref(avg))
    return int(mx.value), float(avg.value)


def einsum_sparse_driven(a: Csr, b: Csr, out: np.ndarray, transpose: bool = False) -> np.ndarray:
    """einsum_sparse_driven (einsum-dyn/src/sparse.rs:70-148) into the dense array `out` (touched
    entries overwritten, the rest kept)."""
    if lib().orc_einsum_sparse_driven(C.byref(a._raw), C.byref(b._raw), out.ctypes.data, out.shape[1],
                                      int(transpose)) != 0:
        raise ValueError("einsum_sparse_driven: u32 or f64 operands of one type")
    return out


def load_edges(path: str):
    """load_edges (src/graph_csr.rs:1209-1224) -> (n, src u32[], dst u32[])."""
    n, m, s, d = C.c_uint64(), C.c_uint64(), C.c_void_p(), C.c_void_p()
    if lib().orc_load_edges(str(path).encode(), C.byref(n), C.byref(m), C.byref(s), C.byref(d)) != 0:
        raise ValueError(f"cannot parse {path}")
    k = int(m.value)
    src = np.ctypeslib.as_array(C.cast(s, C.POINTER(C.c_uint32)), (max(k, 1),))[:k].copy()
    dst = np.ctypeslib.as_array(C.cast(d, C.POINTER(C.c_uint32)), (max(k, 1),))[:k].copy()
    libc = C.CDLL(None)
    libc.free(s)
    libc.free(d)
    return int(n.value), src, dst


def from_edges_undirected(n: int, edges, dtype: int = U32) -> Csr:
    """CsrMatrix::from_edges_undirected (src/graph_csr.rs:138-147)."""
    e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
    off = e[:, 0] != e[:, 1]
    r = np.empty(len(e) + int(off.sum()), np.int64)
    c = np.empty_like(r)
    # triplet order (r,c) then (c,r) per edge, as the reference pushes them
    idx = np.arange(len(e)) + np.concatenate([[0], np.cumsum(off)[:-1]]) if len(e) else np.zeros(0, np.int64)
    r[idx], c[idx] = e[:, 0], e[:, 1]
    r[idx[off] + 1], c[idx[off] + 1] = e[off, 1], e[off, 0]
    return from_coo(n, r, c, np.ones(len(r)), dtype)


def torus_thinned(side: int, epn: float, rng: Rng) -> Csr:
    """The bench_repeated_exponentiation input: side^3 Moore torus thinned to `epn` edges/node
    (src/graph_magnus.rs:707-719)."""
    full = lattice([side, side, side], True)
    density = epn / (full.nnz / full.n)
    return thin(full, rng, density) if density < 1.0 else full


def chacha_block(key_words, counter: int, double_rounds: int = 6):
    """One ChaCha keystream block (16 u32 words) of the oracle's core: 6 double rounds = ChaCha12
    (StdRng), 10 = ChaCha20 (the RFC 8439 vectors)."""
    key = (C.c_uint32 * 8)(*key_words)
    out = (C.c_uint32 * 16)()
    lib().orc_chacha_block(key, counter, double_rounds, out)
    return list(out)
