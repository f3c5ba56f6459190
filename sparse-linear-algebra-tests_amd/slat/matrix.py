"""Host-side mirror of the reference's matrix API, backed by the MI355X engine (libslat.so).

  CsrMatrix    <- src/graph_csr.rs:42-53   (u32 ids, u32 saturating values)
  MagnusMatrix <- src/graph_magnus.rs:11-14 (Sat64 values; usize cols narrowed to u32)
  Csr          <- linalg/src/csr.rs:93-98  (value type u32 | u64 | f64)

Matrices live in device memory (library-owned). `matmul` / `matmul_par` (CsrMatrix),
`matmul` / `matmul_seq` (MagnusMatrix) all run the same HIP SpGEMM: the reference's seq/par
variants differ only in CPU scheduling and produce identical results. Shape mismatches raise
`SlatError(SLAT_EDIM)` where the reference panics on `assert_eq!(self.n, other.n)`.
"""
from __future__ import annotations

import ctypes as C
import threading
from typing import Iterable, Sequence

import numpy as np

from . import _lib as L

_VDT = {L.U32: np.uint32, L.SAT64: np.uint64, L.F64: np.float64}
_CT = {L.U32: C.c_uint32, L.SAT64: C.c_uint64, L.F64: C.c_double}


class Context:
    """One slat_ctx (device + stream). Not shared across host threads."""

    def __init__(self, device: int = 0):
        self._ptr = C.c_void_p()
        L.check(L.lib().slat_ctx_create(device, C.byref(self._ptr)))
        self.device = device

    @property
    def ptr(self):
        return self._ptr

    def close(self):
        if self._ptr:
            L.lib().slat_ctx_destroy(self._ptr)
            self._ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stats(self) -> dict:
        s = L.Stats()
        L.check(L.lib().slat_get_stats(self._ptr, C.byref(s)), self._ptr)
        return s.as_dict()

    def set_stream(self, stream_ptr: int | None):
        L.check(L.lib().slat_ctx_set_stream(self._ptr, C.c_void_p(stream_ptr or 0)), self._ptr)

    def sync(self):
        L.check(L.lib().slat_sync(self._ptr), self._ptr)


_tls = threading.local()


def default_context(device: int = 0) -> Context:
    ctxs = getattr(_tls, "ctxs", None)
    if ctxs is None:
        ctxs = _tls.ctxs = {}
    if device not in ctxs:
        ctxs[device] = Context(device)
    return ctxs[device]


class StdRng:
    """rand 0.9 `StdRng::from_seed` (ChaCha12), as used by the reference's benches."""

    def __init__(self, seed: bytes = bytes([42] * 32)):
        if len(seed) != 32:
            raise ValueError("seed must be 32 bytes")
        self._s = L.RngState()
        L.lib().slat_rng_seed(C.byref(self._s), seed)

    @classmethod
    def from_seed(cls, seed) -> "StdRng":
        return cls(bytes(seed))

    def next_u64(self) -> int:
        return int(L.lib().slat_rng_next_u64(C.byref(self._s)))

    def random_f64(self) -> float:
        return float(L.lib().slat_rng_next_f64(C.byref(self._s)))

    def next_u32(self) -> int:
        return int(L.lib().slat_rng_next_u32(C.byref(self._s)))

    def random_range(self, lo: int, hi: int) -> int:
        """`rng.random_range(lo..hi)` for usize / u32 bounds (rand 0.9: u32 Canon's method)."""
        return int(L.lib().slat_rng_range_u32(C.byref(self._s), lo, hi))


# ------------------------------------------------------------------------------------------------
# host CSR (numpy) produced by the library's constructors
# ------------------------------------------------------------------------------------------------
class HostCsr:
    """Plain host arrays: row_ptr u64 [n+1], col_idx u32, values."""

    def __init__(self, n: int, row_ptr, col_idx, values, dtype: int):
        self.n = int(n)
        self.row_ptr = np.ascontiguousarray(row_ptr, np.uint64)
        self.col_idx = np.ascontiguousarray(col_idx, np.uint32)
        self.values = np.ascontiguousarray(values, _VDT[dtype])
        self.dtype = dtype

    @property
    def nnz(self) -> int:
        return int(len(self.col_idx))

    @staticmethod
    def _take(h: L.HostCsr) -> "HostCsr":
        n, z, dt = int(h.n), int(h.nnz), int(h.dtype)
        rp = np.ctypeslib.as_array(C.cast(h.row_ptr, C.POINTER(C.c_uint64)), (n + 1,)).copy()
        if z:
            col = np.ctypeslib.as_array(C.cast(h.col_idx, C.POINTER(C.c_uint32)), (z,)).copy()
            val = np.ctypeslib.as_array(C.cast(h.values, C.POINTER(_CT[dt])), (z,)).copy()
        else:
            col, val = np.zeros(0, np.uint32), np.zeros(0, _VDT[dt])
        L.lib().slat_host_csr_free(C.byref(h))
        return HostCsr(n, rp, col, val, dt)

    def _raw(self) -> L.HostCsr:
        h = L.HostCsr()
        h.n, h.nnz, h.dtype = self.n, self.nnz, self.dtype
        h.row_ptr, h.col_idx, h.values = self.row_ptr.ctypes.data, self.col_idx.ctypes.data, self.values.ctypes.data
        return h

    def view(self) -> L.CsrView:
        v = L.CsrView()
        v.n_rows = v.n_cols = self.n
        v.nnz = self.nnz
        v.row_ptr, v.col_idx, v.values = self.row_ptr.ctypes.data, self.col_idx.ctypes.data, self.values.ctypes.data
        v.dtype, v.residency = self.dtype, L.HOST
        v.max_row_nnz = int(np.diff(self.row_ptr).max(initial=0))
        return v

    def astype(self, dtype: int) -> "HostCsr":
        return HostCsr(self.n, self.row_ptr, self.col_idx, self.values.astype(_VDT[dtype]), dtype)


def host_from_coo(n: int, rows, cols, vals, dtype: int = L.U32) -> HostCsr:
    rows = np.ascontiguousarray(rows, np.uint32)
    cols = np.ascontiguousarray(cols, np.uint32)
    vals = np.ascontiguousarray(vals, _VDT[dtype])
    h = L.HostCsr()
    L.check(L.lib().slat_host_from_coo(n, len(rows), rows.ctypes.data, cols.ctypes.data, vals.ctypes.data, dtype,
                                       C.byref(h)))
    return HostCsr._take(h)


def host_lattice(dims: Sequence[int], torus: bool) -> HostCsr:
    d = (C.c_uint64 * len(dims))(*dims)
    h = L.HostCsr()
    L.check(L.lib().slat_host_lattice(d, len(dims), int(torus), C.byref(h)))
    return HostCsr._take(h)


def host_thin(m: HostCsr, rng: StdRng, density: float) -> HostCsr:
    raw = m._raw()
    h = L.HostCsr()
    L.check(L.lib().slat_host_thin(C.byref(raw), C.byref(rng._s), float(density), C.byref(h)))
    return HostCsr._take(h)


def host_random(rng: StdRng, n: int, m: int) -> HostCsr:
    """CsrMatrix::random (src/graph_csr.rs:163-174) on the host: m edge draws, no self-loops."""
    h = L.HostCsr()
    L.check(L.lib().slat_host_random(C.byref(rng._s), n, m, C.byref(h)))
    return HostCsr._take(h)


def host_rmat(scale: int, n_edges: int, a=0.57, b=0.19, c=0.19, seed: bytes = bytes([42] * 32)) -> HostCsr:
    h = L.HostCsr()
    L.check(L.lib().slat_host_rmat(scale, n_edges, a, b, c, seed, C.byref(h)))
    return HostCsr._take(h)


def load_edges(path: str):
    """load_edges (src/graph_csr.rs:1209-1224) -> (n, src u32[], dst u32[]); n = max id + 1."""
    n, m, s, d = C.c_uint64(), C.c_uint64(), C.c_void_p(), C.c_void_p()
    L.check(L.lib().slat_load_edges(str(path).encode(), C.byref(n), C.byref(m), C.byref(s), C.byref(d)))
    k = int(m.value)
    try:
        src = np.ctypeslib.as_array(C.cast(s, C.POINTER(C.c_uint32)), (max(k, 1),))[:k].copy()
        dst = np.ctypeslib.as_array(C.cast(d, C.POINTER(C.c_uint32)), (max(k, 1),))[:k].copy()
    finally:
        L.lib().slat_edges_free(s, d)
    return int(n.value), src, dst


def torus_thinned(side: int, epn: float, rng: StdRng) -> HostCsr:
    """side^3 Moore torus thinned to `epn` edges per node (src/graph_magnus.rs:713-719)."""
    full = host_lattice([side, side, side], True)
    density = epn / (full.nnz / full.n)
    return host_thin(full, rng, density) if density < 1.0 else full


def torus_thinned_device(side: int, epn: float, rng: StdRng, ctx: Context | None = None) -> "CsrMatrix":
    """torus_thinned, generated on the device (lattice + thin kernels): same matrix, same draws."""
    full = CsrMatrix.lattice([side, side, side], True, ctx)
    density = epn / (full.nnz() / full.n)
    return full.thin(rng, density) if density < 1.0 else full


# ------------------------------------------------------------------------------------------------
# host-resident products (the reference's Vec in / Vec out calls, PCIe included)
# ------------------------------------------------------------------------------------------------
class _PinnedBuf:
    """Page-locked host bytes (slat_host_alloc), freed with the last array that views them."""

    def __init__(self, nbytes: int):
        self.ptr = C.c_void_p()
        L.check(L.lib().slat_host_alloc(max(int(nbytes), 1), C.byref(self.ptr)))
        self.__array_interface__ = {"shape": (max(int(nbytes), 1),), "typestr": "|u1",
                                    "data": (self.ptr.value, False), "version": 3}

    def __del__(self):
        try:
            L.lib().slat_host_free(self.ptr)
        except Exception:
            pass


def pinned_empty(n: int, dtype) -> np.ndarray:
    """An uninitialised numpy array of n elements in page-locked host memory."""
    dt = np.dtype(dtype)
    return np.asarray(_PinnedBuf(n * dt.itemsize))[:n * dt.itemsize].view(dt)


def spgemm_host(a: HostCsr, b: HostCsr, ctx: Context | None = None, alloc=np.empty, flags: int = 0) -> HostCsr:
    """C = A * B with host operands and a host result: the cost a drop-in pays for the reference's
    signature (CsrMatrix::matmul(&self, &Self) -> Self over Vecs): both operands cross to the device,
    the product runs, C comes back into host arrays from `alloc(n, dtype)` (np.empty: pageable;
    pinned_empty: page-locked), and the device result is freed."""
    ctx = ctx or default_context()
    if a.dtype != b.dtype:
        raise TypeError("operands must have the same value type")
    va, vb = a.view(), b.view()
    out = L.CsrOwned()
    L.check(L.lib().slat_spgemm(ctx.ptr, C.byref(va), C.byref(vb), C.byref(out), flags), ctx.ptr)
    try:
        n, z = int(out.n_rows), int(out.nnz)
        rp = alloc(n + 1, np.uint64)
        col = alloc(max(z, 1), np.uint32)
        val = alloc(max(z, 1), _VDT[a.dtype])
        v = L.lib().slat_csr_view_of(C.byref(out))
        L.check(L.lib().slat_csr_to_host(ctx.ptr, C.byref(v), rp.ctypes.data, col.ctypes.data, val.ctypes.data), ctx.ptr)
    finally:
        L.lib().slat_csr_free(ctx.ptr, C.byref(out))
    return HostCsr(n, rp, col[:z], val[:z], a.dtype)


# ------------------------------------------------------------------------------------------------
# device-resident matrices
# ------------------------------------------------------------------------------------------------
class DeviceCsr:
    """A library-owned device CSR (slat_csr). Host arrays are fetched lazily."""

    DTYPE = L.U32

    def __init__(self, owned: L.CsrOwned, ctx: Context):
        self._m = owned
        self._ctx = ctx
        self._host = None
        self._view = None  # the matrix is immutable between in-place replacements (permute)

    def __del__(self):
        try:
            if self._m is not None and self._m.row_ptr:
                L.lib().slat_csr_free(self._ctx.ptr, C.byref(self._m))
        except Exception:
            pass

    # -- construction ----------------------------------------------------------------------------
    @classmethod
    def from_host(cls, h: HostCsr, ctx: Context | None = None):
        ctx = ctx or default_context()
        if h.dtype != cls.DTYPE:
            h = h.astype(cls.DTYPE)
        v = h.view()
        out = L.CsrOwned()
        L.check(L.lib().slat_csr_create(ctx.ptr, C.byref(v), C.byref(out)), ctx.ptr)
        m = cls(out, ctx)
        m._host = h
        return m

    @classmethod
    def new(cls, n: int):
        return cls.from_host(HostCsr(n, np.zeros(n + 1, np.uint64), [], [], cls.DTYPE))

    @classmethod
    def identity(cls, n: int, ctx: Context | None = None):
        """CsrMatrix::identity (src/graph_csr.rs:68-80), built on the device."""
        ctx = ctx or default_context()
        out = L.CsrOwned()
        L.check(L.lib().slat_csr_identity(ctx.ptr, n, cls.DTYPE, C.byref(out)), ctx.ptr)
        return cls(out, ctx)

    @classmethod
    def random(cls, rng: StdRng, n: int, m: int, ctx: Context | None = None):
        """CsrMatrix::random (src/graph_csr.rs:163-174): the reference's draws, then to the device."""
        return cls.from_host(host_random(rng, n, m), ctx)

    @classmethod
    def from_coo(cls, n: int, triplets: Iterable):
        t = np.asarray(list(triplets), dtype=np.float64 if cls.DTYPE == L.F64 else np.uint64).reshape(-1, 3)
        return cls.from_host(host_from_coo(n, t[:, 0], t[:, 1], t[:, 2], cls.DTYPE))

    @classmethod
    def from_edges(cls, n: int, edges):
        e = np.asarray(list(edges), dtype=np.int64).reshape(-1, 2)
        return cls.from_host(host_from_coo(n, e[:, 0], e[:, 1], np.ones(len(e)), cls.DTYPE))

    @classmethod
    def from_edges_undirected(cls, n: int, edges):
        e = np.asarray(list(edges), dtype=np.int64).reshape(-1, 2)
        off = e[:, 0] != e[:, 1]
        r = np.concatenate([e[:, 0], e[off, 1]])
        c = np.concatenate([e[:, 1], e[off, 0]])
        return cls.from_host(host_from_coo(n, r, c, np.ones(len(r)), cls.DTYPE))

    @classmethod
    def from_adjacency(cls, it):
        names, edges = {}, []
        for a, b in it:
            ai = names.setdefault(a, len(names))
            bi = names.setdefault(b, len(names))
            edges.append((ai, bi))
        return cls.from_edges(len(names), edges), names

    @classmethod
    def lattice(cls, dims: Sequence[int], torus: bool, ctx: Context | None = None):
        """CsrMatrix::lattice (src/graph_csr.rs:177-222), built on the device (u32 values 1)."""
        ctx = ctx or default_context()
        d = (C.c_uint64 * len(dims))(*dims)
        out = L.CsrOwned()
        L.check(L.lib().slat_csr_lattice(ctx.ptr, d, len(dims), int(torus), C.byref(out)), ctx.ptr)
        m = CsrMatrix(out, ctx)
        return m if cls.DTYPE == L.U32 else cls.from_host(m.host().astype(cls.DTYPE), ctx)

    def thin(self, rng: StdRng, density: float):
        """CsrMatrix::thin (src/graph_csr.rs:225-247) on the device; `rng` advances like the reference's."""
        v = self.view()
        out = L.CsrOwned()
        L.check(L.lib().slat_csr_thin(self._ctx.ptr, C.byref(v), C.byref(rng._s), float(density), C.byref(out)),
                self._ctx.ptr)
        return type(self)(out, self._ctx)

    @classmethod
    def from_coo_device(cls, n: int, rows, cols, vals, ctx: Context | None = None):
        """CsrMatrix::from_coo (src/graph_csr.rs:83-129) on the device, from host triplet arrays."""
        ctx = ctx or default_context()
        r = np.ascontiguousarray(rows, np.uint32)
        c = np.ascontiguousarray(cols, np.uint32)
        v = np.ascontiguousarray(vals, _VDT[cls.DTYPE])
        out = L.CsrOwned()
        L.check(L.lib().slat_csr_from_coo(ctx.ptr, n, len(r), r.ctypes.data, c.ctypes.data, v.ctypes.data, cls.DTYPE,
                                          L.HOST, C.byref(out)), ctx.ptr)
        return cls(out, ctx)

    @classmethod
    def from_edges_device(cls, n: int, src, dst, undirected: bool = False, ctx: Context | None = None):
        """CsrMatrix::from_edges / from_edges_undirected (src/graph_csr.rs:132-147) on the device."""
        ctx = ctx or default_context()
        s = np.ascontiguousarray(src, np.uint32)
        d = np.ascontiguousarray(dst, np.uint32)
        if len(s) != len(d):
            raise ValueError("src and dst differ in length")
        out = L.CsrOwned()
        L.check(L.lib().slat_csr_from_edges(ctx.ptr, n, len(s), s.ctypes.data, d.ctypes.data, int(undirected),
                                            L.HOST, C.byref(out)), ctx.ptr)
        m = CsrMatrix(out, ctx)
        return m if cls.DTYPE == L.U32 else cls.from_host(m.host().astype(cls.DTYPE), ctx)

    # -- reordering (src/graph_csr.rs:663-818) -------------------------------------------------------
    perm = None  # perm[new] = old after permute / rcm, like the reference's `perm` field

    def rcm_order(self) -> np.ndarray:
        """The order CsrMatrix::rcm permutes by (perm[new] = old); degree ties in column order."""
        p = np.zeros(max(self.n, 1), np.uint32)
        v = self.view()
        L.check(L.lib().slat_rcm_order(self._ctx.ptr, C.byref(v), p.ctypes.data), self._ctx.ptr)
        return p[:self.n]

    def permute(self, perm):
        """CsrMatrix::permute (src/graph_csr.rs:726-783), in place; stores `perm`."""
        p = np.ascontiguousarray(perm, np.uint32)
        if len(p) != self.n:
            raise ValueError("perm length != n")  # assert_eq!(perm.len(), nu)
        v = self.view()
        out = L.CsrOwned()
        L.check(L.lib().slat_csr_permute(self._ctx.ptr, C.byref(v), p.ctypes.data, L.HOST, C.byref(out)),
                self._ctx.ptr)
        L.lib().slat_csr_free(self._ctx.ptr, C.byref(self._m))
        self._m = out
        self._host = None
        self._view = None
        self.perm = p.copy()

    def rcm(self):
        """CsrMatrix::rcm (src/graph_csr.rs:663-722), in place; stores the permutation."""
        self.permute(self.rcm_order())

    def unpermute(self):
        """CsrMatrix::unpermute (src/graph_csr.rs:786-799): permute by the inverse, drop `perm`."""
        if self.perm is None:
            return
        inv = np.empty_like(self.perm)
        inv[self.perm] = np.arange(len(self.perm), dtype=np.uint32)
        self.permute(inv)
        self.perm = None

    def bandwidth_stats(self):
        """CsrMatrix::bandwidth_stats (src/graph_csr.rs:802-818) -> (max |r-c|, mean |r-c|)."""
        mx, avg = C.c_uint64(), C.c_double()
        v = self.view()
        L.check(L.lib().slat_bandwidth_stats(self._ctx.ptr, C.byref(v), C.byref(mx), C.byref(avg)), self._ctx.ptr)
        return int(mx.value), float(avg.value)

    # -- dense output (einsum-dyn/src/sparse.rs:70-148) ---------------------------------------------
    def einsum_sparse_driven(self, other: "DeviceCsr", out: np.ndarray | None = None, transpose: bool = False):
        """einsum_sparse_driven("ab,bc->ac" | "ab,bc->ca", self, other, out): touched entries of the
        dense host array `out` are overwritten with their sums, the rest kept. u32 values are plain
        (wrapping) u32 here, as in the einsum tests; f64 folds like the reference."""
        rows, cols = (other.n, self.n) if transpose else (self.n, other.n)
        dt = np.uint32 if self.DTYPE == L.U32 else np.float64
        if out is None:
            out = np.zeros((rows, cols), dt)
        if out.dtype != dt or out.ndim != 2 or out.shape[0] != rows or out.shape[1] < cols or not out.flags.c_contiguous:
            raise ValueError("out: C-contiguous (rows, >= cols) array of the value type")
        a, b = self.view(), other.view()
        L.check(L.lib().slat_spgemm_dense(self._ctx.ptr, C.byref(a), C.byref(b), out.ctypes.data, out.shape[1],
                                          int(transpose), L.HOST), self._ctx.ptr)
        return out

    # -- accessors ---------------------------------------------------------------------------------
    @property
    def n(self) -> int:
        return int(self._m.n_rows)

    def nnz(self) -> int:
        return int(self._m.nnz)

    @property
    def capacity(self) -> int:
        return int(self._m.capacity)

    @property
    def max_row_nnz(self) -> int:
        return int(self._m.max_row_nnz)

    def view(self) -> L.CsrView:
        return L.lib().slat_csr_view_of(C.byref(self._m))

    def _cview(self) -> L.CsrView:
        """The view, cached for the product calls (never handed out: callers may edit a view)."""
        if self._view is None:
            self._view = self.view()
        return self._view

    def host(self) -> HostCsr:
        if self._host is None:
            n, z, dt = self.n, self.nnz(), int(self._m.dtype)
            rp = np.empty(n + 1, np.uint64)
            col = np.empty(max(z, 1), np.uint32)
            val = np.empty(max(z, 1), _VDT[dt])
            v = self.view()
            L.check(L.lib().slat_csr_to_host(self._ctx.ptr, C.byref(v), rp.ctypes.data, col.ctypes.data,
                                             val.ctypes.data), self._ctx.ptr)
            self._host = HostCsr(n, rp, col[:z], val[:z], dt)
        return self._host

    @property
    def row_ptr(self):
        return self.host().row_ptr

    @property
    def col_idx(self):
        return self.host().col_idx

    @property
    def values(self):
        return self.host().values

    def get(self, r: int, c: int):
        h = self.host()
        s, e = int(h.row_ptr[r]), int(h.row_ptr[r + 1])
        i = int(np.searchsorted(h.col_idx[s:e], c))
        if i < e - s and h.col_idx[s + i] == c:
            return h.values[s + i].item()
        return 0

    def row_iter(self, r: int):
        h = self.host()
        s, e = int(h.row_ptr[r]), int(h.row_ptr[r + 1])
        return zip(h.col_idx[s:e].tolist(), h.values[s:e].tolist())

    # -- the hot path --------------------------------------------------------------------------------
    def _spgemm(self, other: "DeviceCsr", flags: int = 0):
        if type(other) is not type(self):
            raise TypeError("operands must have the same matrix type")
        a, b = self._cview(), other._cview()
        out = L.CsrOwned()
        L.check(L.lib().slat_spgemm(self._ctx.ptr, C.byref(a), C.byref(b), C.byref(out), flags), self._ctx.ptr)
        return type(self)(out, self._ctx)

    # -- the reference's SpGEMM consumers, device-resident --------------
    def add(self, other: "DeviceCsr"):
        """CsrMatrix::add (src/graph_csr.rs:487-542) / MagnusMatrix::add (src/graph_magnus.rs:245-300)."""
        if type(other) is not type(self):
            raise TypeError("operands must have the same matrix type")
        a, b = self.view(), other.view()
        out = L.CsrOwned()
        L.check(L.lib().slat_csr_add(self._ctx.ptr, C.byref(a), C.byref(b), C.byref(out)), self._ctx.ptr)
        return type(self)(out, self._ctx)

    def same_pattern(self, other: "DeviceCsr") -> bool:
        """nnz, row_ptr and col_idx equal (the test in power_until_stable, src/graph_csr.rs:567-569)."""
        a, b = self.view(), other.view()
        eq = C.c_int32()
        L.check(L.lib().slat_csr_pattern_equal(self._ctx.ptr, C.byref(a), C.byref(b), C.byref(eq)), self._ctx.ptr)
        return bool(eq.value)

    def reachability_sum(self):
        """CsrMatrix::reachability_sum (src/graph_csr.rs:545-559) -> (sum, k)."""
        a, out, k = self.view(), L.CsrOwned(), C.c_uint64()
        L.check(L.lib().slat_reachability_sum(self._ctx.ptr, C.byref(a), C.byref(out), C.byref(k)), self._ctx.ptr)
        return type(self)(out, self._ctx), int(k.value)

    def power_until_stable(self):
        """CsrMatrix::power_until_stable (src/graph_csr.rs:562-577) -> (matrix, k)."""
        a, out, k = self.view(), L.CsrOwned(), C.c_uint64()
        L.check(L.lib().slat_power_until_stable(self._ctx.ptr, C.byref(a), C.byref(out), C.byref(k)), self._ctx.ptr)
        return type(self)(out, self._ctx), int(k.value)

    def connected_components(self) -> list:
        """CsrMatrix::connected_components (src/graph_csr.rs:580-603) -> Vec<usize> as a list."""
        comp = np.zeros(max(self.n, 1), np.uint64)
        a = self.view()
        L.check(L.lib().slat_connected_components(self._ctx.ptr, C.byref(a), comp.ctypes.data), self._ctx.ptr)
        return comp[:self.n].tolist()

    def diameter(self):
        """bench_diameter (src/graph_csr.rs:1228-1319) on this undirected graph, device-resident:
        -> (diameter, squarings, refinements)."""
        a, d, sq, rf = self.view(), C.c_uint64(), C.c_uint64(), C.c_uint64()
        L.check(L.lib().slat_diameter(self._ctx.ptr, C.byref(a), C.byref(d), C.byref(sq), C.byref(rf)), self._ctx.ptr)
        return int(d.value), int(sq.value), int(rf.value)

    def clone(self):
        """`Clone` of the owned matrix: a device-to-device copy."""
        v = self.view()
        out = L.CsrOwned()
        L.check(L.lib().slat_csr_create(self._ctx.ptr, C.byref(v), C.byref(out)), self._ctx.ptr)
        return type(self)(out, self._ctx)

    def matmul_rowblock(self, row_begin: int, row_end: int, other, flags: int = 0):
        """Rows [row_begin, row_end) of self * other (slat_spgemm_rowblock); `other` may be a
        PreparedB of the right operand (slat_spgemm_rowblock_prepared: its ELL image built once)."""
        a = self._cview()
        out = L.CsrOwned()
        if isinstance(other, PreparedB):
            if other.dtype != self.DTYPE:
                raise TypeError("operands must have the same value type")
            if other._ctx is not self._ctx:
                # the handle's ELL image lives in its own context's pool and is released on that
                # context's stream, which has no ordering against this one
                raise ValueError("a PreparedB must be used with the context that prepared it")
            L.check(L.lib().slat_spgemm_rowblock_prepared(self._ctx.ptr, C.byref(a), row_begin, row_end, other.ptr,
                                                          C.byref(out), flags), self._ctx.ptr)
        else:
            b = other._cview()
            L.check(L.lib().slat_spgemm_rowblock(self._ctx.ptr, C.byref(a), row_begin, row_end, C.byref(b),
                                                 C.byref(out), flags), self._ctx.ptr)
        return type(self)(out, self._ctx)

    def prepare(self) -> "PreparedB":
        """This matrix as a prepared right operand (slat_bprep_create)."""
        return PreparedB(self)


class PreparedB:
    """A right operand prepared once (slat_bprep_create: B's padded ELL image and value summary) for
    many row-block products; holds a reference to the matrix, whose arrays it borrows."""

    def __init__(self, m: DeviceCsr):
        self._m = m
        self._ctx = m._ctx
        self.dtype = m.DTYPE
        self.ptr = C.c_void_p()
        v = m._cview()
        L.check(L.lib().slat_bprep_create(self._ctx.ptr, C.byref(v), C.byref(self.ptr)), self._ctx.ptr)

    def __del__(self):
        try:
            if self.ptr:
                L.lib().slat_bprep_free(self._ctx.ptr, self.ptr)
                self.ptr = C.c_void_p()
        except Exception:
            pass


class CsrMatrix(DeviceCsr):
    """`CsrMatrix` (src/graph_csr.rs:42): u32 node ids, saturating u32 values."""

    DTYPE = L.U32

    def matmul(self, other: "CsrMatrix") -> "CsrMatrix":
        """CsrMatrix::matmul (src/graph_csr.rs:306-346) on the MI355X engine."""
        return self._spgemm(other)

    def matmul_par(self, other: "CsrMatrix") -> "CsrMatrix":
        """CsrMatrix::matmul_par (src/graph_csr.rs:350-484): same result as matmul."""
        return self._spgemm(other)


class MagnusMatrix(DeviceCsr):
    """`MagnusMatrix` (src/graph_magnus.rs:11): Sat64 values."""

    DTYPE = L.SAT64

    def matmul(self, other: "MagnusMatrix") -> "MagnusMatrix":
        """MagnusMatrix::matmul (src/graph_magnus.rs:225-232, magnus_spgemm_parallel)."""
        return self._spgemm(other)

    def matmul_seq(self, other: "MagnusMatrix") -> "MagnusMatrix":
        """MagnusMatrix::matmul_seq (src/graph_magnus.rs:235-242, magnus_spgemm)."""
        return self._spgemm(other)


class MagnusMatrixUsize:
    """`MagnusMatrix` in the reference's own layout (src/graph_magnus.rs:11-14): magnus's
    SparseMatrixCSR<Sat64> with usize (u64) column ids, device-resident (slat_magnus)."""

    def __init__(self, owned: L.MagnusOwned, ctx: Context):
        self._m = owned
        self._ctx = ctx

    def __del__(self):
        try:
            if self._m is not None and self._m.row_ptr:
                L.lib().slat_magnus_free(self._ctx.ptr, C.byref(self._m))
        except Exception:
            pass

    @staticmethod
    def host_view(n: int, row_ptr, col_idx, values, n_cols: int | None = None) -> L.MagnusView:
        """A host view over u64 arrays (kept alive by the caller)."""
        v = L.MagnusView()
        v.n_rows, v.n_cols, v.nnz = n, n if n_cols is None else n_cols, len(col_idx)
        v.row_ptr, v.col_idx, v.values = row_ptr.ctypes.data, col_idx.ctypes.data, values.ctypes.data
        v.residency = L.HOST
        return v

    @staticmethod
    def matmul_host(a: L.MagnusView, b: L.MagnusView, ctx: Context | None = None) -> "MagnusMatrixUsize":
        ctx = ctx or default_context()
        out = L.MagnusOwned()
        L.check(L.lib().slat_magnus_matmul(ctx.ptr, C.byref(a), C.byref(b), C.byref(out), 0), ctx.ptr)
        return MagnusMatrixUsize(out, ctx)

    def view(self) -> L.MagnusView:
        return L.lib().slat_magnus_view_of(C.byref(self._m))

    def matmul(self, other: "MagnusMatrixUsize") -> "MagnusMatrixUsize":
        """MagnusMatrix::matmul (src/graph_magnus.rs:225-232) with usize columns in and out."""
        return MagnusMatrixUsize.matmul_host(self.view(), other.view(), self._ctx)

    matmul_seq = matmul  # src/graph_magnus.rs:235-242: the same product

    def add(self, other: "MagnusMatrixUsize") -> "MagnusMatrixUsize":
        """MagnusMatrix::add (src/graph_magnus.rs:245-300): per-row sorted union, Sat64 sums."""
        return MagnusMatrixUsize.add_host(self.view(), other.view(), self._ctx)

    @staticmethod
    def add_host(a: L.MagnusView, b: L.MagnusView, ctx: Context | None = None) -> "MagnusMatrixUsize":
        ctx = ctx or default_context()
        out = L.MagnusOwned()
        L.check(L.lib().slat_magnus_add(ctx.ptr, C.byref(a), C.byref(b), C.byref(out)), ctx.ptr)
        return MagnusMatrixUsize(out, ctx)

    def reachability_sum(self):
        """MagnusMatrix::reachability_sum (src/graph_magnus.rs:303-317): (sum, k)."""
        out, k = L.MagnusOwned(), C.c_uint64()
        v = self.view()
        L.check(L.lib().slat_magnus_reachability_sum(self._ctx.ptr, C.byref(v), C.byref(out), C.byref(k)), self._ctx.ptr)
        return MagnusMatrixUsize(out, self._ctx), int(k.value)

    def power_until_stable(self):
        """MagnusMatrix::power_until_stable (src/graph_magnus.rs:320-335): (closure, squarings)."""
        out, k = L.MagnusOwned(), C.c_uint64()
        v = self.view()
        L.check(L.lib().slat_magnus_power_until_stable(self._ctx.ptr, C.byref(v), C.byref(out), C.byref(k)), self._ctx.ptr)
        return MagnusMatrixUsize(out, self._ctx), int(k.value)

    def connected_components(self) -> list:
        """MagnusMatrix::connected_components (src/graph_magnus.rs:338-359): usize component ids."""
        comp = np.zeros(self.n, np.uint64)
        v = self.view()
        L.check(L.lib().slat_magnus_connected_components(self._ctx.ptr, C.byref(v), comp.ctypes.data), self._ctx.ptr)
        return [int(c) for c in comp]

    @property
    def n(self) -> int:
        return int(self._m.n_rows)

    def nnz(self) -> int:
        return int(self._m.nnz)

    def host(self):
        """(row_ptr u64, col_idx u64, values u64) host arrays."""
        n, z = self.n, self.nnz()
        rp = np.empty(n + 1, np.uint64)
        col = np.empty(max(z, 1), np.uint64)
        val = np.empty(max(z, 1), np.uint64)
        L.check(L.lib().slat_magnus_to_host(self._ctx.ptr, C.byref(self._m), rp.ctypes.data, col.ctypes.data,
                                            val.ctypes.data), self._ctx.ptr)
        return rp, col[:z], val[:z]


class Csr(DeviceCsr):
    """`linalg::csr::Csr<u32, V>` (linalg/src/csr.rs:93) with V chosen by `dtype`."""

    def __init__(self, owned: L.CsrOwned, ctx: Context):
        super().__init__(owned, ctx)

    @classmethod
    def of(cls, dtype: int):
        return {L.U32: CsrU32, L.SAT64: CsrU64, L.F64: CsrF64}[dtype]

    def matmul(self, other):
        """Csr::matmul (linalg/src/csr.rs:308-356)."""
        return self._spgemm(other)

    def matmul_par(self, other):
        """Csr::matmul_par (linalg/src/csr.rs:361-466)."""
        return self._spgemm(other)


class CsrU32(Csr):
    DTYPE = L.U32


class CsrU64(Csr):
    DTYPE = L.SAT64


class CsrF64(Csr):
    DTYPE = L.F64


KEYS_PER_NODE = 16  # src/dense_btree.rs:2
MAX_BTREE_HEIGHT = 8  # src/dense_btree.rs:3


def btree_levels(n: int):
    """compute_levels (src/dense_btree.rs:9-42): (height, level sizes, level starts) of the compact
    K-ary separator tree over n sorted keys; level 0 is the root."""
    kpn = KEYS_PER_NODE
    leaf_count = (n + kpn - 1) // kpn
    sizes, starts = [0] * MAX_BTREE_HEIGHT, [0] * MAX_BTREE_HEIGHT
    if leaf_count <= 1:
        return 0, sizes, starts
    stack, count = [], leaf_count
    while count > 1:
        count = (count + kpn - 1) // kpn
        stack.append(count)
    height = len(stack)
    for i in range(height):
        sizes[i] = stack[height - 1 - i]
    start = 0
    for i in range(height):
        starts[i] = start
        start += sizes[i] * kpn
    return height, sizes, starts


def btree_internal(values: np.ndarray) -> np.ndarray:
    """The separator nodes DenseBTree::extend_from_sorted (src/dense_btree.rs:116-162) writes before
    a row's sorted data: the bottom internal level holds each leaf chunk's last key, every upper
    level each child node's last key, padding with the row's max key. Empty for <= 16 keys."""
    n, kpn = len(values), KEYS_PER_NODE
    if (n + kpn - 1) // kpn <= 1:
        return np.zeros(0, values.dtype)
    height, sizes, starts = btree_levels(n)
    internal_len = starts[height - 1] + sizes[height - 1] * kpn
    nodes = np.full(internal_len, values[n - 1], values.dtype)
    bottom = height - 1
    chunk = np.arange(sizes[bottom] * kpn)
    nodes[starts[bottom]:starts[bottom] + len(chunk)] = values[np.minimum((chunk + 1) * kpn, n) - 1]
    for level in range(bottom - 1, -1, -1):
        child = np.arange(sizes[level] * kpn)
        ok = child < sizes[level + 1]
        base = starts[level]
        nodes[base:base + len(child)][ok] = nodes[starts[level + 1] + child[ok] * kpn + kpn - 1]
    return nodes


def btree_index(nodes: np.ndarray, internal_len: int, value: int):
    """DenseBTree::index (src/dense_btree.rs:176-205) over one row's [separators | data]: ("ok", i)
    on an exact match, ("err", i) with the insertion point otherwise (slice::binary_search's
    answer)."""
    n = len(nodes) - internal_len
    if n == 0:
        return ("err", 0)
    if value > nodes[-1]:
        return ("err", n)
    height, _, starts = btree_levels(n)
    node = 0
    for level in range(height):
        base = starts[level] + node * KEYS_PER_NODE
        node = node * KEYS_PER_NODE + int(np.count_nonzero(value > nodes[base:base + KEYS_PER_NODE]))
    c0 = internal_len + node * KEYS_PER_NODE
    c1 = min(c0 + KEYS_PER_NODE, len(nodes))
    for i in range(c0, c1):
        if nodes[i] == value:
            return ("ok", i - internal_len)
        if nodes[i] > value:
            return ("err", i - internal_len)
    return ("err", c1 - internal_len)


class CsrBTreeMatrix:
    """`CsrBTreeMatrix` (src/graph_csr_btree.rs:44-52) in its host layout: DenseBTreeList's flat
    `nodes` (every row as [separator nodes | sorted data], src/dense_btree.rs:269-330, the
    separators built exactly as DenseBTree::extend_from_sorted does), the flat `values`, and per
    row data_start (NodeEntry::data_start, plus total_data_len() at the end), data_off (offset +
    internal_len) and internal_len. matmul_par runs on the MI355X engine through
    slat_spgemm_btree, which reads only the data slices."""

    def __init__(self, n: int, nodes, values, data_start, data_off, ctx: Context | None = None, internal_len=None):
        self.n = int(n)
        self.nodes = np.ascontiguousarray(nodes, np.uint32)
        self.values = np.ascontiguousarray(values, np.uint32)
        self.data_start = np.ascontiguousarray(data_start, np.uint64)
        self.data_off = np.ascontiguousarray(data_off, np.uint64)
        self.internal_len = None if internal_len is None else np.ascontiguousarray(internal_len, np.uint64)
        self._ctx = ctx or default_context()

    @classmethod
    def from_flat(cls, n: int, row_ptr, col_idx, values, ctx: Context | None = None) -> "CsrBTreeMatrix":
        """CsrBTreeMatrix::from_flat (src/graph_csr_btree.rs:57-63): DenseBTreeList::add_from_sorted
        of every row in row order (src/dense_btree.rs:286-293)."""
        row_ptr = np.asarray(row_ptr, np.uint64)
        col_idx = np.asarray(col_idx, np.uint32)
        parts, offs, ilen, pos = [], np.zeros(n, np.uint64), np.zeros(n, np.uint64), 0
        for r in range(n):
            data = col_idx[int(row_ptr[r]):int(row_ptr[r + 1])]
            sep = btree_internal(data)
            parts += [sep, data]
            offs[r] = pos + len(sep)
            ilen[r] = len(sep)
            pos += len(sep) + len(data)
        nodes = np.concatenate(parts) if parts else np.zeros(0, np.uint32)
        return cls(n, nodes, values, row_ptr, offs, ctx, ilen)

    def index(self, r: int, value: int):
        """DenseBTreeList::index (src/dense_btree.rs:306-309): DenseBTree::index within row r."""
        il = int(self.internal_len[r])
        o = int(self.data_off[r]) - il
        return btree_index(self.nodes[o:int(self.data_off[r]) + int(self.data_start[r + 1] - self.data_start[r])], il, value)

    @classmethod
    def from_host(cls, h: HostCsr, ctx: Context | None = None) -> "CsrBTreeMatrix":
        return cls.from_flat(h.n, h.row_ptr, h.col_idx, h.values, ctx)

    def nnz(self) -> int:
        return int(self.data_start[self.n])

    def data(self, r: int) -> np.ndarray:
        """DenseBTreeList::data (src/dense_btree.rs:311-314): the sorted columns of row r."""
        o = int(self.data_off[r])
        return self.nodes[o:o + int(self.data_start[r + 1] - self.data_start[r])]

    def view(self) -> L.BTreeView:
        v = L.BTreeView()
        v.n_rows = v.n_cols = self.n
        v.nnz = self.nnz()
        v.n_nodes = len(self.nodes)
        v.data_start = self.data_start.ctypes.data
        v.data_off = self.data_off.ctypes.data
        v.nodes = self.nodes.ctypes.data
        v.values = self.values.ctypes.data
        v.residency = L.HOST
        return v

    def matmul_par_csr(self, other: "CsrBTreeMatrix") -> CsrMatrix:
        """CsrBTreeMatrix::matmul_par (src/graph_csr_btree.rs:350-479) up to its from_flat: the
        product as a device CsrMatrix."""
        a, b, out = self.view(), other.view(), L.CsrOwned()
        L.check(L.lib().slat_spgemm_btree(self._ctx.ptr, C.byref(a), C.byref(b), C.byref(out), 0), self._ctx.ptr)
        return CsrMatrix(out, self._ctx)

    def matmul_par(self, other: "CsrBTreeMatrix") -> "CsrBTreeMatrix":
        """CsrBTreeMatrix::matmul_par, the output's trees built on the host as the reference does."""
        h = self.matmul_par_csr(other).host()
        return CsrBTreeMatrix.from_flat(self.n, h.row_ptr, h.col_idx, h.values, self._ctx)
