"""The short-row category of wide launches: batches of consecutive short rows in one LDS hash table
of composite (row, column) keys, emitted by a wave bitonic sort. Bit-exact against the oracle for u32 / Sat64, and
within C5's stated tolerance (rtol 1e-12) for f64 in any order. Cases at the category's edges:
64 / 65 groups and 256 / 257 entries per row, runs of 64 equal keys (every group of the batch
hits the same columns), A entries into empty B rows, explicit zeros and saturation, and one row
per batch when the columns need more than 25 key bits."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu

CLS = {O.U32: slat.CsrMatrix, O.SAT64: slat.MagnusMatrix, O.F64: slat.CsrF64}
SL = {O.U32: slat.U32, O.SAT64: slat.SAT64, O.F64: slat.F64}
NP = {O.U32: np.uint32, O.SAT64: np.uint64, O.F64: np.float64}
N = 80_000  # columns beyond one LDS window: a wide launch


def to_dev(o: O.Csr, cls):
    rp, col, val = o.arrays()
    return cls.from_host(slat.HostCsr(o.n, rp, col, val, cls.DTYPE))


def assert_same(dev, orc: O.Csr, what="", rtol=None):
    h = dev.host()
    rp, col, val = orc.arrays()
    assert dev.nnz() == orc.nnz, f"{what}: nnz {dev.nnz()} != {orc.nnz}"
    np.testing.assert_array_equal(h.row_ptr, rp, err_msg=what)
    np.testing.assert_array_equal(h.col_idx, col, err_msg=what)
    if rtol is not None:
        np.testing.assert_allclose(h.values, val, rtol=rtol, atol=0, err_msg=what)
    elif val.dtype == np.float64:
        np.testing.assert_array_equal(h.values.view(np.uint64), val.view(np.uint64), err_msg=what)
    else:
        np.testing.assert_array_equal(h.values, val, err_msg=what)


def from_rows(n, rows, dtype, rng, vmax=5):
    """CSR from a list of (row, sorted unique columns) with random values in [1, vmax]."""
    lens = np.zeros(n, np.int64)
    cols = []
    for r, c in rows:
        lens[r] = len(c)
    order = sorted(rows, key=lambda x: x[0])
    for _, c in order:
        cols.append(np.asarray(c, np.uint32))
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    col = np.concatenate(cols) if cols else np.zeros(0, np.uint32)
    if dtype == O.F64:
        val = rng.uniform(0.5, 1.5, len(col))
    else:
        val = rng.integers(1, vmax + 1, len(col)).astype(NP[dtype])
    return O.from_arrays(rp, col, val, dtype)


def edge_case_pair(dtype, seed=0):
    """A, B (N x N): B rows of 4 columns (one ELL group) around a few hundred hot rows, some empty;
    A rows sized at the category's limits."""
    rng = np.random.default_rng(seed)
    brows = []
    hot = rng.choice(N, 600, replace=False)
    same4 = np.sort(rng.choice(N, 4, replace=False))
    for i, r in enumerate(hot):
        if i < 70:
            brows.append((int(r), same4))  # 70 B rows hitting the same 4 columns: runs of 64 equal keys
        elif i < 500:
            brows.append((int(r), np.sort(rng.choice(N, rng.integers(1, 5), replace=False))))
        # the remaining hot rows stay empty in B
    B = from_rows(N, brows, dtype, rng)
    same_rows, other_rows, empty_rows = hot[:70], hot[70:500], hot[500:]
    arows = []
    a_specs = [
        np.sort(rng.choice(same_rows, 64, replace=False)),   # 64 groups, every key in runs of 64
        np.sort(rng.choice(same_rows, 65, replace=False)),   # 65 groups: the window launch
        np.sort(rng.choice(other_rows, 64, replace=False)),  # 64 groups of 1..4 columns
        np.sort(np.concatenate([rng.choice(empty_rows, 100, replace=False),
                                rng.choice(other_rows, 20, replace=False)])),
        np.sort(np.concatenate([rng.choice(np.setdiff1d(np.arange(N), hot), 236, replace=False),
                                rng.choice(other_rows, 20, replace=False)])),  # 256 entries, 20 groups
        np.sort(np.concatenate([rng.choice(np.setdiff1d(np.arange(N), hot), 237, replace=False),
                                rng.choice(other_rows, 20, replace=False)])),  # 257 entries: window launch
    ]
    base = 1000
    for j, spec in enumerate(a_specs):
        for rep in range(70):  # many copies: batches of 1..n rows, tiles straddled
            arows.append((base + j * 97 + rep * 1013, spec))
    # plus short random rows everywhere (batches of many rows)
    taken = {r for r, _ in arows}
    for r in rng.choice(N, 20_000, replace=False):
        if int(r) not in taken:
            arows.append((int(r), np.sort(rng.choice(hot, rng.integers(0, 12), replace=False))))
    A = from_rows(N, arows, dtype, rng)
    return A, B


@pytest.mark.parametrize("dtype", [O.U32, O.SAT64])
def test_category_edges_bit_exact(dtype):
    A, B = edge_case_pair(dtype)
    assert_same(to_dev(A, CLS[dtype])._spgemm(to_dev(B, CLS[dtype])), O.matmul_seq(A, B), f"edges {dtype}")


def test_category_edges_f64_any_order():
    A, B = edge_case_pair(O.F64, seed=1)
    got = to_dev(A, slat.CsrF64)._spgemm(to_dev(B, slat.CsrF64), slat.FLAG_F64_ANY_ORDER)
    assert_same(got, O.matmul_seq(A, B), "edges f64 any order", rtol=1e-12)
    # and the ordered f64 numeric after the sorted symbolic: bit-exact
    assert_same(to_dev(A, slat.CsrF64)._spgemm(to_dev(B, slat.CsrF64)), O.matmul_seq(A, B), "edges f64 ordered")


def test_zeros_and_saturation_u32():
    """Explicit zero values (dropped outputs, compaction) and products / sums past 2^32 (clamped)."""
    rng = np.random.default_rng(5)
    t = O.torus_thinned(44, 3.0, O.Rng())  # 85,184 columns: wide
    rp, col, _ = t.arrays()
    val = rng.integers(0, 4, len(col)).astype(np.uint32)  # a quarter zeros
    big = rng.random(len(col)) < 0.05
    val[big] = np.uint32(0xC0000000)
    a = O.from_arrays(rp, col, val, O.U32)
    d = to_dev(a, slat.CsrMatrix)
    assert_same(d._spgemm(d), O.matmul_seq(a, a), "zeros + saturation")


def test_sat64_saturating_sums():
    rng = np.random.default_rng(6)
    t = O.torus_thinned(44, 3.0, O.Rng())
    rp, col, _ = t.arrays()
    val = rng.integers(1, 4, len(col)).astype(np.uint64)
    val[rng.random(len(col)) < 0.1] = np.uint64(1 << 62)
    a = O.from_arrays(rp, col, val, O.SAT64)
    d = to_dev(a, slat.MagnusMatrix)
    assert_same(d._spgemm(d), O.matmul_seq(a, a), "sat64 saturation")


@pytest.mark.parametrize("dtype", [O.U32, O.F64])
def test_one_row_per_batch_past_2_25_columns(dtype):
    """40M columns: composite keys would need > 31 bits, so every batch is one row (cbits 0)."""
    rng = np.random.default_rng(8)
    n, ncols = 5000, 40_000_000
    ar = rng.integers(0, n, 40_000)
    ac = rng.integers(0, n, 40_000)
    key = np.unique(ar.astype(np.int64) * n + ac)
    ar, ac = (key // n).astype(np.int64), (key % n).astype(np.uint32)
    av = rng.integers(1, 4, len(ar)).astype(NP[dtype])
    blen = rng.integers(0, 9, n)
    bc = np.concatenate([np.sort(rng.choice(ncols, k, replace=False)) for k in blen]).astype(np.uint32)
    bv = rng.integers(1, 4, len(bc)).astype(av.dtype)
    Ah = slat.HostCsr(n, np.concatenate([[0], np.cumsum(np.bincount(ar, minlength=n))]).astype(np.uint64), ac, av, SL[dtype])
    Bh = slat.HostCsr(n, np.concatenate([[0], np.cumsum(blen)]).astype(np.uint64), bc, bv, SL[dtype])
    cls = CLS[dtype]
    da, db = cls.from_host(Ah), cls.from_host(Bh)
    vb = db.view()
    vb.n_cols = ncols
    out = slat._lib.CsrOwned()
    va = da.view()
    flags = slat.FLAG_F64_ANY_ORDER if dtype == O.F64 else 0
    slat._lib.check(slat.lib().slat_spgemm(da._ctx.ptr, slat._lib.C.byref(va), slat._lib.C.byref(vb),
                                           slat._lib.C.byref(out), flags), da._ctx.ptr)
    got = cls(out, da._ctx).host()
    import scipy.sparse as sp
    Am = sp.csr_matrix((av.astype(np.float64), ac, Ah.row_ptr.astype(np.int64)), shape=(n, n))
    Bm = sp.csr_matrix((bv.astype(np.float64), bc, Bh.row_ptr.astype(np.int64)), shape=(n, ncols))
    Cm = (Am @ Bm).tocsr()
    Cm.sort_indices()
    np.testing.assert_array_equal(got.row_ptr, Cm.indptr)
    np.testing.assert_array_equal(got.col_idx, Cm.indices)
    np.testing.assert_array_equal(got.values.astype(np.float64), Cm.data)  # small integers: exact in f64


def test_row_bounds_with_long_rows_at_chunk_edges():
    """k_symbolic_short bounds each row's products per 64-row tile from 256-entry chunks of the tile,
    jumping over rows of > 256 entries: long rows starting exactly at a chunk edge or at the tile's
    first entry, empty rows between them, short rows after them."""
    rng = np.random.default_rng(12)
    B = from_rows(N, [(r, np.sort(rng.choice(N, rng.integers(1, 5), replace=False))) for r in range(N)], O.U32, rng)
    sizes = {6400: 256, 6401: 300, 6402: 10, 6403: 0, 6404: 500, 6405: 5, 6406: 251, 6407: 257, 6408: 7,
             6464: 600, 6465: 3, 6466: 256, 6467: 1000, 6468: 2}
    rows = [(r, np.sort(rng.choice(N, k, replace=False))) for r, k in sizes.items() if k]
    taken = set(sizes)
    rows += [(int(r), np.sort(rng.choice(N, rng.integers(1, 30), replace=False)))
             for r in range(6300, 6700) if r not in taken]
    A = from_rows(N, rows, O.U32, rng)
    assert_same(to_dev(A, slat.CsrMatrix)._spgemm(to_dev(B, slat.CsrMatrix)), O.matmul_seq(A, B), "chunk edges")
