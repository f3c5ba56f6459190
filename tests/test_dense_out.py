"""Sparse x sparse with a dense output: einsum_sparse_driven
(einsum-dyn/src/sparse.rs:70-148). CPU: the oracle against the reference's own tests
(sparse.rs:1127-1161). GPU (marked): slat_spgemm_dense against the oracle, bit-exact for plain
(wrapping) u32 and for f64 (the reference's left fold), both output orientations, untouched
entries kept."""
import numpy as np
import pytest

import oracle_py as O
import slat


def naive(n, ta, tb):
    a = np.zeros((n, n), np.uint64)
    b = np.zeros((n, n), np.uint64)
    for r, c, v in ta:
        a[r, c] += v
    for r, c, v in tb:
        b[r, c] += v
    return (a @ b).astype(np.uint32)


def coo(n, t, dtype=O.U32):
    t = np.asarray(t).reshape(-1, 3)
    return O.from_coo(n, t[:, 0], t[:, 1], t[:, 2], dtype)


def test_oracle_reference_cases():
    ta = [(0, 1, 2), (0, 2, 3), (1, 3, 1), (2, 3, 4)]
    tb = [(1, 0, 5), (2, 0, 6), (3, 1, 7)]
    out = O.einsum_sparse_driven(coo(4, ta), coo(4, tb), np.zeros((4, 4), np.uint32))
    np.testing.assert_array_equal(out, naive(4, ta, tb))  # sparse.rs:1127-1146
    ident = O.einsum_sparse_driven(coo(3, [(0, 1, 5), (1, 2, 3), (2, 0, 7)]),
                                   coo(3, [(0, 0, 1), (1, 1, 1), (2, 2, 1)]), np.zeros((3, 3), np.uint32))
    assert ident[0, 1] == 5 and ident[1, 2] == 3 and ident[2, 0] == 7 and ident[0, 0] == 0  # :1148-1161


def test_oracle_touched_entries_only_and_transpose():
    a = coo(3, [(0, 1, 2)])
    b = coo(3, [(1, 2, 3)])
    out = np.full((3, 3), 9, np.uint32)
    O.einsum_sparse_driven(a, b, out)
    assert out.tolist() == [[9, 9, 6], [9, 9, 9], [9, 9, 9]]
    out_t = np.full((3, 3), 9, np.uint32)
    O.einsum_sparse_driven(a, b, out_t, transpose=True)
    assert out_t.tolist() == [[9, 9, 9], [9, 9, 9], [6, 9, 9]]


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def rand_pair(n, nnz, dtype, seed):
    g = np.random.default_rng(seed)
    mk = lambda: (g.integers(0, n, nnz), g.integers(0, n, nnz))  # noqa: E731
    (ra, ca), (rb, cb) = mk(), mk()
    if dtype == O.F64:
        va, vb = g.standard_normal(nnz), g.standard_normal(nnz)
    else:
        va, vb = g.integers(1, 1 << 31, nnz), g.integers(1, 1 << 31, nnz)  # products and sums wrap
    return O.from_coo(n, ra, ca, va, dtype), O.from_coo(n, rb, cb, vb, dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [O.U32, O.F64])
@pytest.mark.parametrize("transpose", [False, True])
@pytest.mark.parametrize("n,nnz", [(5, 8), (300, 3000), (2000, 60_000)])
def test_dense_out_matches_oracle(ctx, dtype, transpose, n, nnz):
    oa, ob = rand_pair(n, nnz, dtype, n + nnz + dtype)
    cls = slat.CsrMatrix if dtype == O.U32 else slat.CsrF64
    da = cls.from_host(slat.HostCsr(n, *oa.arrays(), dtype), ctx)
    db = cls.from_host(slat.HostCsr(n, *ob.arrays(), dtype), ctx)
    vt = np.uint32 if dtype == O.U32 else np.float64
    init = np.random.default_rng(1).integers(0, 100, (n, n + 3)).astype(vt)  # ld > n, prior content
    want = O.einsum_sparse_driven(oa, ob, init.copy(), transpose)
    got = da.einsum_sparse_driven(db, init.copy(), transpose)
    np.testing.assert_array_equal(got.view(np.uint64) if dtype == O.F64 else got,
                                  want.view(np.uint64) if dtype == O.F64 else want)


def _relisted_pair(dtype):
    """Operands whose running sums pass through 0 in the reference's visiting order (A row entries
    ascending, then the B row): the column is listed twice in nz_cols and ends at 0
    (einsum-dyn/src/sparse.rs:126-143)."""
    if dtype == O.U32:
        big, m1 = 65536, 0xFFFFFFFF
        # (row 0, col 3): 65536*65536 wraps to 0, then +5  -> listed twice -> 0
        # (row 1, col 3): 65536, then 65536*65536 (= +0)   -> listed once  -> 65536
        # (row 2, col 0): 0xFFFFFFFF + 1 = 0, then +7      -> listed twice -> 0
        # (row 3, col 0): 0xFFFFFFFF + 1 = 0 at the end     -> listed once  -> 0 (the sum)
        ta = [(0, 1, big), (0, 2, 1), (1, 1, 1), (1, 4, big), (2, 5, m1), (2, 6, 1), (2, 7, 1), (3, 5, m1), (3, 6, 1)]
        tb = [(1, 3, big), (2, 3, 5), (4, 3, big), (5, 0, 1), (6, 0, 1), (7, 0, 7), (1, 2, 5)]
    else:
        # row 0: 1.5 - 1.5 + 2 -> 0 ; row 1: 2 + 1.5 - 1.5 -> 2 ; row 2: 1e16 + 1 - 1e16 (not exact 0 midway)
        ta = [(0, 1, 1.5), (0, 2, -1.5), (0, 4, 2.0), (1, 4, 2.0), (1, 5, 1.5), (1, 6, -1.5), (2, 7, 1e16), (2, 8, 1.0),
              (2, 9, -1e16)]
        tb = [(1, 3, 1.0), (2, 3, 1.0), (4, 3, 1.0), (5, 3, 1.0), (6, 3, 1.0), (7, 3, 1.0), (8, 3, 1.0), (9, 3, 1.0)]
    n = 10
    return coo(n, ta, dtype), coo(n, tb, dtype)


def test_oracle_relisted_columns_end_at_zero():
    for dtype in (O.U32, O.F64):
        oa, ob = _relisted_pair(dtype)
        vt = np.uint32 if dtype == O.U32 else np.float64
        out = O.einsum_sparse_driven(oa, ob, np.full((10, 10), 9, vt))
        if dtype == O.U32:
            assert (out[0, 3], out[1, 3], out[2, 0], out[3, 0]) == (0, 65536, 0, 0)
            assert out[1, 2] == 5 and out[0, 2] == 65536 * 5 and out[0, 0] == 9
        else:
            assert out[0, 3] == 0.0 and out[1, 3] == 2.0 and out[2, 3] == (1e16 + 1.0) - 1e16


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [O.U32, O.F64])
@pytest.mark.parametrize("transpose", [False, True])
def test_dense_out_relisted_columns(ctx, dtype, transpose):
    # u32 65536*65536 wraps and f64 +x/-x cancellations: bit-exact with the oracle's listing semantics
    oa, ob = _relisted_pair(dtype)
    cls = slat.CsrMatrix if dtype == O.U32 else slat.CsrF64
    da = cls.from_host(slat.HostCsr(10, *oa.arrays(), dtype), ctx)
    db = cls.from_host(slat.HostCsr(10, *ob.arrays(), dtype), ctx)
    vt = np.uint32 if dtype == O.U32 else np.float64
    init = np.full((10, 12), 9, vt)
    want = O.einsum_sparse_driven(oa, ob, init.copy(), transpose)
    got = da.einsum_sparse_driven(db, init.copy(), transpose)
    np.testing.assert_array_equal(got.view(np.uint64) if dtype == O.F64 else got,
                                  want.view(np.uint64) if dtype == O.F64 else want)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [O.U32, O.F64])
@pytest.mark.parametrize("transpose", [False, True])
def test_dense_out_frequent_cancellation(ctx, dtype, transpose):
    # values +-1 (f64) / 1 and 0xFFFFFFFF (u32 wrap): running sums hit 0 all the time
    g = np.random.default_rng(7 + dtype)
    n, nnz = 400, 6000
    if dtype == O.F64:
        va, vb = g.choice([1.0, -1.0], nnz), g.choice([1.0, -1.0, 2.0], nnz)
    else:
        va, vb = g.choice([1, 0xFFFFFFFF, 65536], nnz), g.choice([1, 0xFFFFFFFF, 65536], nnz)
    oa = O.from_coo(n, g.integers(0, n, nnz), g.integers(0, n, nnz), va, dtype)
    ob = O.from_coo(n, g.integers(0, n, nnz), g.integers(0, n, nnz), vb, dtype)
    cls = slat.CsrMatrix if dtype == O.U32 else slat.CsrF64
    da = cls.from_host(slat.HostCsr(n, *oa.arrays(), dtype), ctx)
    db = cls.from_host(slat.HostCsr(n, *ob.arrays(), dtype), ctx)
    vt = np.uint32 if dtype == O.U32 else np.float64
    init = np.full((n, n), 3, vt)
    want = O.einsum_sparse_driven(oa, ob, init.copy(), transpose)
    got = da.einsum_sparse_driven(db, init.copy(), transpose)
    np.testing.assert_array_equal(got.view(np.uint64) if dtype == O.F64 else got,
                                  want.view(np.uint64) if dtype == O.F64 else want)


@pytest.mark.gpu
def test_dense_out_torus_equals_saturating_product_when_no_overflow(ctx):
    # small counts: plain u32 = Saturating<u32>, so the dense output equals densify(A*A)
    t = O.torus_thinned(12, 3.0, O.Rng())
    d = slat.CsrMatrix.from_host(slat.HostCsr(t.n, *t.arrays(), O.U32), ctx)
    dense = d.einsum_sparse_driven(d)
    h = d.matmul(d).host()
    want = np.zeros((t.n, t.n), np.uint32)
    rows = np.repeat(np.arange(t.n), np.diff(h.row_ptr).astype(np.int64))
    want[rows, h.col_idx] = h.values
    np.testing.assert_array_equal(dense, want)


@pytest.mark.gpu
def test_dense_out_rejects_sat64(ctx):
    m = slat.MagnusMatrix.from_host(slat.HostCsr(2, [0, 1, 1], [1], [3], O.SAT64), ctx)
    with pytest.raises(Exception):
        m.einsum_sparse_driven(m)
