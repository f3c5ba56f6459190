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
