"""The fat-row category (csrc/slat_fat.hip: rows with >= 8192 products get a workgroup and a dense LDS
accumulator indexed by column), bit-exact against the oracle for every value type, f64 in the
reference's fold order included; f64 in any order within C5's stated tolerance (rtol 1e-12).
Inputs: dense powers of directed R-MAT graphs (thousands of outputs per row), a wide matrix past
2^20 columns (several symbolic passes and accumulator chunks), explicit zeros and cancellation."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu

CLS = {O.U32: slat.CsrMatrix, O.SAT64: slat.MagnusMatrix, O.F64: slat.CsrF64}


def to_dev(o: O.Csr, cls):
    rp, col, val = o.arrays()
    return cls.from_host(slat.HostCsr(o.n, rp, col, val, cls.DTYPE))


def assert_same(dev, orc: O.Csr, what=""):
    h = dev.host()
    rp, col, val = orc.arrays()
    assert dev.nnz() == orc.nnz, f"{what}: nnz {dev.nnz()} != {orc.nnz}"
    np.testing.assert_array_equal(h.row_ptr, rp, err_msg=what)
    np.testing.assert_array_equal(h.col_idx, col, err_msg=what)
    if val.dtype == np.float64:
        np.testing.assert_array_equal(h.values.view(np.uint64), val.view(np.uint64), err_msg=what)
    else:
        np.testing.assert_array_equal(h.values, val, err_msg=what)


def rmat(scale, deg, dtype, seed=42):
    h = slat.host_rmat(scale, (1 << scale) * deg, seed=bytes([seed] * 32))
    if dtype == O.F64:
        v = h.values
    else:
        v = (np.arange(h.nnz, dtype=np.uint64) % 5 + 1).astype(np.uint32 if dtype == O.U32 else np.uint64)
    return O.from_arrays(h.row_ptr, h.col_idx, v, dtype)


def max_products(a: O.Csr, b: O.Csr) -> int:
    arp, acol, _ = a.arrays()
    blen = np.diff(b.arrays()[0].astype(np.int64))
    per = blen[acol.astype(np.int64)]
    cs = np.concatenate([[0], np.cumsum(per)])
    return int((cs[arp[1:].astype(np.int64)] - cs[arp[:-1].astype(np.int64)]).max())


@pytest.mark.parametrize("dtype", [O.U32, O.SAT64, O.F64])
def test_dense_powers_bit_exact(dtype):
    cls = CLS[dtype]
    a = rmat(12, 8, dtype)
    p2 = O.matmul_seq(a, a)
    assert max_products(p2, a) >= 8192  # some rows take the fat-row kernels
    da = to_dev(a, cls)
    dp = to_dev(p2, cls)
    assert_same(dp._spgemm(da), O.matmul_seq(p2, a), "A^2*A")
    assert_same(dp._spgemm(dp), O.matmul_seq(p2, p2), "A^2*A^2")
    assert_same(dp._spgemm(da, slat.FLAG_IDX64), O.matmul_seq(p2, a), "A^2*A idx64")


def test_f64_any_order_within_tolerance():
    a = rmat(12, 16, O.F64)
    da = to_dev(a, slat.CsrF64)
    want = O.matmul_seq(a, a)
    got = da._spgemm(da, slat.FLAG_F64_ANY_ORDER).host()
    wrp, wcol, wval = want.arrays()
    np.testing.assert_array_equal(got.row_ptr, wrp)
    np.testing.assert_array_equal(got.col_idx, wcol)
    np.testing.assert_allclose(got.values, wval, rtol=1e-12, atol=0)


@pytest.mark.parametrize("flags", [0, slat.FLAG_FAT_BUCKETS])
@pytest.mark.parametrize("dtype", [O.U32, O.F64])
def test_wide_fat_rows_past_2_20_columns(dtype, flags):
    """3M columns: symbolic passes of 2^20 columns, accumulator chunks skipped by the touched mask.
    FLAG_FAT_BUCKETS: the same with MAGNUS's fine-level reordering (products bucketed by chunk)."""
    rng = np.random.default_rng(3)
    n, ncols = 64, 3_000_000
    # A: 64 x 64 dense-ish; B: 64 rows, each with 600 random columns spread over 3M
    ar, ac = np.nonzero(rng.random((n, n)) < 0.6)
    av = rng.integers(1, 4, len(ar)).astype(np.uint32 if dtype == O.U32 else np.float64)
    br = np.repeat(np.arange(n), 600)
    bc = np.concatenate([np.sort(rng.choice(ncols, 600, replace=False)) for _ in range(n)])
    bv = rng.integers(1, 4, len(br)).astype(av.dtype)
    A = slat.HostCsr(n, np.concatenate([[0], np.cumsum(np.bincount(ar, minlength=n))]), ac, av,
                     slat.U32 if dtype == O.U32 else slat.F64)
    Bh = slat.HostCsr(n, np.concatenate([[0], np.cumsum(np.bincount(br, minlength=n))]), bc, bv, A.dtype)
    cls = CLS[dtype]
    da, db = cls.from_host(A), cls.from_host(Bh)
    # B is n x ncols: widen its view's column count
    vb = db.view()
    vb.n_cols = ncols
    out = slat._lib.CsrOwned()
    va = da.view()
    slat._lib.check(slat.lib().slat_spgemm(da._ctx.ptr, slat._lib.C.byref(va), slat._lib.C.byref(vb),
                                           slat._lib.C.byref(out), flags), da._ctx.ptr)
    got = cls(out, da._ctx).host()
    # exact restatement: dense rows of the product (small n)
    import scipy.sparse as sp
    Am = sp.csr_matrix((av.astype(np.float64), ac, A.row_ptr.astype(np.int64)), shape=(n, n))
    Bm = sp.csr_matrix((bv.astype(np.float64), bc, Bh.row_ptr.astype(np.int64)), shape=(n, ncols))
    Cm = (Am @ Bm).tocsr()
    Cm.sort_indices()
    np.testing.assert_array_equal(got.row_ptr, Cm.indptr)
    np.testing.assert_array_equal(got.col_idx, Cm.indices)
    np.testing.assert_array_equal(got.values.astype(np.float64), Cm.data)  # small integers: exact in f64


@pytest.mark.parametrize("flags", [0, slat.FLAG_FAT_BUCKETS])
def test_zeros_and_cancellation_in_fat_rows(flags):
    """Explicit zero inputs (u32) and exact f64 cancellation inside fat rows are dropped like
    CsrMatrix::matmul does (src/graph_csr.rs:334, linalg/src/csr.rs:344)."""
    a = rmat(11, 8, O.U32)
    rp, col, val = a.arrays()
    val = val.copy()
    val[::7] = 0
    az = O.from_arrays(rp, col, val, O.U32)
    p2 = O.matmul_seq(a, a)
    assert_same(to_dev(p2, slat.CsrMatrix)._spgemm(to_dev(az, slat.CsrMatrix), flags), O.matmul_seq(p2, az), "u32 zeros")
    f = rmat(11, 8, O.F64)
    frp, fcol, fval = f.arrays()
    fval = fval.copy()
    fval[1::2] *= -1.0  # signed values: sums can cancel exactly
    fs = O.from_arrays(frp, fcol, fval, O.F64)
    fp = O.matmul_seq(fs, fs)
    assert_same(to_dev(fp, slat.CsrF64)._spgemm(to_dev(fs, slat.CsrF64), flags), O.matmul_seq(fp, fs), "f64 signs")
