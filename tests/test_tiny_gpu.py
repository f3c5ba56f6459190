"""The one-kernel small path (csrc/slat_tiny.hip: one wave per row builds the row's bitmap and ranks,
the blocks' offsets come from a decoupled look-back, then the values are accumulated and emitted, in
one regular launch) against the oracle and against the regular multi-kernel pipeline
(SLAT_FLAG_NO_TINY) on the same inputs: bit-exact for u32 / Sat64 / f64
in the reference's fold order, within rtol 1e-12 for f64 in any order. Small products take the path
by default, so config C3's small cells run through it."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu

DT = {slat.U32: O.U32, slat.SAT64: O.SAT64, slat.F64: O.F64}
CLS = {slat.U32: slat.CsrMatrix, slat.SAT64: slat.MagnusMatrix, slat.F64: slat.CsrF64}
TINY = 4  # slat_stats.mode bit of the one-kernel path


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def to_dev(o: O.Csr, dtype: int):
    rp, col, val = o.arrays()
    return CLS[dtype].from_host(slat.HostCsr(o.n, rp, col, val, dtype))


def arrays(dev):
    h = dev.host()
    return h.row_ptr, h.col_idx, h.values


def check(ctx, a, b, want: O.Csr, what, flags=0, exact=True):
    got = a._spgemm(b, flags)
    assert ctx.stats()["mode"] & TINY, f"{what}: the small path was not taken"
    ref = a._spgemm(b, flags | slat.FLAG_NO_TINY)
    assert not ctx.stats()["mode"] & TINY
    rp, col, val = arrays(got)
    rrp, rcol, rval = arrays(ref)
    wrp, wcol, wval = want.arrays()
    for x, y in ((rp, wrp), (rrp, wrp), (col, wcol), (rcol, wcol)):
        np.testing.assert_array_equal(x, y, err_msg=what)
    if exact:
        if val.dtype == np.float64:
            np.testing.assert_array_equal(val.view(np.uint64), wval.view(np.uint64), err_msg=what)
            np.testing.assert_array_equal(rval.view(np.uint64), wval.view(np.uint64), err_msg=what)
        else:
            np.testing.assert_array_equal(val, wval, err_msg=what)
            np.testing.assert_array_equal(rval, wval, err_msg=what)
    else:
        np.testing.assert_allclose(val, wval, rtol=1e-12, err_msg=what)
        np.testing.assert_allclose(rval, wval, rtol=1e-12, err_msg=what)
    return got


@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64, slat.F64])
@pytest.mark.parametrize("side", [4, 5, 10])
def test_torus_chain(ctx, dtype, side):
    A = O.convert(O.torus_thinned(side, 3.0, O.Rng()), DT[dtype])
    da = to_dev(A, dtype)
    want, dp = A, da
    for k in range(2, 5):
        want = O.matmul_seq(want, A)
        dp = check(ctx, dp, da, want, f"side {side} A^{k} dtype {dtype}")


def test_f64_any_order(ctx):
    rng = np.random.default_rng(3)
    n = 700
    r, c = rng.integers(0, n, 5000), rng.integers(0, n, 5000)
    A = O.from_coo(n, r, c, rng.standard_normal(5000) + 2.0, O.F64)
    d = to_dev(A, slat.F64)
    check(ctx, d, d, O.matmul_seq(A, A), "f64 any order", slat.FLAG_F64_ANY_ORDER, exact=False)


def test_ragged_and_empty_rows(ctx):
    rng = np.random.default_rng(9)
    n = 2000  # the small path takes <= 2048 rows
    r = rng.integers(0, n, 6000)
    r = r[r % 7 != 0]  # every 7th row of A empty
    a = O.from_coo(n, r, rng.integers(0, n, len(r)), rng.integers(1, 100, len(r)), O.U32)
    br = rng.integers(0, n, 4000)
    br = br[br % 5 != 0]  # and every 5th row of B
    b = O.from_coo(n, br, rng.integers(0, n, len(br)), rng.integers(1, 100, len(br)), O.U32)
    check(ctx, to_dev(a, slat.U32), to_dev(b, slat.U32), O.matmul_seq(a, b), "ragged")


def test_explicit_zeros_dropped(ctx):
    # zero inputs (raw arrays only) and zero products drop out of the rows; the compaction that
    # follows the one-kernel path reads its non-zero counts
    rp = np.array([0, 2, 3, 4, 4], np.uint64)
    col = np.array([0, 1, 2, 1], np.uint32)
    val = np.array([0, 5, 0, 3], np.uint32)
    A = slat.CsrMatrix.from_host(slat.HostCsr(4, rp, col, val, slat.U32))
    got = A.matmul(A)
    assert ctx.stats()["mode"] & TINY
    ref = A._spgemm(A, slat.FLAG_NO_TINY)
    for x, y in zip(arrays(got), arrays(ref)):
        np.testing.assert_array_equal(x, y)
    assert 0 not in set(arrays(got)[2].tolist())


def test_f64_cancellation(ctx):
    A = O.from_coo(3, [0, 0, 1], [1, 2, 2], np.array([1.0, 1.0, 2.0]), O.F64)
    B = O.from_coo(3, [1, 1, 2, 2], [0, 1, 1, 2], np.array([3.0, 1.5, -1.5, 4.0]), O.F64)
    check(ctx, to_dev(A, slat.F64), to_dev(B, slat.F64), O.matmul_seq(A, B), "cancellation")


def test_saturating_values(ctx):
    n = 40
    rows = np.repeat(np.arange(n), n)
    cols = np.tile(np.arange(n), n)
    v = np.full(n * n, 0x10000, np.uint64)
    v[::3] = 0xFFFFFFFF
    o = O.from_coo(n, rows, cols, v, O.U32)
    check(ctx, to_dev(o, slat.U32), to_dev(o, slat.U32), O.matmul_seq(o, o), "u32 saturation")
    v64 = np.full(n * n, 1 << 40, np.uint64)
    v64[::5] = (1 << 63) + 12345
    o = O.from_coo(n, rows, cols, v64, O.SAT64)
    check(ctx, to_dev(o, slat.SAT64), to_dev(o, slat.SAT64), O.matmul_seq(o, o), "sat64 saturation")


def test_row_block(ctx):
    A = O.torus_thinned(10, 3.0, O.Rng())
    d = to_dev(A, slat.U32)
    full = O.matmul_seq(A, A)
    rp, col, val = full.arrays()
    lo, hi = 137, 611
    got = d.matmul_rowblock(lo, hi, d, 0)
    assert ctx.stats()["mode"] & TINY
    grp, gcol, gval = arrays(got)
    np.testing.assert_array_equal(grp, rp[lo:hi + 1] - rp[lo])
    np.testing.assert_array_equal(gcol, col[rp[lo]:rp[hi]])
    np.testing.assert_array_equal(gval, val[rp[lo]:rp[hi]])


def test_many_calls(ctx):
    # the look-back's epoch-tagged status words are never reset: 400 calls in a row stay correct
    A = O.torus_thinned(5, 3.0, O.Rng())
    d = to_dev(A, slat.U32)
    want = O.matmul_seq(A, A)
    wrp, wcol, wval = want.arrays()
    for i in range(400):
        c = d.matmul(d)
        if i % 97 == 0:
            rp, col, val = arrays(c)
            np.testing.assert_array_equal(rp, wrp)
            np.testing.assert_array_equal(col, wcol)
            np.testing.assert_array_equal(val, wval)
        assert c.nnz() == want.nnz
