"""A prepared right operand (slat_bprep_create + slat_spgemm_rowblock_prepared: B's ELL image and value
summary built once) gives bit-identical results to the plain row-block call, which the other tests pin
to the oracle: every value type, row blocks of a wide (1 M-column) launch and of a single-window one,
a B past the ELL limit (no image: the handle carries the view only), and one handle reused by many
calls with other products in between (the context's own per-call image must not disturb it)."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu

CLS = {slat.U32: slat.CsrMatrix, slat.SAT64: slat.MagnusMatrix, slat.F64: slat.CsrF64}


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def to_dev(o: O.Csr, dtype: int):
    rp, col, val = o.arrays()
    return CLS[dtype].from_host(slat.HostCsr(o.n, rp, col, val, dtype))


def same(x, y, what):
    hx, hy = x.host(), y.host()
    np.testing.assert_array_equal(hx.row_ptr, hy.row_ptr, err_msg=f"{what} row_ptr")
    np.testing.assert_array_equal(hx.col_idx, hy.col_idx, err_msg=f"{what} col_idx")
    if hx.values.dtype == np.float64:
        np.testing.assert_array_equal(hx.values.view(np.uint64), hy.values.view(np.uint64), err_msg=f"{what} f64 bits")
    else:
        np.testing.assert_array_equal(hx.values, hy.values, err_msg=f"{what} values")


@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64, slat.F64])
def test_prepared_rowblocks_single_window(ctx, dtype):
    a = O.torus_thinned(16, 3.0, O.Rng())
    a3 = O.matmul_seq(O.matmul_seq(a, a), a)
    P, B = to_dev(a3, dtype), to_dev(a, dtype)
    pb = B.prepare()
    n = a.n
    for lo, hi in [(0, n), (0, 1), (n - 1, n), (n // 3, n // 3 + 700), (5, n - 5)]:
        for flags in (0, slat.FLAG_NO_TINY):
            same(P.matmul_rowblock(lo, hi, pb, flags), P.matmul_rowblock(lo, hi, B, flags), f"[{lo},{hi}) {flags}")
    want = O.matmul_seq(a3, a)
    got = P.matmul_rowblock(0, n, pb, slat.FLAG_NO_TINY).host()
    rp, col, val = want.arrays()
    np.testing.assert_array_equal(got.row_ptr, rp)
    np.testing.assert_array_equal(got.col_idx, col)


def test_prepared_rowblocks_wide_launch_c4_shape(ctx, golden):
    # the 100^3 torus (10^6 columns: the wide launch's short-row categories), A^3 * A by eighths
    # with one prepared B, concatenated and checked against the golden digests of A^4
    A = slat.torus_thinned_device(100, 3.0, slat.StdRng(), ctx)
    P = A.matmul(A).matmul(A)
    pb = A.prepare()
    n = P.n
    rows, cols, vals = [np.zeros(1, np.uint64)], [], []
    base = 0
    for k in range(8):
        lo, hi = k * n // 8, (k + 1) * n // 8
        h = P.matmul_rowblock(lo, hi, pb).host()
        rows.append(h.row_ptr[1:] + base)
        base += int(h.row_ptr[-1])
        cols.append(h.col_idx)
        vals.append(h.values)
    from helpers import assert_digest, digest
    assert_digest(digest(np.concatenate(rows), np.concatenate(cols), np.concatenate(vals)),
                  golden["torus100_powers"][3], "A^4 by prepared eighths")


def test_prepared_b_without_ell_image(ctx):
    # B rows past the ELL limit (a row of 40 entries): the handle has no image; results unchanged
    rng = np.random.default_rng(7)
    n = 3000
    r = rng.integers(0, n, 20000)
    c = rng.integers(0, n, 20000)
    r = np.concatenate([r, np.zeros(40, np.int64)])
    c = np.concatenate([c, np.arange(40) * 50])
    o = O.from_coo(n, r, c, np.ones(len(r), np.uint64), O.U32)
    d = to_dev(o, slat.U32)
    pb = d.prepare()
    for lo, hi in [(0, n), (100, 2000)]:
        same(d.matmul_rowblock(lo, hi, pb, slat.FLAG_NO_TINY), d.matmul_rowblock(lo, hi, d, slat.FLAG_NO_TINY), "no ELL")


def test_prepared_handle_reused_between_other_products(ctx):
    a = O.torus_thinned(20, 3.0, O.Rng())
    A = to_dev(a, slat.U32)
    pb = A.prepare()
    P = A
    for k in range(2, 6):
        other = A.matmul(A)  # a product with its own per-call image in between
        P2 = P.matmul_rowblock(0, P.n, pb, slat.FLAG_NO_TINY)
        same(P2, P.matmul(A), f"A^{k}")
        P = P2
        del other


def test_prepared_wrong_dtype_is_an_error(ctx):
    a = O.torus_thinned(8, 3.0, O.Rng())
    pb = to_dev(a, slat.SAT64).prepare()
    with pytest.raises(TypeError):
        to_dev(a, slat.U32).matmul_rowblock(0, a.n, pb)
