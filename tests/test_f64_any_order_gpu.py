"""f64 in any summation order (SLAT_FLAG_F64_ANY_ORDER, config C5 "tolerance-checked"): the same
structure as the reference's left fold (row_ptr, col_idx bit-exact) and values within a relative
1e-12 of the oracle's `Csr<u32,f64>::matmul` (linalg/src/csr.rs:308-356). Positive values (the C5
generator: uniform [0.5, 1.5)) cannot cancel, so the bound is the sum's rounding drift. Covers the
LDS slots, the hash categories, and rows with more outputs than the slots (global accumulation)."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu
RTOL = 1e-12


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def check(got, want, what):
    h = got.host()
    rp, col, val = want.arrays()
    np.testing.assert_array_equal(h.row_ptr, rp, err_msg=f"{what} row_ptr")
    np.testing.assert_array_equal(h.col_idx, col, err_msg=f"{what} col_idx")
    np.testing.assert_allclose(h.values, val, rtol=RTOL, atol=0, err_msg=f"{what} values")


@pytest.mark.parametrize("scale,deg", [(10, 8), (12, 10), (16, 4)])
def test_rmat_any_order_within_tolerance(ctx, scale, deg):
    # scale 16: 65,536 columns (a wide launch), power-law rows with thousands of outputs (beyond
    # the LDS slots: global accumulation)
    h = slat.host_rmat(scale, (1 << scale) * deg)
    o = O.from_arrays(h.row_ptr, h.col_idx, h.values, O.F64)
    d = slat.CsrF64.from_host(h)
    check(d._spgemm(d, slat.FLAG_F64_ANY_ORDER), O.matmul_seq(o, o), f"rmat {scale}/{deg}")


def test_any_order_dense_rows_torus(ctx):
    # rows of 3000+ distinct outputs in a one-window launch
    rng = np.random.default_rng(2)
    n = 6000
    r = np.concatenate([np.zeros(400, np.int64), rng.integers(0, n, 20000)])
    c = np.concatenate([rng.choice(n, 400, replace=False), rng.integers(0, n, 20000)])
    a = O.from_coo(n, r, c, rng.uniform(0.5, 1.5, len(r)), O.F64)
    d = slat.CsrF64.from_host(slat.HostCsr(n, *a.arrays(), slat.F64))
    check(d._spgemm(d, slat.FLAG_F64_ANY_ORDER), O.matmul_seq(a, a), "dense rows")


def test_any_order_exact_cancellation_dropped(ctx):
    A = O.from_coo(3, [0, 0, 1], [1, 2, 2], np.array([1.0, 1.0, 2.0]), O.F64)
    B = O.from_coo(3, [1, 1, 2, 2], [0, 1, 1, 2], np.array([3.0, 1.5, -1.5, 4.0]), O.F64)
    da = slat.CsrF64.from_host(slat.HostCsr(3, *A.arrays(), slat.F64))
    db = slat.CsrF64.from_host(slat.HostCsr(3, *B.arrays(), slat.F64))
    got = da._spgemm(db, slat.FLAG_F64_ANY_ORDER)
    want = O.matmul_seq(A, B)
    check(got, want, "cancellation")


def test_rmat_scale18_c5_size(ctx):
    # SURVEY §8(d) C5 at its stated size: R-MAT 2^18 rows, degree 16 (1.28 G outputs). The
    # reference's fold order bit-exact and the any-order mode within rtol 1e-12, both against one
    # oracle product (matmul_par, 16 threads)
    h = slat.host_rmat(18, (1 << 18) * 16)
    o = O.from_arrays(h.row_ptr, h.col_idx, h.values, O.F64)
    d = slat.CsrF64.from_host(h)
    del h
    want = O.matmul_par(o, o, 16)
    rp, col, val = want.arrays()
    for flags in (0, slat.FLAG_F64_ANY_ORDER):
        got = d._spgemm(d, flags).host()
        np.testing.assert_array_equal(got.row_ptr, rp, err_msg=f"scale 18 flags={flags} row_ptr")
        np.testing.assert_array_equal(got.col_idx, col, err_msg=f"scale 18 flags={flags} col_idx")
        if flags:
            np.testing.assert_allclose(got.values, val, rtol=RTOL, atol=0, err_msg="scale 18 any order")
        else:
            np.testing.assert_array_equal(got.values.view(np.uint64), val.view(np.uint64), err_msg="scale 18 fold bits")
        del got
