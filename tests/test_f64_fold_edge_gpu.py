"""f64 in the reference's fold order (linalg/src/csr.rs:325-337: each output the left fold from 0.0 of
its products in A-row order) on values whose sums depend on every rounding step: subnormals (the
slot adds are LDS atomic adds, which must neither flush them nor reorder), signed zeros, magnitudes
that cancel, and mixed exponents; through every ordered category (hash rows, window rows, fat rows
with a dense accumulator per column slice). Bar: bit-exact against the oracle's fold."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu

VALS = np.array([5e-324, -5e-324, 1e-310, -1e-310, 2.2e-308, -0.0, 0.0, 1.0, -1.0, 3.0, 1e300, -1e300,
                 0.1, -0.3, 7e-17, 1e16])


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def build(n, rows, cols, seed):
    rng = np.random.default_rng(seed)
    v = VALS[rng.integers(0, len(VALS), len(rows))]
    return O.from_coo(n, rows, cols, v, O.F64)


def same_bits(g, o, what):
    h = g.host()
    rp, col, val = o.arrays()
    assert g.nnz() == o.nnz, f"{what}: nnz {g.nnz()} != {o.nnz}"
    np.testing.assert_array_equal(h.row_ptr, rp, err_msg=f"{what} row_ptr")
    np.testing.assert_array_equal(h.col_idx, col, err_msg=f"{what} col_idx")
    np.testing.assert_array_equal(h.values.view(np.uint64), val.view(np.uint64), err_msg=f"{what} f64 bits")


@pytest.mark.parametrize("n,deg", [(3000, 6), (90_000, 6)])
def test_fold_short_and_window_rows(ctx, n, deg):
    # 3 000 columns: one window (window rows); 90 000: a wide launch (hash rows, listed window rows)
    rng = np.random.default_rng(n)
    m = n * deg
    a = build(n, rng.integers(0, n, m), rng.integers(0, min(n, 400), m), 3)  # few columns: many collisions
    d = slat.CsrF64.from_host(slat.HostCsr(a.n, *a.arrays(), slat.F64))
    same_bits(d._spgemm(d), O.matmul_seq(a, a), f"n={n}")


def test_fold_fat_rows(ctx):
    # hub rows of 2 000 entries over B rows of ~24 entries in 6 000 columns: ~48 000 products a row,
    # fat rows (the per-slice ordered walk), many products per column
    rng = np.random.default_rng(17)
    n = 20_000
    r = rng.integers(0, n, n * 4)
    c = rng.integers(0, 6000, n * 4)
    hubs = np.repeat(np.array([7, 4321, 19_999]), 2000)
    rows = np.concatenate([r, hubs, np.repeat(np.arange(6000), 20)])
    cols = np.concatenate([c, rng.integers(0, 6000, len(hubs)), rng.integers(0, 6000, 6000 * 20)])
    a = build(n, rows, cols, 5)
    d = slat.CsrF64.from_host(slat.HostCsr(a.n, *a.arrays(), slat.F64))
    same_bits(d._spgemm(d), O.matmul_seq(a, a), "fat rows")
