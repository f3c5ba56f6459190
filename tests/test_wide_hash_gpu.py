"""Wide launches (more columns than one LDS window): the MAGNUS-style row categories. Short rows
accumulate in the per-wave LDS hash table (symbolic: product bound <= 0.7 * 1024 keys; numeric:
outputs <= 256) and emit by rank-by-count; the rest take row-span windows that skip untouched
column chunks. Bar: bit-exact against the oracle (u32 / Sat64 / f64) and, at full size, the
golden digests of the 100^3 torus powers (config C4: A^4 = A^3 * A, 57,288,151 nnz)."""
import numpy as np
import pytest

import oracle_py as O
import slat
from helpers import assert_digest, digest

pytestmark = pytest.mark.gpu

DT = {slat.U32: O.U32, slat.SAT64: O.SAT64, slat.F64: O.F64}
CLS = {slat.U32: slat.CsrMatrix, slat.SAT64: slat.MagnusMatrix, slat.F64: slat.CsrF64}


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def to_dev(o: O.Csr, dtype: int):
    rp, col, val = o.arrays()
    return CLS[dtype].from_host(slat.HostCsr(o.n, rp, col, val, dtype))


def assert_same(dev, orc: O.Csr, what=""):
    h = dev.host()
    rp, col, val = orc.arrays()
    assert dev.nnz() == orc.nnz, f"{what}: nnz {dev.nnz()} != {orc.nnz}"
    np.testing.assert_array_equal(h.row_ptr, rp, err_msg=f"{what} row_ptr")
    np.testing.assert_array_equal(h.col_idx, col, err_msg=f"{what} col_idx")
    if val.dtype == np.float64:
        np.testing.assert_array_equal(h.values.view(np.uint64), val.view(np.uint64), err_msg=f"{what} f64 bits")
    else:
        np.testing.assert_array_equal(h.values, val, err_msg=f"{what} values")


@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64, slat.F64])
def test_torus41_powers_hash_rows(ctx, dtype):
    # 41^3 = 68,921 columns > 63,488: a wide launch; every row is short (hash path), rows near the
    # torus boundary wrap around the column range
    a = O.convert(O.torus_thinned(41, 3.0, O.Rng()), DT[dtype])
    if dtype == slat.F64:  # non-trivial values: the f64 fold order matters
        rp, col, _ = a.arrays()
        a = O.from_arrays(rp, col, np.random.default_rng(3).uniform(0.5, 1.5, len(col)), O.F64)
    d = to_dev(a, dtype)
    o, g = a, d
    for k in range(2, 6):
        o = O.matmul_seq(o, a)
        g = g._spgemm(d)
        assert_same(g, o, f"41^3 A^{k} dtype={dtype}")


@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64, slat.F64])
def test_wide_mixed_short_and_long_rows(ctx, dtype):
    # n = 150,000: most rows short (hash), a few rows with thousands of products over the whole
    # column range (window fallback, chunk skipping), some rows empty
    rng = np.random.default_rng(7)
    n = 150_000
    r = rng.integers(0, n, 200_000)
    c = rng.integers(0, n, 200_000)
    heavy = np.repeat(np.array([5, 77_777, 149_999]), 3000)
    r = np.concatenate([r, heavy])
    c = np.concatenate([c, rng.integers(0, n, len(heavy))])
    v = rng.integers(1, 1000, len(r)) if dtype != slat.F64 else rng.uniform(-1.0, 1.0, len(r))
    a = O.from_coo(n, r, c, v, DT[dtype])
    d = to_dev(a, dtype)
    assert_same(d._spgemm(d), O.matmul_seq(a, a), f"mixed dtype={dtype}")


def test_wide_clustered_row_windows_skip_gaps(ctx):
    # rows whose columns sit in two far-apart clusters (0..5k and n-5k..n): > 256 outputs, so the
    # numeric pass takes windows, which must skip the empty middle without missing a column
    rng = np.random.default_rng(11)
    n = 400_000
    rows = np.repeat(np.arange(0, 40), 400)
    cols = np.concatenate([rng.integers(0, 5000, 200) if i % 2 else rng.integers(n - 5000, n, 200)
                           for i in range(len(rows) // 200)])
    a = O.from_coo(n, rows, cols, np.ones(len(rows)), O.U32)
    eye_ish = O.from_coo(n, np.arange(n), np.arange(n), np.full(n, 2), O.U32)
    d, e = to_dev(a, slat.U32), to_dev(eye_ish, slat.U32)
    assert_same(d._spgemm(e), O.matmul_seq(a, eye_ish), "clustered rows")


def test_torus100_a4_golden(ctx, golden):
    # config C4 at full size on one GPU: A^2, A^3, A^4 of the 100^3 torus against the digests
    A = slat.CsrMatrix.from_host(slat.torus_thinned(100, 3.0, slat.StdRng()))
    P = A
    for want in golden["torus100_powers"][1:]:
        P = P.matmul(A)
        h = P.host()
        assert_digest(digest(h.row_ptr, h.col_idx, h.values), want, f"100^3 A^{want['k']}")
