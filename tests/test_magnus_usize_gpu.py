"""MagnusMatrix in the reference's own layout (src/graph_magnus.rs:11-14: usize column ids, Sat64
values) through slat_magnus_matmul: u64 columns in and out, bit-exact against the oracle's Sat64
CSR product (the MagnusMatrix results equal CsrMatrix's on Sat64, src/graph_magnus.rs:751-753)."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu


def _arrays(o: O.Csr):
    rp, col, val = o.arrays()
    return rp.astype(np.uint64), col.astype(np.uint64), val.astype(np.uint64)


def _check(got: slat.MagnusMatrixUsize, want: O.Csr):
    rp, col, val = got.host()
    wrp, wcol, wval = want.arrays()
    assert got.nnz() == want.nnz
    assert col.dtype == np.uint64
    np.testing.assert_array_equal(rp, wrp)
    np.testing.assert_array_equal(col, wcol.astype(np.uint64))
    np.testing.assert_array_equal(val, wval)


@pytest.mark.parametrize("side,epn", [(10, 3.0), (30, 3.0)])
def test_torus_chain_usize_cols(side, epn):
    A = O.convert(O.torus_thinned(side, epn, O.Rng()), O.SAT64)
    a = _arrays(A)
    va = slat.MagnusMatrixUsize.host_view(A.n, *a)
    P = slat.MagnusMatrixUsize.matmul_host(va, va)
    want = O.matmul_seq(A, A)
    _check(P, want)
    for _ in range(2):  # A^3, A^4: device-resident left operand, host right operand
        P = slat.MagnusMatrixUsize.matmul_host(P.view(), va, P._ctx)
        want = O.matmul_seq(want, A)
        _check(P, want)
    assert P.matmul_seq(P).nnz() == P.matmul(P).nnz()


def test_saturating_values_usize_cols():
    rng = np.random.default_rng(7)
    n, m = 300, 3000
    r = rng.integers(0, n, m)
    c = rng.integers(0, n, m)
    v = rng.integers(1, 2**40, m, dtype=np.uint64)  # products overflow u64: Sat64 clamps
    A = O.from_coo(n, r, c, v, O.SAT64)
    a = _arrays(A)
    va = slat.MagnusMatrixUsize.host_view(n, *a)
    _check(slat.MagnusMatrixUsize.matmul_host(va, va), O.matmul_seq(A, A))


@pytest.mark.parametrize("bad_id", [2**32 + 1, 2, 70_000, 2**32 - 1])
def test_column_out_of_range_is_an_error(bad_id):
    """An id no u32 can hold (2^32 + 1 would wrap to the valid id 1) and ids in [n_cols, 2^32) are
    refused before the product runs, with the context still usable afterwards."""
    rp = np.array([0, 1, 1], np.uint64)
    col = np.array([bad_id], np.uint64)
    val = np.array([1], np.uint64)
    v = slat.MagnusMatrixUsize.host_view(2, rp, col, val)
    with pytest.raises(slat.SlatError) as e:
        slat.MagnusMatrixUsize.matmul_host(v, v)
    assert e.value.status == 1  # SLAT_EINVAL (the reference would index out of bounds and panic)
    # a wide B (80 000 columns: the LDS-hash and window categories) with one id past n_cols in A
    n = 80_000
    brp = np.arange(n + 1, dtype=np.uint64)
    bcol = np.arange(n, dtype=np.uint64)[::-1].copy()
    one = np.ones(n, np.uint64)
    vb = slat.MagnusMatrixUsize.host_view(n, brp, bcol, one)
    acol = np.array([5, n + 7], np.uint64)
    va = slat.MagnusMatrixUsize.host_view(n, np.array([0] + [2] * n, np.uint64), acol, np.ones(2, np.uint64))
    with pytest.raises(slat.SlatError) as e:
        slat.MagnusMatrixUsize.matmul_host(va, vb)
    assert e.value.status == 1
    # and a valid product right after the refusals
    A = O.convert(O.torus_thinned(10, 3.0, O.Rng()), O.SAT64)
    a = _arrays(A)
    va = slat.MagnusMatrixUsize.host_view(A.n, *a)
    _check(slat.MagnusMatrixUsize.matmul_host(va, va), O.matmul_seq(A, A))


def test_dimension_mismatch_usize():
    rp = np.zeros(3, np.uint64)
    e = np.zeros(0, np.uint64)
    a = slat.MagnusMatrixUsize.host_view(2, rp, e, e)
    b = slat.MagnusMatrixUsize.host_view(3, np.zeros(4, np.uint64), e, e)
    with pytest.raises(slat.SlatError) as ex:
        slat.MagnusMatrixUsize.matmul_host(a, b)
    assert ex.value.status == 2


def _usize(o: O.Csr):
    rp, col, val = _arrays(o)
    return slat.MagnusMatrixUsize.host_view(o.n, rp, col, val), (rp, col, val)


def test_add_and_drivers_usize_cols():
    """MagnusMatrix::add / reachability_sum / power_until_stable / connected_components
    (src/graph_magnus.rs:245-359) in the usize layout, bit-exact against the oracle's Sat64 restatement
    of the CsrMatrix drivers (the reference's MagnusMatrix versions are the same algorithms)."""
    A = O.convert(O.torus_thinned(8, 3.0, O.Rng()), O.SAT64)
    va, keep = _usize(A)
    M = slat.MagnusMatrixUsize.matmul_host(va, va)  # A^2, device-resident
    got = M.add(M)
    _check(got, O.add(O.matmul_seq(A, A), O.matmul_seq(A, A)))
    ga = slat.MagnusMatrixUsize.add_host(va, va)
    _check(ga, O.add(A, A))
    s, k = ga.reachability_sum()
    ws, wk = O.reachability_sum(O.add(A, A))
    assert k == wk
    _check(s, ws)
    c, k = ga.power_until_stable()
    wc, wk = O.power_until_stable(O.add(A, A))
    assert k == wk
    _check(c, wc)
    assert ga.connected_components() == [int(x) for x in O.connected_components(O.add(A, A))]


def test_saturating_chain_usize():
    """The reference's 64-node chain (I + N) squared until stable (src/graph_csr.rs:931-939 and its
    MagnusMatrix twin): 7 squarings, 1176 entries saturated at u64::MAX in Sat64 (SURVEY.md
    section 8(c), golden 2), bit-exact against the oracle."""
    n = 64
    rows = np.concatenate([np.arange(n), np.arange(n - 1)])
    cols = np.concatenate([np.arange(n), np.arange(1, n)])
    A = O.from_coo(n, rows, cols, np.ones(len(rows), np.uint64), O.SAT64)
    va, keep = _usize(A)
    eye = np.arange(n + 1, dtype=np.uint64), np.arange(n, dtype=np.uint64), np.ones(n, np.uint64)
    dev = slat.MagnusMatrixUsize.matmul_host(va, slat.MagnusMatrixUsize.host_view(n, *eye))  # A on the device
    c, k = dev.power_until_stable()
    wc, wk = O.power_until_stable(A)
    assert k == wk == 7
    _check(c, wc)
    _, _, val = c.host()
    assert int((val == np.uint64(2**64 - 1)).sum()) == 1176
