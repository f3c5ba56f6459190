"""Speculative wide launches: the listed-row launches (the window rows of the symbolic and numeric
passes) are skipped as if every row were short; a short-row kernel that lists a row voids the call,
which reruns with them, and the (A, B, row block) triple is remembered so the next call does not
speculate. Bar: bit-exact against the oracle in every case, and the stats mode bits (32: the
speculation held, 64: it was voided and rerun) say which path ran."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def to_dev(o: O.Csr, cls=slat.CsrMatrix, dtype=slat.U32):
    rp, col, val = o.arrays()
    return cls.from_host(slat.HostCsr(o.n, rp, col, val, dtype))


def assert_same(dev, orc: O.Csr, what=""):
    h = dev.host()
    rp, col, val = orc.arrays()
    assert dev.nnz() == orc.nnz, f"{what}: nnz {dev.nnz()} != {orc.nnz}"
    np.testing.assert_array_equal(h.row_ptr, rp, err_msg=f"{what} row_ptr")
    np.testing.assert_array_equal(h.col_idx, col, err_msg=f"{what} col_idx")
    np.testing.assert_array_equal(h.values, val, err_msg=f"{what} values")


def mode(ctx):
    return ctx.stats()["mode"]


def test_every_row_short_speculation_holds(ctx):
    # 41^3 = 68,921 columns: a wide launch whose rows are all short (A^2, A^3)
    a = O.torus_thinned(41, 3.0, O.Rng())
    d = to_dev(a)
    o, g = a, d
    for k in (2, 3, 4):
        o = O.matmul_seq(o, a)
        g = g._spgemm(d)
        if k > 2:  # (A * A takes the one-kernel lane path)
            assert mode(ctx) & 32 and not mode(ctx) & 64, f"A^{k}: mode {mode(ctx)}"
        assert_same(g, o, f"41^3 A^{k}")


def rand_b(n, rng, per_row=4):
    # B with at most per_row entries a row (its ELL image applies; max row(A) x max row(B) stays
    # below the fat-row threshold, so no fat-row kernel follows and the call may speculate)
    r = np.repeat(np.arange(n), per_row)
    return O.from_coo(n, r, rng.integers(0, n, len(r)), rng.integers(1, 20, len(r)), O.U32)


def test_symbolic_listed_row_voids_and_is_remembered(ctx):
    # rows of 250 entries (bound 1000 products > 0.7 * 1024: symbolic's window category): the first
    # call is voided and rerun, the second goes straight to the listed-row launches; both bit-exact
    rng = np.random.default_rng(7)
    n = 150_000
    r = np.concatenate([rng.integers(0, n, 200_000), np.repeat(np.array([5, 77_777]), 250)])
    a = O.from_coo(n, r, rng.integers(0, n, len(r)), rng.integers(1, 1000, len(r)), O.U32)
    b = rand_b(n, rng)
    want = O.matmul_seq(a, b)
    d, e = to_dev(a), to_dev(b)
    g = d._spgemm(e)
    assert mode(ctx) & 64 and not mode(ctx) & 32, f"first call: mode {mode(ctx)}"
    assert_same(g, want, "first call (voided, rerun)")
    g = d._spgemm(e)
    assert not mode(ctx) & 96, f"second call: mode {mode(ctx)}"
    assert_same(g, want, "second call (remembered)")


def test_numeric_listed_row_voids(ctx):
    # a row of 120 entries whose B rows hold 3 entries each: 360 products (symbolic's short
    # category, bound 480 <= 716) but ~350 outputs (> 256: numeric's window category)
    rng = np.random.default_rng(19)
    n = 100_000
    r = np.concatenate([np.repeat(np.arange(n), 3), np.full(120, 4242)])
    c = np.concatenate([rng.integers(0, n, 3 * n), rng.choice(n, 120, replace=False)])
    a = O.from_coo(n, r, c, rng.integers(1, 50, len(r)), O.U32)
    b = rand_b(n, rng, 3)
    want = O.matmul_seq(a, b)
    g = to_dev(a)._spgemm(to_dev(b))
    assert mode(ctx) & 64, f"mode {mode(ctx)}"
    assert_same(g, want, "numeric-listed row")


def test_row_blocks_speculate_per_block(ctx):
    # the same operands, row blocks with and without the long rows: each block decides on its own
    rng = np.random.default_rng(23)
    n = 120_000
    r = np.concatenate([rng.integers(0, n, 150_000), np.repeat(np.array([100_000]), 250)])
    a = O.from_coo(n, r, rng.integers(0, n, len(r)), rng.integers(1, 100, len(r)), O.U32)
    b = rand_b(n, rng)
    want = O.matmul_seq(a, b)
    wrp, wcol, wval = want.arrays()
    d, e = to_dev(a), to_dev(b)
    for lo, hi, voided in ((0, 60_000, False), (60_000, n, True), (60_000, n, False)):
        g = d.matmul_rowblock(lo, hi, e)
        m = mode(ctx)
        assert bool(m & 64) == voided, f"[{lo}, {hi}): mode {m}"
        h = g.host()
        s, t = int(wrp[lo]), int(wrp[hi])
        np.testing.assert_array_equal(h.row_ptr, wrp[lo:hi + 1] - wrp[lo])
        np.testing.assert_array_equal(h.col_idx, wcol[s:t])
        np.testing.assert_array_equal(h.values, wval[s:t])
