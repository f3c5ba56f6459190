"""Single-window MODE 4 launches with the row offsets folded into the two passes (no k_scan_rows):
k_symbolic's blocks of R consecutive rows store their count sums, the last block turns them into
prefixes (and stores nnz / the max row), and k_numeric takes each row's slice from its group's prefix
plus the counts before it, storing row_ptr itself. R = max(8, ceil(n / 4096)), folded while R <= 64.
Bar: bit-exact against the oracle (CsrMatrix::matmul, src/graph_csr.rs:306-346) for row blocks of
every group shape (partial last group, one group, thousands), tall left operands up to R = 64 and past
it (the scan again), and the zero-drop compaction after a folded call; stats mode bit 128 says which."""
import ctypes as C

import numpy as np
import pytest

import oracle_py as O
import slat
from slat import _lib as L

pytestmark = pytest.mark.gpu

N = 40_000  # one LDS window


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def rand_rows(rng, nrows, ncols, lens, vals=3):
    lens = np.asarray(lens, np.int64)
    rows = np.repeat(np.arange(nrows), lens)
    cols = np.concatenate([rng.choice(ncols, int(k), replace=False) for k in lens if k]) if lens.sum() else []
    return rows, np.asarray(cols, np.int64), rng.integers(1, vals + 1, len(rows))


def mode(ctx):
    return ctx.stats()["mode"]


def test_fold_row_blocks(ctx):
    rng = np.random.default_rng(29)
    r, c, v = rand_rows(rng, N, N, rng.integers(0, 200, N))
    a = O.from_coo(N, r, c, v, O.U32)
    rb, cb, vb = rand_rows(rng, N, N, rng.integers(1, 7, N), 1)
    b = O.from_coo(N, rb, cb, vb, O.U32)
    want = O.matmul_seq(a, b)
    wrp, wcol, wval = want.arrays()
    rp, col, val = a.arrays()
    A = slat.CsrMatrix.from_host(slat.HostCsr(N, rp, col, val, slat.U32))
    brp, bcol, bval = b.arrays()
    B = slat.CsrMatrix.from_host(slat.HostCsr(N, brp, bcol, bval, slat.U32))
    # (blocks of <= 2048 rows with <= 8192 columns would take the one-kernel path; these have 40 000)
    for lo, hi in ((0, 2501), (7, 15), (100, 108), (1000, 33_777), (0, N), (N - 4097, N)):
        g = A.matmul_rowblock(lo, hi, B)
        assert mode(ctx) & 128 and mode(ctx) & 16, f"[{lo}, {hi}): mode {mode(ctx):#x}"
        h = g.host()
        s, e = int(wrp[lo]), int(wrp[hi])
        np.testing.assert_array_equal(h.row_ptr, wrp[lo:hi + 1] - wrp[lo], err_msg=f"[{lo}, {hi}) row_ptr")
        np.testing.assert_array_equal(h.col_idx, wcol[s:e], err_msg=f"[{lo}, {hi}) col")
        np.testing.assert_array_equal(h.values, wval[s:e], err_msg=f"[{lo}, {hi}) val")


@pytest.mark.parametrize("tall, folded", [(150_001, True), (262_144, True), (262_145, False)])
def test_fold_tall_left_operand(ctx, tall, folded):
    # A: `tall` rows over N columns (declared tall x tall for the mirror, its view narrowed to N
    # columns), B: N x N. R = ceil(tall / 4096): 37, 64, then 65 (the scan)
    rng = np.random.default_rng(31)
    lens = rng.integers(0, 40, tall)
    r, c, v = rand_rows(rng, tall, N, lens)
    a = O.from_coo(tall, r, c, v, O.U32)
    rb, cb, vb = rand_rows(rng, N, N, rng.integers(1, 6, N), 1)
    b_or = O.from_coo(tall, rb, cb, vb, O.U32)  # (the oracle's square B: rows past N empty)
    want = O.matmul_seq(a, b_or)
    rp, col, val = a.arrays()
    A = slat.CsrMatrix.from_host(slat.HostCsr(tall, rp, col, val, slat.U32))
    brp, bcol, bval = O.from_coo(N, rb, cb, vb, O.U32).arrays()
    B = slat.CsrMatrix.from_host(slat.HostCsr(N, brp, bcol, bval, slat.U32))
    va, vb_ = A.view(), B.view()
    va.n_cols = N
    out = L.CsrOwned()
    L.check(L.lib().slat_spgemm(ctx.ptr, C.byref(va), C.byref(vb_), C.byref(out), 0), ctx.ptr)
    assert bool(mode(ctx) & 128) == folded, f"mode {mode(ctx):#x}"
    g = slat.CsrMatrix(out, ctx)
    h = g.host()
    wrp, wcol, wval = want.arrays()
    np.testing.assert_array_equal(h.row_ptr, wrp)
    np.testing.assert_array_equal(h.col_idx, wcol)
    np.testing.assert_array_equal(h.values, wval)


def test_fold_with_dropped_zeros(ctx):
    # explicit zeros in A: outputs whose every term is 0 are dropped after the folded passes (the
    # compaction rebuilds row_ptr from numeric's zero-dropped counts, not symbolic's)
    rng = np.random.default_rng(37)
    r, c, v = rand_rows(rng, N, N, rng.integers(0, 150, N))
    v[rng.random(len(v)) < 0.4] = 0
    a = O.from_coo(N, r, c, v, O.U32)  # (the oracle's from_coo drops zeros: the same product)
    rb, cb, vb = rand_rows(rng, N, N, rng.integers(1, 7, N), 1)
    b = O.from_coo(N, rb, cb, vb, O.U32)
    want = O.matmul_seq(a, b)
    # the device's A keeps its explicit zeros
    order = np.lexsort((c, r))
    rp = np.concatenate([[0], np.cumsum(np.bincount(r, minlength=N))]).astype(np.uint64)
    A = slat.CsrMatrix.from_host(slat.HostCsr(N, rp, c[order], v[order], slat.U32))
    assert (A.host().values == 0).sum() > 0
    brp, bcol, bval = b.arrays()
    B = slat.CsrMatrix.from_host(slat.HostCsr(N, brp, bcol, bval, slat.U32))
    g = A.matmul(B)
    st = ctx.stats()
    assert st["mode"] & 128 and st["dropped_rows"] > 0, st
    h = g.host()
    wrp, wcol, wval = want.arrays()
    np.testing.assert_array_equal(h.row_ptr, wrp)
    np.testing.assert_array_equal(h.col_idx, wcol)
    np.testing.assert_array_equal(h.values, wval)
