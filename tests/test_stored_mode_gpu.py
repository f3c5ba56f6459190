"""The single-window numeric pass over stored bitmaps (k_numeric MODE 4, csrc/spgemm_stored.hpp):
bit-exact against the oracle (CsrMatrix::matmul, src/graph_csr.rs:306-346) for u32 / Sat64, and within
C5's stated tolerance (rtol 1e-12) for f64 in any order. Each case checks that the call took MODE 4
(stats mode bit 16) and covers one of its paths:
  * pattern B under the narrow bound (the preloaded first segment, the 30^3 chain's case), rows of
    more than one 512-entry segment, rows touching more than 8 stored bitmap blocks;
  * more tail groups than the LDS queue holds (the per-entry walk);
  * rank chunks after the first (rows of more outputs than the LDS slots);
  * a B with other values, sums past 2^32 (wide slots), Sat64 values past 2^32, f64 any order;
  * empty rows, entries into empty B rows, explicit zeros (dropped, as matmul's `v != 0`)."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu

CLS = {O.U32: slat.CsrMatrix, O.SAT64: slat.MagnusMatrix, O.F64: slat.CsrF64}
NP = {O.U32: np.uint32, O.SAT64: np.uint64, O.F64: np.float64}
N = 40_000  # one LDS window (<= 63 488 columns), 20 bitmap blocks of 2048 columns


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def to_dev(o: O.Csr, cls):
    rp, col, val = o.arrays()
    return cls.from_host(slat.HostCsr(o.n, rp, col, val, cls.DTYPE))


def rand_csr(rng, lens, dtype, vals, n=N, spread=True):
    """n x n CSR with lens[r] distinct sorted columns per row; vals: 'one', an int v (values in
    [1, v]), 'big' (u32 values up to 2^31; Sat64 up to 2^40), 'f64' ([0.5, 1.5))."""
    lens = np.asarray(lens, np.int64)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    cols = []
    for r, k in enumerate(lens):
        if k == 0:
            continue
        if spread:
            c = rng.choice(n, size=int(k), replace=False)
        else:  # a band around the row: neighbouring rows share columns (as a torus power)
            lo = max(0, min(n - int(k) * 2, r - int(k)))
            c = lo + rng.choice(2 * int(k), size=int(k), replace=False)
        cols.append(np.sort(c).astype(np.uint32))
    col = np.concatenate(cols) if cols else np.zeros(0, np.uint32)
    m = len(col)
    if vals == "one":
        val = np.ones(m, NP[dtype])
    elif vals == "big":
        hi = 1 << 31 if dtype == O.U32 else 1 << 40
        val = rng.integers(1, hi, m, dtype=np.uint64).astype(NP[dtype])
    elif vals == "f64":
        val = rng.uniform(0.5, 1.5, m)
    else:
        val = rng.integers(1, int(vals) + 1, m).astype(NP[dtype])
    return O.from_arrays(rp, col, val, dtype)


def check(ctx, a: O.Csr, b: O.Csr, dtype, flags=0, rtol=None, what=""):
    cls = CLS[dtype]
    A, B = to_dev(a, cls), to_dev(b, cls)
    C = A._spgemm(B, flags)
    mode = ctx.stats()["mode"]
    assert mode & 16, f"{what}: MODE 4 not taken (stats mode {mode:#x})"
    ref = O.matmul_seq(a, b)
    h = C.host()
    rp, col, val = ref.arrays()
    assert C.nnz() == ref.nnz, f"{what}: nnz {C.nnz()} != {ref.nnz}"
    np.testing.assert_array_equal(h.row_ptr, rp, err_msg=what)
    np.testing.assert_array_equal(h.col_idx, col, err_msg=what)
    if rtol is not None:
        np.testing.assert_allclose(h.values, val, rtol=rtol, atol=0, err_msg=what)
    elif val.dtype == np.float64:
        np.testing.assert_array_equal(h.values.view(np.uint64), val.view(np.uint64), err_msg=what)
    else:
        np.testing.assert_array_equal(h.values, val, err_msg=what)
    return h


def a_lens(rng, n=N):
    """Mostly rows of 0-300 entries, some of 513-1100 (two or three segments), some empty."""
    lens = rng.integers(0, 300, n)
    lens[rng.choice(n, 300, replace=False)] = rng.integers(513, 1100, 300)
    lens[rng.choice(n, 500, replace=False)] = 0
    return lens


def b_lens(rng, n=N, long_frac=0.05):
    """Mostly 1-6 entries (one or two ELL groups), some 20-32 (up to eight), some empty."""
    lens = rng.integers(1, 7, n)
    long = rng.random(n) < long_frac
    lens[long] = rng.integers(20, 33, int(long.sum()))
    lens[rng.choice(n, 400, replace=False)] = 0
    return lens


@pytest.mark.parametrize("dtype", [O.U32, O.SAT64])
def test_pattern_b_narrow(ctx, dtype):
    rng = np.random.default_rng(11 + dtype)
    a = rand_csr(rng, a_lens(rng) // 3, dtype, 5)  # rows of <= 366 entries: products below the fat threshold
    b = rand_csr(rng, b_lens(rng), dtype, "one")
    check(ctx, a, b, dtype, what="pattern B")


def test_pattern_b_multi_segment_band(ctx):
    # rows of 513-1100 entries in a band (neighbouring rows share columns), B rows of 1-6 entries:
    # later segments through the generic walker, rows over more than 8 touched blocks (spread rows)
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 200, N)
    lens[::37] = rng.integers(513, 1100, len(lens[::37]))
    a = rand_csr(rng, lens, O.U32, 3, spread=False)
    b = rand_csr(rng, np.minimum(b_lens(rng, long_frac=0.0), 6), O.U32, "one")
    check(ctx, a, b, O.U32, what="band")
    a2 = rand_csr(rng, lens, O.U32, 3, spread=True)
    check(ctx, a2, b, O.U32, what="spread")


def test_tail_queue_overflow(ctx):
    # every entry's B row has 8 entries (two groups): a 512-entry segment has 512 tail groups, past the
    # queue's 256, so the segment's entries walk their later groups themselves
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 100, N)
    lens[::50] = 512
    a = rand_csr(rng, lens, O.U32, 4)
    b = rand_csr(rng, np.full(N, 8), O.U32, "one")
    check(ctx, a, b, O.U32, what="queue overflow")
    check(ctx, rand_csr(rng, lens, O.U32, 4), rand_csr(rng, np.full(N, 8), O.U32, 9), O.U32, what="overflow, values")


@pytest.mark.parametrize("bvals", ["one", 6])
def test_rank_chunks(ctx, bvals):
    # rows of ~1500-2700 outputs: two or three rank chunks of 895 slots
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 50, N)
    lens[::97] = rng.integers(400, 700, len(lens[::97]))
    a = rand_csr(rng, lens, O.U32, 3)
    b = rand_csr(rng, rng.integers(3, 9, N), O.U32, bvals)
    h = check(ctx, a, b, O.U32, what=f"chunks {bvals}")
    assert int(np.diff(h.row_ptr).max()) > 2 * 895


def test_values_wide_and_saturating(ctx):
    rng = np.random.default_rng(9)
    a = rand_csr(rng, a_lens(rng) // 3, O.U32, "big")
    b = rand_csr(rng, b_lens(rng), O.U32, "big")
    h = check(ctx, a, b, O.U32, what="u32 big")
    assert (h.values == 0xFFFFFFFF).any()  # saturated sums
    b1 = rand_csr(rng, b_lens(rng), O.U32, "one")
    check(ctx, a, b1, O.U32, what="u32 big A, pattern B (wide slots, pattern products)")


def test_sat64_past_2_32(ctx):
    rng = np.random.default_rng(13)
    a = rand_csr(rng, a_lens(rng) // 4, O.SAT64, "big")
    b = rand_csr(rng, b_lens(rng), O.SAT64, "big")
    check(ctx, a, b, O.SAT64, what="Sat64 big")
    b1 = rand_csr(rng, b_lens(rng), O.SAT64, 3)
    check(ctx, a, b1, O.SAT64, what="Sat64 big A")


def test_f64_any_order(ctx):
    rng = np.random.default_rng(17)
    a = rand_csr(rng, a_lens(rng) // 3, O.F64, "f64")
    b = rand_csr(rng, b_lens(rng), O.F64, "f64")
    check(ctx, a, b, O.F64, flags=slat.FLAG_F64_ANY_ORDER, rtol=1e-12, what="f64 any order")


def test_empty_rows_and_zeros(ctx):
    rng = np.random.default_rng(19)
    lens = rng.integers(0, 120, N)
    lens[: N // 4] = 0
    a = rand_csr(rng, lens, O.U32, 3)
    bl = b_lens(rng)
    bl[N // 2:] = 0  # entries into empty B rows: rows with no products
    b = rand_csr(rng, bl, O.U32, "one")
    check(ctx, a, b, O.U32, what="empty")
    # explicit zeros in A: products of 0, outputs whose every term is 0 are dropped. (The oracle's
    # constructors drop zeros, which gives the same product; the device's A keeps them)
    rp, col, val = a.arrays()
    val = val.copy()
    val[rng.random(len(val)) < 0.3] = 0
    az = O.from_arrays(rp, col, val, O.U32)
    A = slat.CsrMatrix.from_host(slat.HostCsr(a.n, rp, col, val, slat.U32))
    assert (A.host().values == 0).sum() > 0
    C = A._spgemm(to_dev(b, slat.CsrMatrix))
    st = ctx.stats()
    assert st["mode"] & 16 and st["dropped_rows"] > 0, st
    ref = O.matmul_seq(az, b)
    h = C.host()
    wrp, wcol, wval = ref.arrays()
    np.testing.assert_array_equal(h.row_ptr, wrp)
    np.testing.assert_array_equal(h.col_idx, wcol)
    np.testing.assert_array_equal(h.values, wval)


@pytest.mark.parametrize("dtype", [O.U32, O.SAT64])
def test_torus_chain_takes_stored_mode(ctx, dtype):
    # the bench's chain: A^4 * A of the 30^3 torus against the oracle
    a = O.torus_thinned(30, 3.0, O.Rng())
    if dtype != O.U32:
        a = O.convert(a, dtype)
    p = a
    for _ in range(3):
        p = O.matmul_seq(p, a)
    check(ctx, p, a, dtype, what="torus A^4 * A")
