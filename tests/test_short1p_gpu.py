"""The one-kernel wide product (slat_short1p.hip): u32 products with more columns than one LDS window
whose rows are all short (config C4's shape) run as ONE kernel with tile offsets by look-back instead
of symbolic + scan + numeric. Bar: bit-exact against the oracle and against the pipeline (FLAG_STATS
keeps a call on the pipeline); row blocks of a prepared B; explicit zeros dropped; u32 saturation in
the wrap-bit slots; rows the tables cannot take (> 512 products, > 256 distinct columns) rerun through
the pipeline, and the operands are remembered. Stats mode bit 16 tells which path ran."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu

ONEP = 16  # slat_stats.mode bit of the one-kernel wide product


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def dev(o: O.Csr):
    rp, col, val = o.arrays()
    return slat.CsrMatrix.from_host(slat.HostCsr(o.n, rp, col, val, slat.U32))


def same_as_oracle(g, o, what):
    h = g.host()
    rp, col, val = o.arrays()
    assert g.nnz() == o.nnz, f"{what}: nnz {g.nnz()} != {o.nnz}"
    np.testing.assert_array_equal(h.row_ptr, rp, err_msg=f"{what} row_ptr")
    np.testing.assert_array_equal(h.col_idx, col, err_msg=f"{what} col_idx")
    np.testing.assert_array_equal(h.values, val, err_msg=f"{what} values")


def same(x, y, what):
    hx, hy = x.host(), y.host()
    np.testing.assert_array_equal(hx.row_ptr, hy.row_ptr, err_msg=f"{what} row_ptr")
    np.testing.assert_array_equal(hx.col_idx, hy.col_idx, err_msg=f"{what} col_idx")
    np.testing.assert_array_equal(hx.values, hy.values, err_msg=f"{what} values")


def random_wide(n, deg, seed, vmax=1000, zeros=0.0):
    rng = np.random.default_rng(seed)
    m = n * deg
    r = rng.integers(0, n, m)
    c = rng.integers(0, n, m)
    v = rng.integers(1, vmax, m).astype(np.uint64)
    if zeros:
        v[rng.random(m) < zeros] = 0
    return O.from_coo(n, r, c, v, O.U32)


def test_torus41_a3a_one_kernel(ctx):
    # 41^3 = 68,921 columns: a wide launch, every row short
    a = O.torus_thinned(41, 3.0, O.Rng())
    a3 = O.matmul_seq(O.matmul_seq(a, a), a)
    d, d3 = dev(a), dev(a3)
    g = d3._spgemm(d)
    assert ctx.stats()["mode"] & ONEP, "the one-kernel path did not run"
    same_as_oracle(g, O.matmul_seq(a3, a), "41^3 A^3*A")
    p = d3._spgemm(d, slat.FLAG_STATS)  # the pipeline
    assert not ctx.stats()["mode"] & ONEP
    same(g, p, "one kernel vs pipeline")


@pytest.mark.parametrize("deg", [2, 8, 16])
def test_random_wide_one_kernel(ctx, deg):
    # uniform random rows (few repeated columns: nearly every product its own output), empty rows;
    # degree 2 takes the lane kernel (max row(A) x max row(B) within its bound), 8 this one; at 16
    # some rows reach > 256 distinct columns, so the call reruns through the pipeline
    a = random_wide(120_000, deg, 5 + deg)
    d = dev(a)
    g = d._spgemm(d)
    if deg <= 8:
        assert ctx.stats()["mode"] & (ONEP if deg > 2 else 8)
    same_as_oracle(g, O.matmul_seq(a, a), f"random deg {deg}")


def test_row_blocks_prepared(ctx):
    # row blocks of every size class (one row, a tile and a half, odd lengths, a block ending at n)
    a = O.torus_thinned(41, 3.0, O.Rng())
    a2 = O.matmul_seq(a, a)
    want = O.matmul_seq(a2, a)
    d, d2 = dev(a), dev(a2)
    B = d.prepare()
    n = a.n
    wrp, wcol, wval = want.arrays()
    for lo, hi in ((0, 1), (1, 13), (7, 7), (100, 4099), (n // 3, n // 2 + 5), (n - 17, n), (0, n)):
        g = d2.matmul_rowblock(lo, hi, B)
        h = g.host()
        rp = wrp[lo:hi + 1] - wrp[lo]
        np.testing.assert_array_equal(h.row_ptr, rp, err_msg=f"[{lo},{hi}) row_ptr")
        np.testing.assert_array_equal(h.col_idx, wcol[wrp[lo]:wrp[hi]], err_msg=f"[{lo},{hi}) col_idx")
        np.testing.assert_array_equal(h.values, wval[wrp[lo]:wrp[hi]], err_msg=f"[{lo},{hi}) values")


def test_explicit_zeros_dropped(ctx):
    # zero values in A: zero sums are dropped after the kernel (counts per row, host compaction)
    a = random_wide(120_000, 8, 13, vmax=3, zeros=0.4)
    d = dev(a)
    g = d._spgemm(d)
    assert ctx.stats()["mode"] & ONEP
    same_as_oracle(g, O.matmul_seq(a, a), "explicit zeros")


def test_u32_saturation_wide(ctx):
    # products and sums past 2^32 (wrap bits of the u32 slots, Saturating<u32>): every column in
    # [0, 50), one row of 30 entries of u32::MAX (A's longest row keeps the lane kernel out)
    rng = np.random.default_rng(9)
    n = 70_000
    r = np.concatenate([rng.integers(0, n, 280_000), np.full(30, 11)])
    c = np.concatenate([rng.integers(0, 50, 280_000), np.arange(30)])
    v = np.concatenate([rng.integers(1 << 20, 1 << 31, 280_000), np.full(30, 0xFFFFFFFF)]).astype(np.uint64)
    a = O.from_coo(n, r, c, v, O.U32)
    d = dev(a)
    g = d._spgemm(d)
    assert ctx.stats()["mode"] & ONEP
    same_as_oracle(g, O.matmul_seq(a, a), "u32 saturation")


@pytest.mark.parametrize("kind", ["products", "distinct"])
def test_rows_past_the_tables_rerun(ctx, kind):
    # short rows plus one row the tables cannot take: > 512 products (64 entries x B rows of 10), or
    # ~300 products onto ~300 distinct columns; the call reruns through the pipeline and the second
    # call goes there directly
    rng = np.random.default_rng(31)
    n = 80_000
    r = rng.integers(0, n, 160_000)
    c = rng.integers(0, n, 160_000)
    if kind == "products":
        hub = np.arange(1000, 1064)
        r = np.concatenate([r, np.full(64, 4242), np.repeat(hub, 10)])
        c = np.concatenate([c, hub, rng.integers(0, n, 640)])
    else:
        hub = np.arange(2000, 2030)
        r = np.concatenate([r, np.full(30, 777), np.repeat(hub, 10)])
        c = np.concatenate([c, hub, rng.integers(0, n, 300)])
    a = O.from_coo(n, r, c, np.ones(len(r), np.uint64), O.U32)
    d = dev(a)
    want = O.matmul_seq(a, a)
    same_as_oracle(d._spgemm(d), want, f"{kind}: first call")
    same_as_oracle(d._spgemm(d), want, f"{kind}: second call")
    assert not ctx.stats()["mode"] & ONEP, "remembered operands should go to the pipeline"


def test_torus100_a3a_one_kernel_vs_pipeline(ctx):
    # config C4 at full size and one eighth: the one-kernel result equals the pipeline's
    A = slat.torus_thinned_device(100, 3.0, slat.StdRng(), ctx)
    P = A.matmul(A).matmul(A)
    g = P.matmul(A)
    assert ctx.stats()["mode"] & ONEP
    same(g, P._spgemm(A, slat.FLAG_STATS), "C4")
    B = A.prepare()
    n = P.n
    for k in (0, 5):
        lo, hi = k * n // 8, (k + 1) * n // 8
        same(P.matmul_rowblock(lo, hi, B), P.matmul_rowblock(lo, hi, A, slat.FLAG_STATS), f"C4 eighth {k}")
