"""Parity of the HIP SpGEMM (through the C ABI) with the oracle and the golden vectors. Needs an
MI355X: every test is marked `gpu`. Bar: bit-exact arrays for u32 / Sat64 / f64 (the f64 kernel
reproduces the reference's left fold in A-row order; the tolerance is therefore 0 ulp)."""
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


# ---- the reference's own unit tests (src/graph_csr.rs:878-1145, src/graph_magnus.rs:455-697) ----
@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64, slat.F64])
def test_reference_unit_cases(ctx, dtype):
    M = CLS[dtype]
    m = M.from_edges(3, [(0, 1), (1, 2)])
    r = m._spgemm(M.identity(3))
    assert r.get(0, 1) == 1 and r.get(1, 2) == 1 and r.get(0, 2) == 0 and r.nnz() == 2
    t = M.from_edges(3, [(0, 1), (1, 2), (2, 0)])
    t2 = t._spgemm(t)
    assert t2.get(0, 2) == 1 and t2.get(1, 0) == 1 and t2.get(2, 1) == 1
    t3 = t2._spgemm(t)
    assert t3.get(0, 0) == 1 and t3.get(1, 1) == 1 and t3.get(2, 2) == 1
    assert M.from_edges(2, [(0, 1), (0, 1)]).get(0, 1) == 2
    d = M.from_edges(4, [(0, 1), (0, 2), (1, 3), (2, 3)])
    assert d._spgemm(d).get(0, 3) == 2
    assert M.new(5)._spgemm(M.new(5)).nnz() == 0


def test_csr_and_magnus_api_names(ctx):
    m = slat.CsrMatrix.from_edges(4, [(0, 1), (0, 2), (1, 3), (2, 3)])
    assert m.matmul(m).get(0, 3) == 2 and m.matmul_par(m).get(0, 3) == 2
    g = slat.MagnusMatrix.from_edges(4, [(0, 1), (0, 2), (1, 3), (2, 3)])
    seq, par = g.matmul_seq(g), g.matmul(g)  # test_matmul_seq_vs_par (src/graph_magnus.rs:690-697)
    assert seq.nnz() == par.nnz() and seq.get(0, 3) == par.get(0, 3) == 2


def test_dimension_mismatch_is_an_error(ctx):
    a, b = slat.CsrMatrix.new(3), slat.CsrMatrix.new(4)
    with pytest.raises(slat.SlatError) as e:
        a.matmul(b)
    assert e.value.status == 2  # SLAT_EDIM where the reference panics


# ---- C1/C2: 30^3 torus repeated exponentiation, golden digests ----
def test_torus30_powers_u32_golden(ctx, golden):
    A = slat.CsrMatrix.from_host(slat.torus_thinned(30, 3.0, slat.StdRng()))
    P = A
    for k in range(2, 8):
        P = P.matmul(A)
        h = P.host()
        assert_digest(digest(h.row_ptr, h.col_idx, h.values), golden["torus30_powers"][k - 1], f"A^{k}")


def test_torus30_powers_sat64_and_exact_alloc(ctx, golden):
    A = slat.MagnusMatrix.from_host(slat.torus_thinned(30, 3.0, slat.StdRng()))
    P = A
    for k in range(2, 6):
        P = P._spgemm(A, slat.FLAG_EXACT_ALLOC if k % 2 else 0)
        h = P.host()
        g = golden["torus30_powers"][k - 1]
        assert_digest(digest(h.row_ptr, h.col_idx, h.values.astype(np.uint32)), g, f"Sat64 A^{k}")
        assert P.capacity >= P.nnz()


def test_output_trimmed_to_nnz(ctx):
    """C is allocated by the bound nnz(A)*maxrow(B) (no mid-call sync) and trimmed to nnz(C) before
    the call returns: a device-resident A^k chain holds ~nnz, not 6.7x (30^3 A^7: 79.1M-slot bound,
    11.7M nnz). The retained powers stay intact while later products reuse the freed tails."""
    A = slat.CsrMatrix.from_host(slat.torus_thinned(30, 3.0, slat.StdRng()))
    powers = [A]
    for k in range(2, 8):
        P = powers[-1].matmul(A)
        assert P.capacity <= 1.1 * P.nnz() + 1, (k, P.capacity, P.nnz())
        powers.append(P)
    o = O.torus_thinned(30, 3.0, O.Rng())
    w = o
    for k in range(2, 6):  # every retained power still holds its product (no tail reuse overlap)
        w = O.matmul_seq(w, o)
        assert_same(powers[k - 1], w, f"retained A^{k}")


# ---- C3: sweep grid, all 20 cells, golden digests of A^2 ----
def test_sweep_grid_golden(ctx, golden):
    rng = slat.StdRng()
    cells = iter(golden["sweep"])
    for s in [5, 10, 20, 30]:
        full = slat.host_lattice([s, s, s], True)
        for epn in [2.0, 3.0, 4.0, 8.0, 26.0]:
            cell = next(cells)
            density = epn / (full.nnz / full.n)
            A = slat.host_thin(full, rng, density) if density < 1.0 else full
            d = slat.CsrMatrix.from_host(A)
            C2 = d.matmul(d)
            h = C2.host()
            assert_digest(digest(h.row_ptr, h.col_idx, h.values), cell["A2"], f"s={s} epn={epn}")


# ---- saturation (test_power_until_stable_chain, src/graph_csr.rs:931-939) ----
@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64])
def test_saturation_chain_matches_oracle(ctx, dtype):
    n = 64
    o = O.add(O.from_edges(n, [(i, i + 1) for i in range(n - 1)], DT[dtype]), O.identity(n, DT[dtype]))
    d = to_dev(o, dtype)
    for it in range(1, 9):
        o2 = O.matmul_seq(o, o)
        d2 = d._spgemm(d)
        assert_same(d2, o2, f"iteration {it}")
        o, d = o2, d2


def test_large_values_saturate_u32_products(ctx):
    # products and sums beyond u32::MAX clamp exactly like Saturating<u32>
    n = 8
    rows = np.repeat(np.arange(n), n)
    cols = np.tile(np.arange(n), n)
    vals = np.full(n * n, 0x10000, dtype=np.uint64)
    vals[::3] = 0xFFFFFFFF
    o = O.from_coo(n, rows, cols, vals, O.U32)
    assert_same(to_dev(o, slat.U32)._spgemm(to_dev(o, slat.U32)), O.matmul_seq(o, o), "u32 sat")
    vals64 = np.full(n * n, 1 << 40, dtype=np.uint64)
    vals64[::5] = (1 << 63) + 12345
    o = O.from_coo(n, rows, cols, vals64, O.SAT64)
    assert_same(to_dev(o, slat.SAT64)._spgemm(to_dev(o, slat.SAT64)), O.matmul_seq(o, o), "sat64")


@pytest.mark.parametrize("k", [3, 4, 5])
def test_u32_narrow_slot_bound(ctx, k):
    # The kernel accumulates a row in u32 slots only when max(A row) * max(B) * len(A row) < 2^32,
    # else in u64 slots. Row 0 has k entries of 2^30 that all hit column 0 of B (value 1):
    # k = 3 -> narrow (sum 3 * 2^30), k = 4 -> wide (sum 2^32 saturates), k = 5 -> wide (saturates).
    n = 64
    r = np.concatenate([np.zeros(k, np.int64), np.arange(1, n)])
    c = np.concatenate([np.arange(1, k + 1), np.arange(1, n)])
    v = np.concatenate([np.full(k, 1 << 30), np.full(n - 1, 7)]).astype(np.uint64)
    a = O.from_coo(n, r, c, v, O.U32)
    br = np.concatenate([np.arange(1, k + 1), np.arange(n)])
    bc = np.concatenate([np.zeros(k, np.int64), (np.arange(n) * 7) % n])
    b = O.from_coo(n, br, bc, np.ones(len(br), np.uint64), O.U32)
    want = O.matmul_seq(a, b)
    assert_same(to_dev(a, slat.U32)._spgemm(to_dev(b, slat.U32)), want, f"narrow bound k={k}")
    if k >= 4:
        assert want.get(0, 0) == 0xFFFFFFFF


@pytest.mark.parametrize("v0", [7, 0, 0xFFFFFFFF])
def test_u32_pattern_b(ctx, v0):
    # Every B value equal (a pattern B, as the torus chain's B = A): the kernel skips the B-value
    # loads and forms one product a * v0 per A entry. v0 = 0: every product is zero and every row
    # drops out; v0 = 2^32 - 1: the rows are not narrow (the u64-slot, saturating path).
    rng = np.random.default_rng(11)
    n = 3000
    ar = np.repeat(np.arange(n), 24)
    ac = rng.integers(0, n, len(ar))
    av = rng.integers(1, 1000, len(ar)).astype(np.uint64)
    a = O.from_coo(n, ar, ac, av, O.U32)
    br = np.repeat(np.arange(n), 9)
    bc = rng.integers(0, n, len(br))
    if v0 == 0:
        # explicit zeros only enter through raw arrays (the COO builders drop them)
        rp, col, _ = O.from_coo(n, br, bc, np.ones(len(br), np.uint64), O.U32).arrays()
        B = slat.CsrMatrix.from_host(slat.HostCsr(n, rp, col, np.zeros(len(col), np.uint32), slat.U32))
        h = to_dev(a, slat.U32)._spgemm(B).host()
        assert len(h.col_idx) == 0
        np.testing.assert_array_equal(h.row_ptr, np.zeros(n + 1, np.uint64))
        return
    b = O.from_coo(n, br, bc, np.full(len(br), v0, np.uint64), O.U32)
    assert_same(to_dev(a, slat.U32)._spgemm(to_dev(b, slat.U32)), O.matmul_seq(a, b), f"pattern B v0={v0}")


# ---- f64 (config C5 shape, small): bit-exact left fold ----
def test_f64_rmat_bit_exact(ctx):
    h = slat.host_rmat(12, 40000)
    rp, col, val = h.row_ptr, h.col_idx, h.values
    o = O.from_arrays(rp, col, val, O.F64)
    d = slat.CsrF64.from_host(h)
    assert_same(d.matmul(d), O.matmul_seq(o, o), "rmat f64 A^2")
    d2 = d.matmul(d)
    o2 = O.matmul_seq(o, o)
    assert_same(d2.matmul(d), O.matmul_seq(o2, o), "rmat f64 A^3")


def test_f64_cancellation_drops_zeros(ctx):
    # row 0 of A*B cancels exactly at column 1: the entry must be dropped (linalg/src/csr.rs:344)
    A = O.from_coo(3, [0, 0, 1], [1, 2, 2], np.array([1.0, 1.0, 2.0]), O.F64)
    B = O.from_coo(3, [1, 1, 2, 2], [0, 1, 1, 2], np.array([3.0, 1.5, -1.5, 4.0]), O.F64)
    want = O.matmul_seq(A, B)
    got = to_dev(A, slat.F64)._spgemm(to_dev(B, slat.F64))
    assert_same(got, want, "cancellation")
    assert ctx.stats()["dropped_rows"] == 1


def test_explicit_zero_inputs_u32(ctx):
    # zero values can only enter through raw arrays; the output keeps matmul's zero-free rows
    rp = np.array([0, 2, 3, 4], np.uint64)
    col = np.array([0, 1, 2, 1], np.uint32)
    val = np.array([0, 5, 0, 3], np.uint32)
    A = slat.CsrMatrix.from_host(slat.HostCsr(3, rp, col, val, slat.U32))
    h = A.matmul(A).host()
    dense = np.zeros((3, 3), np.uint64)
    for r in range(3):
        for i in range(rp[r], rp[r + 1]):
            k = col[i]
            for j in range(rp[k], rp[k + 1]):
                dense[r, col[j]] += np.uint64(val[i]) * np.uint64(val[j])
    want_rp = np.concatenate([[0], np.cumsum((dense != 0).sum(1))]).astype(np.uint64)
    np.testing.assert_array_equal(h.row_ptr, want_rp)
    np.testing.assert_array_equal(h.col_idx, np.nonzero(dense)[1].astype(np.uint32))
    np.testing.assert_array_equal(h.values, dense[dense != 0].astype(np.uint32))


# ---- kernel paths: wave-per-A-entry (long B rows), rank chunks (>1024 per row), wide windows ----
def test_wave_mode_long_b_rows(ctx):
    full = O.lattice([10, 10, 10], True)
    B = O.matmul_seq(full, full)                     # 125 nnz per row: wave-per-A traversal
    for dt in (slat.U32, slat.SAT64, slat.F64):
        a, b = O.convert(full, DT[dt]), O.convert(B, DT[dt])
        assert_same(to_dev(a, dt)._spgemm(to_dev(b, dt)), O.matmul_seq(a, b), f"wave mode dt={dt}")


def test_rank_chunks_long_output_rows(ctx):
    # a row with 3000 distinct output columns exceeds one LDS value chunk
    rng = np.random.default_rng(5)
    n = 4000
    r = np.concatenate([np.zeros(300, np.int64), rng.integers(0, n, 3000)])
    c = np.concatenate([rng.choice(n, 300, replace=False), rng.integers(0, n, 3000)])
    o = O.from_coo(n, r, c, np.ones(len(r)), O.U32)
    B = O.from_coo(n, rng.integers(0, n, 60000), rng.integers(0, n, 60000), rng.integers(1, 9, 60000), O.U32)
    for dt in (slat.U32, slat.SAT64, slat.F64):
        a, b = O.convert(o, DT[dt]), O.convert(B, DT[dt])
        assert_same(to_dev(a, dt)._spgemm(to_dev(b, dt)), O.matmul_seq(a, b), f"chunks dt={dt}")


@pytest.mark.parametrize("dt", [slat.U32, slat.SAT64, slat.F64])
def test_compacted_bitmap_block_groups(ctx, dt):
    # 60,000 columns: one window of 30 blocks (2048 columns each). Numeric keeps only a row's touched
    # blocks in LDS, at most 8 per pass: rows touching 1, 7, 8, 9, 16, 17 and all 30 blocks, through
    # B = I (C = A exactly) and through a random B (outputs spread over every block)
    rng = np.random.default_rng(11)
    n = 60000
    rows, cols = [], []
    for r, nb in enumerate([1, 7, 8, 9, 16, 17, 30, 0, 3, 30, 12, 8, 9]):
        blocks = rng.choice(30, nb, replace=False) if nb < 30 else np.arange(30)
        for b in blocks:
            k = int(rng.integers(1, 6))
            c = np.unique(np.minimum(b * 2048 + rng.integers(0, 2048, k), n - 1))
            rows += [r] * len(c)
            cols += list(c)
    more = rng.integers(0, n, 3000)
    rows += list(20 + (more % 400))
    cols += list(rng.integers(0, n, 3000))
    a = O.convert(O.from_coo(n, rows, cols, rng.integers(1, 9, len(rows)), O.U32), DT[dt])
    eye = O.convert(O.from_coo(n, np.arange(n), np.arange(n), np.ones(n), O.U32), DT[dt])
    B = O.convert(O.from_coo(n, rng.integers(0, n, 3 * n), rng.integers(0, n, 3 * n),
                             rng.integers(1, 9, 3 * n), O.U32), DT[dt])
    da = to_dev(a, dt)
    assert_same(da._spgemm(to_dev(eye, dt)), O.matmul_seq(a, eye), f"A*I dt={dt}")
    assert_same(da._spgemm(to_dev(B, dt)), O.matmul_seq(a, B), f"A*B dt={dt}")


def test_wide_windows_torus46(ctx):
    # n = 97,336 columns > one 63,488-column window: rows iterate windows from their min column
    rng = O.Rng()
    a = O.torus_thinned(46, 3.0, rng)
    a2 = O.matmul_seq(a, a)
    d = to_dev(a, slat.U32)
    assert_same(d._spgemm(d), a2, "46^3 A^2")
    assert_same(to_dev(a2, slat.U32)._spgemm(d), O.matmul_seq(a2, a), "46^3 A^3")


def test_rowblock_partition_concatenates_to_full(ctx):
    A = slat.CsrMatrix.from_host(slat.torus_thinned(20, 4.0, slat.StdRng()))
    full = A.matmul(A).host()
    n = A.n
    bounds = [0, n // 3, n // 2, n]
    cols, vals, rps = [], [], [np.zeros(1, np.uint64)]
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        blk = A.matmul_rowblock(lo, hi, A).host()
        assert blk.n == hi - lo
        rps.append(blk.row_ptr[1:] + rps[-1][-1])
        cols.append(blk.col_idx)
        vals.append(blk.values)
    np.testing.assert_array_equal(np.concatenate(rps), full.row_ptr)
    np.testing.assert_array_equal(np.concatenate(cols), full.col_idx)
    np.testing.assert_array_equal(np.concatenate(vals), full.values)


@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64, slat.F64])
def test_rowblock_slices_of_full_product(ctx, dtype):
    # row blocks of A^3 * A through the pipeline (B in its ELL image): one-row blocks, the first and
    # last rows, a middle stretch, and blocks in both orders on one context (nothing of an earlier
    # call's workspace may leak into the next); each block is the full product's row slice
    a = O.torus_thinned(16, 3.0, O.Rng())
    a3 = O.matmul_seq(O.matmul_seq(a, a), a)
    full = O.matmul_seq(a3, a)
    rp, col, val = full.arrays()
    P, B = to_dev(a3, dtype), to_dev(a, dtype)
    n = a.n
    blocks = [(0, 1), (n - 1, n), (0, 300), (n - 300, n), (n // 2, n // 2 + 700), (n // 3, n // 3 + 1), (5, n - 5)]
    for lo, hi in blocks + blocks[::-1]:
        h = P.matmul_rowblock(lo, hi, B, slat.FLAG_NO_TINY).host()  # (the pipeline: blocks <= 2048 rows would run one kernel)
        s0, s1 = int(rp[lo]), int(rp[hi])
        np.testing.assert_array_equal(h.row_ptr, rp[lo:hi + 1] - rp[lo], err_msg=f"[{lo},{hi}) row_ptr")
        np.testing.assert_array_equal(h.col_idx, col[s0:s1], err_msg=f"[{lo},{hi}) col_idx")
        if val.dtype == np.float64:
            np.testing.assert_array_equal(h.values.view(np.uint64), val[s0:s1].view(np.uint64))
        else:
            np.testing.assert_array_equal(h.values, val[s0:s1], err_msg=f"[{lo},{hi}) values")


def test_empty_and_ragged(ctx):
    for n in (1, 2, 65, 1000):
        z = slat.CsrMatrix.new(n)
        assert z.matmul(z).nnz() == 0
    o = O.from_coo(300, [0, 299, 150], [299, 0, 150], [1, 1, 1], O.U32)
    d = to_dev(o, slat.U32)
    assert_same(d._spgemm(d), O.matmul_seq(o, o), "ragged")


def test_timing_stats(ctx):
    A = slat.CsrMatrix.from_host(slat.torus_thinned(30, 3.0, slat.StdRng()))
    A._spgemm(A, slat.FLAG_TIMING | slat.FLAG_STATS)
    st = ctx.stats()
    assert st["nnz"] == 251590 and st["flops"] == 317168
    assert st["numeric_ms"] > 0 and st["symbolic_ms"] > 0


@pytest.mark.parametrize("vmax", [3, 1 << 14, 1 << 20])
@pytest.mark.parametrize("wide", [False, True])
def test_u32_csr_walk_narrow_and_hub_rows(ctx, vmax, wide):
    # B rows longer than the ELL limit (CSR walk) with k_bvmax's max(B): small values take narrow
    # slots and hub rows (more outputs than slots) accumulate in C; 2^20 values saturate products
    # and sums (u64 slots, rank chunks). wide: more columns than one LDS window.
    n = 70_000 if wide else 6000
    g = np.random.default_rng(vmax + wide)
    rows = np.concatenate([g.integers(0, n, 6 * n), np.zeros(3000, np.int64), np.full(800, 1)])
    cols = np.concatenate([g.integers(0, n, 6 * n), g.integers(0, n, 3000), g.integers(0, n, 800)])
    b_rows = np.concatenate([rows, np.repeat(np.arange(40), 120)])
    b_cols = np.concatenate([cols, g.integers(0, n, 40 * 120)])
    a = O.from_coo(n, rows, cols, g.integers(1, vmax + 1, len(rows)), O.U32)
    b = O.from_coo(n, b_rows, b_cols, g.integers(1, vmax + 1, len(b_rows)), O.U32)
    got = to_dev(a, slat.U32).matmul(to_dev(b, slat.U32))
    assert_same(got, O.matmul_seq(a, b), f"csr walk vmax={vmax} wide={wide}")


def test_matmul_progress_lines(ctx, capfd):
    """MATMUL_PROGRESS (src/graph_csr.rs:10-11, 404-408, 477-481): the pass summary lines on stderr."""
    a = slat.torus_thinned_device(10, 3.0, slat.StdRng(), ctx)
    prev = slat.set_matmul_progress(True)
    try:
        c = a.matmul_par(a)
    finally:
        slat.set_matmul_progress(prev)
    err = capfd.readouterr().err
    assert "  symbolic: done in " in err and "  numeric:  done in " in err and "rows/s)" in err
    assert c.nnz() > 0
    a.matmul_par(a)
    assert "symbolic:" not in capfd.readouterr().err  # off again


@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64])
@pytest.mark.parametrize("vbig", [1 << 12, 1 << 20, (1 << 31) + 5])
def test_long_rows_narrow_bound_stored_bitmap(ctx, dtype, vbig):
    """Rows of more than one A segment (> 256 entries) in a single-window launch, whose stored
    bitmap means numeric never walked their later segments before choosing the slot width: the
    narrow (u32-slot) bound must still see every A value. Large values in the later segments make
    the exact sums pass 2^32 (u32 saturates, Sat64 keeps them)."""
    rng = np.random.default_rng(31)
    n = 3000
    rows, cols, vals = [], [], []
    for r in range(0, n, 7):  # rows of 300..700 entries, the big values only past entry 256
        k = int(rng.integers(300, 700))
        c = np.sort(rng.choice(n, k, replace=False))
        v = np.ones(k, np.uint64)
        v[260:] = rng.integers(1, vbig, k - 260)
        rows.append(np.full(k, r)), cols.append(c), vals.append(v)
    for r in range(n):  # B-side rows for every column: short, value 3
        rows.append(np.array([r, r])), cols.append(np.array([r, (r * 7 + 1) % n])), vals.append(np.full(2, 3, np.uint64))
    R, Cc, Vv = np.concatenate(rows), np.concatenate(cols), np.concatenate(vals)
    key = R.astype(np.int64) * n + Cc
    _, first = np.unique(key, return_index=True)
    R, Cc, Vv = R[first], Cc[first], Vv[first]
    a = O.from_coo(n, R, Cc, Vv.astype(np.uint32) if dtype == slat.U32 else Vv, DT[dtype])
    assert_same(to_dev(a, dtype)._spgemm(to_dev(a, dtype)), O.matmul_seq(a, a), f"long rows vbig={vbig}")


@pytest.mark.parametrize("b_form", ["ell", "csr"])
@pytest.mark.parametrize("n", [3000, 70000])
def test_sat64_narrow_bound_clamped_a_values(ctx, b_form, n):
    """Sat64 A values of 2^32 and more against a 0/1 pattern B. The narrow-slot bound sees A values
    clamped to u32 (0xFFFFFFFF), so a one-entry row with bound 0xFFFFFFFF * 1 * 1 < 2^32 must still
    take wide slots: in u32 slots 2^32 + 5 became 5 and 2^32 became 0 (dropped as a zero).
    b_form: B rows of <= 32 entries (the ELL image) or a 40-entry row (B walked in CSR form);
    n = 70000 is a wide launch (columns past one LDS window)."""
    rng = np.random.default_rng(7)
    big = np.array([1 << 32, (1 << 32) + 5, (1 << 33) + 1, 0xFFFFFFFF, 1, (1 << 63) + 3], np.uint64)
    ar = np.arange(0, n, 3, dtype=np.int64)  # one entry per listed A row
    ac = rng.integers(0, n, len(ar))
    av = big[np.arange(len(ar)) % len(big)]
    a = O.from_coo(n, ar, ac, av, O.SAT64)
    br, bc = [], []
    for r in range(n):
        k = 40 if (b_form == "csr" and r % 500 == 0) else int(rng.integers(1, 6))
        br.append(np.full(k, r)), bc.append(rng.choice(n, k, replace=False))
    R, Cc = np.concatenate(br), np.concatenate(bc)
    b = O.from_coo(n, R, Cc, np.ones(len(R), np.uint64), O.SAT64)
    for flags in (0, slat.FLAG_NO_TINY):
        got = to_dev(a, slat.SAT64)._spgemm(to_dev(b, slat.SAT64), flags)
        assert_same(got, O.matmul_seq(a, b), f"Sat64 clamped A max, B {b_form}, n={n}, flags={flags}")


@pytest.mark.parametrize("case", ["all_short", "mixed", "empty_b", "zeros"])
@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64])
def test_single_window_short_row_categories(ctx, case, dtype):
    """Single-window launches (columns within one LDS window, > 2048 rows: not the one-kernel path)
    batch their short rows in hash tables. all_short: max row of A x max row of B rounded up to ELL
    groups <= 256, so no row is listed and only the short-row kernels run (the completion word is
    stored by the numeric short launch); mixed: rows of 100 entries among short ones go to the
    window kernels; empty_b: A rows of 300 entries against an empty B (nothing listed, every count
    0); zeros: explicit zero values in B's short rows (the zero-row count of the short kernels)."""
    rng = np.random.default_rng({"all_short": 1, "mixed": 2, "empty_b": 3, "zeros": 4}[case])
    n = 5000
    lens = rng.integers(0, 9, n)
    if case == "mixed":
        lens[::97] = 100
    if case == "empty_b":
        lens[::50] = 300
    ar = np.repeat(np.arange(n), lens)
    ac = np.concatenate([rng.choice(n, k, replace=False) for k in lens])
    av = rng.integers(1, 1 << 20, len(ar))
    a = O.from_coo(n, ar, ac, av, DT[dtype])
    if case == "empty_b":
        b = O.from_coo(n, [], [], [], DT[dtype])
    else:
        bl = rng.integers(1, 8, n)
        br = np.repeat(np.arange(n), bl)
        bc = np.concatenate([rng.choice(n, k, replace=False) for k in bl])
        bv = rng.integers(0 if case == "zeros" else 1, 5, len(br))
        b = O.from_coo(n, br, bc, bv, DT[dtype])
    got = to_dev(a, dtype)._spgemm(to_dev(b, dtype))
    assert_same(got, O.matmul_seq(a, b), f"single-window {case}")


@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64, slat.F64])
@pytest.mark.parametrize("vals", ["small", "big", "zeros"])
def test_wide_csr_b_short_row_batches(ctx, dtype, vals):
    """Wide launches (columns past one LDS window) whose B has rows longer than the ELL image allows
    read B in CSR form; their short rows are batched in the hash tables all the same, each B row's
    entries taken 4 at a time where they lie (the last group partial: rows of 1..9 entries and a few
    of 40..300, so groups of every count 1..4). big: products and sums past 2^32 (u32 saturates);
    zeros: explicit zero B values (the zero-row count)."""
    rng = np.random.default_rng({"small": 11, "big": 12, "zeros": 13}[vals])
    n = 70_000
    lens = rng.integers(0, 6, n)
    lens[::1000] = 40  # a few medium A rows (window category)
    ar = np.repeat(np.arange(n), lens)
    ac = np.concatenate([rng.choice(n, k, replace=False) for k in lens])
    bl = rng.integers(1, 10, n)
    bl[::997] = rng.integers(40, 300, len(bl[::997]))  # B rows past the ELL limit (32)
    br = np.repeat(np.arange(n), bl)
    bc = np.concatenate([rng.choice(n, k, replace=False) for k in bl])
    hi = {"small": 7, "big": (1 << 31) + 7, "zeros": 3}[vals]
    lo = 0 if vals == "zeros" else 1
    if dtype == slat.F64:
        av, bv = rng.standard_normal(len(ar)), rng.standard_normal(len(br))
        if vals == "zeros":
            bv[::5] = 0.0
    else:
        av, bv = rng.integers(1, hi, len(ar)), rng.integers(lo, hi, len(br))
    a = O.from_coo(n, ar, ac, av, DT[dtype])
    b = O.from_coo(n, br, bc, bv, DT[dtype])
    flags = slat.FLAG_F64_ANY_ORDER if dtype == slat.F64 else 0
    got = to_dev(a, dtype)._spgemm(to_dev(b, dtype), flags)
    want = O.matmul_seq(a, b)
    if dtype == slat.F64:  # any order: within rtol 1e-12 of the fold order
        h = got.host()
        rp, col, val = want.arrays()
        np.testing.assert_array_equal(h.row_ptr, rp)
        np.testing.assert_array_equal(h.col_idx, col)
        np.testing.assert_allclose(h.values, val, rtol=1e-12, atol=1e-12)
    else:
        assert_same(got, want, f"wide CSR-B short batches {vals}")


@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64, slat.F64])
@pytest.mark.parametrize("case", ["c1", "overflow", "zeros", "big", "wide"])
def test_lane_rows(ctx, dtype, case):
    """Products whose rows hold at most 64 products run as one kernel, a row per lane
    (slat_lane.hip, mode bit 8): the 30^3 chain's A * A (C1) and its variants. overflow: a bound
    that admits the kernel (max row(A) x max row(B) <= 256) but a row of 100 products, so the call
    reruns through the pipeline; zeros: explicit zero values (zero sums dropped in-kernel); big:
    products and sums past 2^32 (u32 saturates, Sat64 keeps them); wide: 70 000 columns. Every case
    against the oracle and against the pipeline (SLAT_FLAG_NO_TINY)."""
    rng = np.random.default_rng({"c1": 1, "overflow": 2, "zeros": 3, "big": 4, "wide": 5}[case])
    if case == "c1":
        h = slat.torus_thinned(30, 3.0, slat.StdRng())
        rp = h.row_ptr.astype(np.int64)
        rows = np.repeat(np.arange(h.n), np.diff(rp))
        vals = rng.integers(1, 5, len(rows)) if dtype != slat.F64 else rng.standard_normal(len(rows))
        a = O.from_coo(h.n, rows, h.col_idx.astype(np.int64), vals, DT[dtype])
        b = a
    else:
        n = 70_000 if case == "wide" else 5000
        lens = rng.integers(0, 6, n)
        if case == "overflow":
            lens[17] = 10  # 10 entries x B rows of 10 = 100 products > 64
        ar = np.repeat(np.arange(n), lens)
        ac = np.concatenate([rng.choice(n, k, replace=False) for k in lens])
        bl = rng.integers(1, 7, n)
        if case == "overflow":
            bl[ac[lens[:17].sum():lens[:18].sum()]] = 10
        br = np.repeat(np.arange(n), bl)
        bc = np.concatenate([rng.choice(n, k, replace=False) for k in bl])
        if dtype == slat.F64:
            av, bv = rng.standard_normal(len(ar)), rng.standard_normal(len(br))
            if case == "zeros":
                bv[::4] = 0.0
        else:
            hi = (1 << 31) + 9 if case == "big" else 5
            av = rng.integers(1, hi, len(ar))
            bv = rng.integers(0 if case == "zeros" else 1, hi, len(br))
        a = O.from_coo(n, ar, ac, av, DT[dtype])
        b = O.from_coo(n, br, bc, bv, DT[dtype])
    da, db = to_dev(a, dtype), to_dev(b, dtype)
    want = O.matmul_seq(a, b)
    got = da._spgemm(db)
    if case != "overflow":
        assert ctx.stats()["mode"] & 8, "the lane kernel did not run"
    assert_same(got, want, f"lane rows {case}")
    assert_same(da._spgemm(db, slat.FLAG_NO_TINY), want, f"pipeline {case}")
    if case == "overflow":
        # the pair is remembered: the next call goes to the pipeline without the lane attempt
        assert_same(da._spgemm(db), want, "overflow, second call")
        assert not ctx.stats()["mode"] & 8, "the remembered pair ran the lane kernel again"


@pytest.mark.parametrize("ncols", [(1 << 26) - 1, 1 << 26])
def test_lane_sort_key_column_limit(ctx, ncols):
    # The lane kernel's sort key is (column << 6) | slot; with 2^26 columns the last column at slot 63
    # would equal the padding key 0xFFFFFFFF and the product would be dropped, so the kernel takes
    # only n_cols < 2^26. A row of 64 products, all in the last column: its sum
    # must be 64 whichever path runs (rectangular views through the C ABI: 1 x 64 times 64 x ncols)
    import ctypes as C
    from slat import _lib as L
    last = ncols - 1

    def host_view(n_rows, n_cols, rp, col, val):
        v = L.CsrView()
        v.n_rows, v.n_cols, v.nnz = n_rows, n_cols, len(col)
        v.row_ptr, v.col_idx, v.values = rp.ctypes.data, col.ctypes.data, val.ctypes.data
        v.dtype, v.residency = slat.U32, L.HOST
        v.max_row_nnz = int(np.diff(rp.astype(np.int64)).max(initial=0))
        return v
    arp, acol, aval = np.array([0, 64], np.uint64), np.arange(64, dtype=np.uint32), np.ones(64, np.uint32)
    brp, bcol, bval = np.arange(65, dtype=np.uint64), np.full(64, last, np.uint32), np.ones(64, np.uint32)
    va, vb = host_view(1, 64, arp, acol, aval), host_view(64, ncols, brp, bcol, bval)
    out = L.CsrOwned()
    L.check(L.lib().slat_spgemm(ctx.ptr, C.byref(va), C.byref(vb), C.byref(out), 0), ctx.ptr)
    try:
        lane_ran = bool(ctx.stats()["mode"] & 8)
        assert int(out.nnz) == 1
        rp, col, val = np.empty(2, np.uint64), np.empty(1, np.uint32), np.empty(1, np.uint32)
        v = L.lib().slat_csr_view_of(C.byref(out))
        L.check(L.lib().slat_csr_to_host(ctx.ptr, C.byref(v), rp.ctypes.data, col.ctypes.data, val.ctypes.data), ctx.ptr)
        assert int(col[0]) == last and int(val[0]) == 64, (col, val)
        assert lane_ran == (ncols < (1 << 26))
    finally:
        L.lib().slat_csr_free(ctx.ptr, C.byref(out))
