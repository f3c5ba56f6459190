"""Parity of the device-resident SpGEMM consumers with the oracle and the
reference's own unit tests: CsrMatrix::add / identity / reachability_sum / power_until_stable /
connected_components (src/graph_csr.rs:68-80, 487-603) and their MagnusMatrix twins
(src/graph_magnus.rs:245-360). Bar: bit-exact arrays (u32 / Sat64 / f64), equal iteration counts,
equal component ids. Every test needs an MI355X."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu

DT = {slat.U32: O.U32, slat.SAT64: O.SAT64, slat.F64: O.F64}
CLS = {slat.U32: slat.CsrMatrix, slat.SAT64: slat.MagnusMatrix, slat.F64: slat.CsrF64}
ALL = [slat.U32, slat.SAT64, slat.F64]


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


def random_csr(n, nnz, dtype, seed, lo=1, hi=9):
    g = np.random.default_rng(seed)
    r = g.integers(0, n, nnz)
    c = g.integers(0, n, nnz)
    if dtype == O.F64:
        v = g.uniform(0.5, 1.5, nnz)
    else:
        v = g.integers(lo, hi, nnz)
    return O.from_coo(n, r, c, v, dtype)


def undirected(n, edges, dtype=O.U32):
    e = [(a, b) for a, b in edges] + [(b, a) for a, b in edges if a != b]
    return O.from_edges(n, e, dtype)


# ---- the reference's own unit tests (src/graph_csr.rs:918-965, 1096-1106) ----------------------
@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64])
def test_reachability_chain(ctx, dtype):
    m = CLS[dtype].from_edges(4, [(0, 1), (1, 2), (2, 3)])
    s, k = m.reachability_sum()
    for a, b in [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]:
        assert s.get(a, b) > 0
    assert s.get(3, 0) == 0 and s.get(2, 0) == 0
    assert k == 4  # A^4 = 0 adds nothing: nnz repeats at the 4th power


@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64])
def test_power_until_stable_chain(ctx, dtype):
    n = 64
    M = CLS[dtype]
    m = M.from_edges(n, [(i, i + 1) for i in range(n - 1)])
    with_id = m.add(M.identity(n))
    stable, iters = with_id.power_until_stable()
    assert iters <= 8
    # golden 2: 7 squarings; saturated entries at the last one: 1711 u32, 1176 Sat64
    assert iters == 7
    mx = 0xFFFFFFFF if dtype == slat.U32 else 0xFFFFFFFFFFFFFFFF
    assert int((stable.host().values == mx).sum()) == (1711 if dtype == slat.U32 else 1176)
    assert stable.nnz() == n * (n + 1) // 2


@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64])
def test_connected_components_reference_cases(ctx, dtype):
    M = CLS[dtype]
    tri = M.from_edges_undirected(6, [(0, 1), (1, 2), (2, 0), (3, 4), (4, 5), (5, 3)])
    comp = tri.connected_components()
    assert comp[0] == comp[1] == comp[2] and comp[3] == comp[4] == comp[5] and comp[0] != comp[3]
    assert len(set(M.new(5).connected_components())) == 5
    one = M.from_edges_undirected(4, [(0, 1), (1, 2), (2, 3)])
    c = one.connected_components()
    assert c[0] == c[1] == c[2] == c[3]


# ---- add: bit-exact against orc_add (CsrMatrix::add restated) ---------------------------------
@pytest.mark.parametrize("dtype", ALL)
@pytest.mark.parametrize("n,za,zb", [(1, 1, 0), (50, 200, 300), (300, 3000, 500), (2000, 40000, 40000)])
def test_add_matches_oracle(ctx, dtype, n, za, zb):
    oa = random_csr(n, za, DT[dtype], 11 + n)
    ob = random_csr(n, zb, DT[dtype], 29 + n)
    got = to_dev(oa, dtype).add(to_dev(ob, dtype))
    assert_same(got, O.add(oa, ob), f"add n={n}")


def test_add_long_rows_and_empty_rows(ctx):
    # rows far longer than a wavefront (chunk carries), empty rows on either side
    n = 4
    rows_a = [0] * 1000 + [2] * 7
    cols_a = list(range(0, 3000, 3)) + list(range(7))
    rows_b = [0] * 700 + [1] * 5 + [2] * 300
    cols_b = list(range(0, 1400, 2)) + list(range(5)) + list(range(100, 400))
    oa = O.from_coo(n, rows_a, cols_a, np.arange(1, len(rows_a) + 1), O.U32)
    ob = O.from_coo(n, rows_b, cols_b, np.arange(1, len(rows_b) + 1), O.U32)
    got = to_dev(oa, slat.U32).add(to_dev(ob, slat.U32))
    assert_same(got, O.add(oa, ob), "long rows")


def test_add_saturates(ctx):
    for dtype, big in [(slat.U32, 0xFFFFFFF0), (slat.SAT64, 0xFFFFFFFFFFFFFFF0)]:
        oa = O.from_coo(3, [0, 0, 1], [0, 2, 1], [big, 5, 1], DT[dtype])
        ob = O.from_coo(3, [0, 1, 2], [0, 1, 2], [big, 2, 3], DT[dtype])
        got = to_dev(oa, dtype).add(to_dev(ob, dtype))
        assert_same(got, O.add(oa, ob), "saturating add")
        mx = 0xFFFFFFFF if dtype == slat.U32 else 0xFFFFFFFFFFFFFFFF
        assert got.get(0, 0) == mx


def test_add_f64_cancellation_drops_entries(ctx):
    # equal columns whose sum is exactly zero are dropped (`if v != 0`), others kept in order
    oa = O.from_coo(3, [0, 0, 0, 1, 2], [1, 4, 9, 2, 0], [1.5, -2.0, 3.0, 0.25, 7.0], O.F64)
    ob = O.from_coo(3, [0, 0, 0, 1, 2], [1, 4, 5, 2, 1], [-1.5, 2.5, 1.0, -0.25, 1.0], O.F64)
    got = to_dev(oa, slat.F64).add(to_dev(ob, slat.F64))
    want = O.add(oa, ob)
    assert_same(got, want, "f64 cancellation")
    assert got.nnz() == 5 and got.get(0, 1) == 0 and got.get(1, 2) == 0


def test_add_shape_mismatch_is_edim(ctx):
    a = slat.CsrMatrix.from_edges(3, [(0, 1)])
    b = slat.CsrMatrix.from_edges(4, [(0, 1)])
    with pytest.raises(slat.SlatError) as e:
        a.add(b)
    assert e.value.status == 2


def test_identity_and_pattern_equal(ctx):
    i5 = slat.CsrMatrix.identity(5)
    assert i5.nnz() == 5 and all(i5.get(k, k) == 1 for k in range(5))
    m = slat.CsrMatrix.from_edges(5, [(0, 1), (3, 4)])
    assert m.same_pattern(m.clone())
    assert not m.same_pattern(slat.CsrMatrix.from_edges(5, [(0, 1), (3, 2)]))
    assert not m.same_pattern(i5)
    assert slat.CsrMatrix.identity(0).nnz() == 0


# ---- the drivers against their oracle restatements --------------------------------------------
def graphs():
    rng = O.Rng()
    torus = O.torus_thinned(6, 3.0, rng)
    yield "torus6", torus
    yield "random_dir", random_csr(120, 180, O.U32, 5)
    yield "random_sparse", random_csr(200, 150, O.U32, 6)
    yield "two_tri_plus_isolated", undirected(9, [(0, 1), (1, 2), (2, 0), (5, 6), (6, 7), (7, 5)])


@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64])
def test_power_until_stable_matches_oracle(ctx, dtype):
    for name, g in graphs():
        g = O.convert(g, DT[dtype])
        w = O.add(g, O.identity(g.n, DT[dtype]))
        want, k_want = O.power_until_stable(w)
        got, k = to_dev(w, dtype).power_until_stable()
        assert k == k_want, name
        assert_same(got, want, name)


@pytest.mark.parametrize("dtype", [slat.U32, slat.SAT64])
def test_reachability_sum_matches_oracle(ctx, dtype):
    for name, g in graphs():
        g = O.convert(g, DT[dtype])
        want, k_want = O.reachability_sum(g)
        got, k = to_dev(g, dtype).reachability_sum()
        assert k == k_want, name
        assert_same(got, want, name)


def test_connected_components_matches_oracle(ctx):
    for name, g in graphs():
        want = O.connected_components(g)
        got = to_dev(g, slat.U32).connected_components()
        assert got == want.tolist(), name


def test_connected_components_directed_is_strongly_connected(ctx):
    # directed cycle 0->1->2->0 and a tail 2->3: {0,1,2} mutually reachable, 3 alone, 4 isolated
    g = O.from_edges(5, [(0, 1), (1, 2), (2, 0), (2, 3)])
    got = to_dev(g, slat.U32).connected_components()
    assert got == O.connected_components(g).tolist() == [0, 0, 0, 1, 2]


def test_f64_drivers(ctx):
    g = O.convert(random_csr(60, 90, O.U32, 9), O.F64)
    want, k_want = O.reachability_sum(g)
    got, k = to_dev(g, slat.F64).reachability_sum()
    assert k == k_want
    assert_same(got, want, "f64 reachability_sum")
