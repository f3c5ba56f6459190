"""The real-graph path on the device through the C ABI:
from_edges / from_edges_undirected (src/graph_csr.rs:132-147), the rcm order (:663-722),
permute / unpermute (:726-799) and bandwidth_stats (:802-818), against the oracle. Bar: bit-exact
arrays and the same permutation (degree ties in column order on both sides; the reference's own
tie order is unpinned), plus the reference's round-trip tests and the A^2 equivalence its
analyze_graph_structure asserts (:1546-1549)."""
import numpy as np
import pytest

import oracle_py as O
import slat
from test_coo_gpu import CLS, assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def graphs():
    g = np.random.default_rng(7)
    yield "ref6", O.from_edges_undirected(6, [(0, 3), (1, 4), (2, 5), (0, 1), (3, 4)])
    yield "lattice4x4", O.lattice([4, 4], False)
    yield "directed5", O.from_edges(5, [(0, 1), (1, 2), (2, 3), (3, 4), (4, 0), (0, 3)])
    t = O.torus_thinned(20, 3.0, O.Rng())
    yield "torus20_shuffled", O.permute(t, g.permutation(t.n).astype(np.uint32))
    h = slat.host_rmat(12, 40_000)  # power-law, symmetrised
    rows = np.repeat(np.arange(h.n), np.diff(h.row_ptr).astype(np.int64))
    yield "rmat12_undirected", O.from_edges_undirected(h.n, np.stack([rows, h.col_idx], 1).tolist())
    e = g.integers(0, 3000, (12_000, 2))
    yield "random_undirected", O.from_edges_undirected(3000, e.tolist())
    yield "isolated_nodes", O.from_edges_undirected(50, [(3, 4), (10, 11), (11, 12)])


def dev(m: O.Csr, ctx, dtype=O.U32):
    rp, col, val = m.arrays()
    return CLS[dtype].from_host(slat.HostCsr(m.n, rp, col, val, dtype), ctx)


@pytest.mark.parametrize("undirected", [False, True])
@pytest.mark.parametrize("n,m", [(1, 0), (10, 30), (5000, 40_000)])
def test_from_edges_matches_oracle(ctx, undirected, n, m):
    g = np.random.default_rng(n + m)
    e = g.integers(0, n, (m, 2))
    e[: m // 10, 1] = e[: m // 10, 0]  # self loops
    want = O.from_edges_undirected(n, e.tolist()) if undirected else O.from_edges(n, e.tolist())
    got = slat.CsrMatrix.from_edges_device(n, e[:, 0], e[:, 1], undirected, ctx)
    assert_same(got, want, f"from_edges n={n} m={m} und={undirected}")


def test_from_edges_bad_id_raises(ctx):
    with pytest.raises(slat.SlatError):
        slat.CsrMatrix.from_edges_device(3, [0, 3], [1, 1], False, ctx)


@pytest.mark.parametrize("name,m", list(graphs()), ids=[n for n, _ in graphs()])
def test_rcm_order_matches_oracle(ctx, name, m):
    d = dev(m, ctx)
    np.testing.assert_array_equal(d.rcm_order(), O.rcm_order(m), err_msg=name)


@pytest.mark.parametrize("dtype", [O.U32, O.SAT64, O.F64])
def test_permute_matches_oracle(ctx, dtype):
    t = O.torus_thinned(15, 3.0, O.Rng())
    m = O.convert(t, dtype) if dtype != O.U32 else t
    perm = np.random.default_rng(dtype).permutation(m.n).astype(np.uint32)
    d = dev(m, ctx, dtype)
    d.permute(perm)
    assert_same(d, O.permute(m, perm), f"permute dtype {dtype}")
    np.testing.assert_array_equal(d.perm, perm)


def test_permute_rejects_non_permutation(ctx):
    d = dev(O.lattice([3, 3], True), ctx)
    with pytest.raises(slat.SlatError):
        d.permute(np.zeros(9, np.uint32))
    with pytest.raises(slat.SlatError):
        d.permute(np.full(9, 9, np.uint32))


@pytest.mark.parametrize("name,m", list(graphs()), ids=[n for n, _ in graphs()])
def test_rcm_unpermute_roundtrip(ctx, name, m):
    # src/graph_csr.rs:1107-1145 on the device: rcm, then unpermute restores the arrays
    d = dev(m, ctx)
    d.rcm()
    assert d.perm is not None
    assert_same(d, O.permute(m, O.rcm_order(m)), f"{name} after rcm")
    d.unpermute()
    assert d.perm is None
    assert_same(d, m, f"{name} after unpermute")


@pytest.mark.parametrize("name,m", list(graphs()), ids=[n for n, _ in graphs()])
def test_bandwidth_stats_matches_oracle(ctx, name, m):
    assert dev(m, ctx).bandwidth_stats() == O.bandwidth_stats(m)


def test_rcm_product_is_permuted_product(ctx):
    # analyze_graph_structure (src/graph_csr.rs:1532-1549): A^2 after RCM has A^2's nnz; exactly,
    # (P A P^T)^2 = P A^2 P^T
    t = O.torus_thinned(16, 3.0, O.Rng())
    a = O.permute(t, np.random.default_rng(3).permutation(t.n).astype(np.uint32))
    d = dev(a, ctx)
    p = d.rcm_order()
    dp = d.clone()
    dp.permute(p)
    sq = dp.matmul(dp)
    assert_same(sq, O.permute(O.matmul_seq(a, a), p), "(PAP^T)^2")
