"""The reference's real-graph drivers on the device (src/graph_csr.rs:1228-1468): bench_diameter's
squaring + refinement (slat_diameter) and bench_real_graphs' A^k = A^(k-1) * A chain, bit-exact
against the oracle; and the 64-bit-offset kernel instances (the ones a chain past 2^32 nnz runs),
forced on small inputs with SLAT_FLAG_IDX64."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu

CLS = {O.U32: slat.CsrMatrix, O.SAT64: slat.MagnusMatrix, O.F64: slat.CsrF64}


def to_dev(o: O.Csr, cls=slat.CsrMatrix):
    rp, col, val = o.arrays()
    return cls.from_host(slat.HostCsr(o.n, rp, col, val, cls.DTYPE))


def assert_same(dev, orc: O.Csr, what=""):
    h = dev.host()
    rp, col, val = orc.arrays()
    assert dev.nnz() == orc.nnz, what
    np.testing.assert_array_equal(h.row_ptr, rp, err_msg=what)
    np.testing.assert_array_equal(h.col_idx, col, err_msg=what)
    if val.dtype == np.float64:
        np.testing.assert_array_equal(h.values.view(np.uint64), val.view(np.uint64), err_msg=what)
    else:
        np.testing.assert_array_equal(h.values, val, err_msg=what)


def bfs_diameter(o: O.Csr) -> int:
    """Largest finite shortest-path distance (an independent check of the closure algorithm)."""
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import shortest_path
    rp, col, _ = o.arrays()
    m = csr_matrix((np.ones(len(col)), col.astype(np.int64), rp.astype(np.int64)), shape=(o.n, o.n))
    d = shortest_path(m, unweighted=True, directed=False)
    return int(d[np.isfinite(d)].max())


def rmat_edges(scale, deg, seed=42):
    h = slat.host_rmat(scale, (1 << scale) * deg, seed=bytes([seed] * 32))
    src = np.repeat(np.arange(h.n, dtype=np.uint32), np.diff(h.row_ptr).astype(np.int64))
    return h.n, src, h.col_idx


@pytest.mark.parametrize("case", ["path", "cycle", "star", "edge", "torus", "rmat", "forest"])
def test_diameter_matches_oracle_and_bfs(case):
    if case == "path":
        n, e = 40, [(i, i + 1) for i in range(39)]
    elif case == "cycle":
        n, e = 33, [(i, (i + 1) % 33) for i in range(33)]
    elif case == "star":
        n, e = 9, [(0, i) for i in range(1, 9)]
    elif case == "edge":
        n, e = 2, [(0, 1)]
    elif case == "forest":  # two components: the largest finite distance over both
        n, e = 30, [(i, i + 1) for i in range(9)] + [(i, i + 1) for i in range(10, 29)]
    elif case == "torus":
        t = O.torus_thinned(8, 3.0, O.Rng())
        rp, col, _ = t.arrays()
        n = t.n
        e = list(zip(np.repeat(np.arange(n), np.diff(rp).astype(np.int64)).tolist(), col.tolist()))
    else:
        n, s, d = rmat_edges(9, 4)
        e = list(zip(s.tolist(), d.tolist()))
    o = O.from_edges_undirected(n, e)
    want = O.diameter(o)
    got = to_dev(o).diameter()
    assert got == want, (case, got, want)
    assert got[0] == bfs_diameter(o)


def test_real_graph_chain_directed_rmat():
    """bench_real_graphs (src/graph_csr.rs:1427-1468): A = from_edges (directed), A^k = A^(k-1) * A."""
    n, s, d = rmat_edges(11, 4)
    A = slat.CsrMatrix.from_edges_device(n, s, d)
    oA = O.from_edges(n, np.stack([s, d], 1))
    assert_same(A, oA, "from_edges")
    P, oP = A, oA
    for k in range(2, 7):
        P, oP = P.matmul_par(A), O.matmul_seq(oP, oA)
        assert_same(P, oP, f"A^{k}")


@pytest.mark.parametrize("dtype", [O.U32, O.SAT64, O.F64])
def test_idx64_kernels_bit_exact(dtype):
    """The uint64-offset instances of every traversal: single window with the ELL copy (30^3 torus
    powers), wide launches (40^3: 64000 columns), CSR walks of long B rows (R-MAT)."""
    cls = CLS[dtype]
    t = O.convert(O.torus_thinned(30, 3.0, O.Rng()), dtype)
    P3 = O.matmul_seq(O.matmul_seq(t, t), t)
    w = O.convert(O.torus_thinned(40, 3.0, O.Rng()), dtype)
    h = slat.host_rmat(12, 8 << 12)
    rv = h.values if dtype == O.F64 else np.arange(1, h.nnz + 1, dtype=np.uint64) % 7 + 1  # no zeros
    r = O.from_arrays(h.row_ptr, h.col_idx, rv.astype(np.uint32 if dtype == O.U32 else rv.dtype), dtype)
    for name, a, b in [("torus30 A^3*A", P3, t), ("torus40 A*A", w, w), ("rmat12 A*A", r, r)]:
        da, db = to_dev(a, cls), to_dev(b, cls)
        want = O.matmul_seq(a, b)
        assert_same(da._spgemm(db, slat.FLAG_IDX64), want, f"{name} idx64")
        if dtype == O.F64:
            got = da._spgemm(db, slat.FLAG_IDX64 | slat.FLAG_F64_ANY_ORDER).host()
            wrp, wcol, wval = want.arrays()
            np.testing.assert_array_equal(got.col_idx, wcol)
            np.testing.assert_allclose(got.values, wval, rtol=1e-12, atol=0)  # C5's stated tolerance
