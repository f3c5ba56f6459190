"""The host mirror of CsrBTreeMatrix's layout (no GPU): every row's data slice sits after its
separator nodes and reads back as the CSR row (src/graph_csr_btree.rs:57-63, src/dense_btree.rs:311)."""
import numpy as np

import oracle_py as O
import slat


def test_from_flat_layout_round_trips():
    a = O.torus_thinned(6, 3.0, O.Rng())
    rp, col, val = a.arrays()
    m = slat.CsrBTreeMatrix.from_flat(a.n, rp, col, val, ctx=object())
    assert m.nnz() == a.nnz and len(m.nodes) >= a.nnz
    for r in range(a.n):
        np.testing.assert_array_equal(m.data(r), col[rp[r]:rp[r + 1]])
    v = m.view()
    assert v.n_rows == a.n and v.nnz == a.nnz and v.n_nodes == len(m.nodes) and v.residency == slat.HOST


def test_separators_sit_between_rows():
    n = 2
    rp = np.array([0, 40, 45], np.uint64)
    col = np.concatenate([np.arange(40), np.arange(5)]).astype(np.uint32)
    m = slat.CsrBTreeMatrix.from_flat(n, rp, col, np.ones(45, np.uint32), ctx=object())
    assert int(m.data_off[0]) == 2 and int(m.data_off[1]) == 42 and len(m.nodes) == 47
