"""The host mirror of CsrBTreeMatrix's layout (no GPU). The separator nodes follow
DenseBTree::extend_from_sorted (src/dense_btree.rs:116-162): their count is pinned by the reference's
own printout of it (btree_overhead.csv, src/dense_btree.rs:418-426, n = 1..10000), the lookups
through them answer as the reference's unit tests require (src/dense_btree.rs:336-534), and every
row's data slice sits after its separators and reads back as the CSR row
(src/graph_csr_btree.rs:57-63, src/dense_btree.rs:311)."""
import bisect
import os

import numpy as np

import oracle_py as O
import slat
from slat.matrix import btree_index, btree_internal

HERE = os.path.dirname(os.path.abspath(__file__))


def tree(vals):
    vals = np.asarray(vals, np.uint32)
    sep = btree_internal(vals)
    return np.concatenate([sep, vals]), len(sep)


def bs(vals, q):
    i = bisect.bisect_left(vals, q)
    return ("ok", i) if i < len(vals) and vals[i] == q else ("err", i)


def test_internal_len_matches_reference_printout():
    fx = np.load(os.path.join(HERE, "golden", "btree_overhead.npz"))
    for n, il, tl in zip(fx["n"], fx["internal_len"], fx["total_len"]):
        nodes, got = tree(np.arange(n))
        assert got == il and len(nodes) == tl, (n, got, il)


def test_reference_unit_cases():
    nodes, il = tree([])
    assert btree_index(nodes, il, 0) == ("err", 0)  # test_empty
    nodes, il = tree([42])
    assert [btree_index(nodes, il, q) for q in (42, 0, 100)] == [("ok", 0), ("err", 0), ("err", 1)]  # test_single
    nodes, il = tree([10, 20, 30, 40, 50])
    assert btree_index(nodes, il, 30) == ("ok", 2) and btree_index(nodes, il, 25) == ("err", 2)  # the doc example
    for n in (8, 9, 16, 17, 64, 65, 72, 73, 80, 81, 100, 128, 255, 256, 10000):  # boundaries, test_large
        nodes, il = tree(np.arange(n))
        for i in list(range(0, n, max(1, n // 300))) + [n - 1]:
            assert btree_index(nodes, il, i) == ("ok", i), (n, i)
        assert btree_index(nodes, il, n) == ("err", n)


def test_matches_binary_search():
    # test_matches_binary_search: keys 0, 3, 6, ... (n in 0..=200, every query up to 3n + 5)
    for n in range(0, 201, 7):
        vals = [3 * x for x in range(n)]
        nodes, il = tree(vals)
        for q in range(3 * n + 6):
            assert btree_index(nodes, il, q) == bs(vals, q), (n, q)


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
    """Two rows of 40 and 20 keys: 40 keys -> 3 leaf chunks -> one internal node of 16 separators;
    20 keys -> 2 chunks -> 16 separators; so data_off = 16 and 16 + 40 + 16 = 72."""
    n = 2
    rp = np.array([0, 40, 60], np.uint64)
    col = np.concatenate([np.arange(40), np.arange(100, 120)]).astype(np.uint32)
    m = slat.CsrBTreeMatrix.from_flat(n, rp, col, np.ones(60, np.uint32), ctx=object())
    assert int(m.data_off[0]) == 16 and int(m.data_off[1]) == 72 and len(m.nodes) == 92
    np.testing.assert_array_equal(m.nodes[:3], [15, 31, 39])  # leaf chunks' last keys, then max padding
    assert (m.nodes[3:16] == 39).all()
    for r in range(n):
        for q in col[rp[r]:rp[r + 1]]:
            assert m.index(r, int(q)) == ("ok", int(q) - (0 if r == 0 else 100))
