"""CsrBTreeMatrix::matmul_par (src/graph_csr_btree.rs:350-479) through slat_spgemm_btree: the
DenseBTreeList layout (separator nodes between the rows' data, src/dense_btree.rs:269-330) in host
memory, the product bit-exact against the oracle's CSR matmul (the B-tree variant computes the same
saturating u32 product). Malformed layouts are refused before any product runs."""
import numpy as np
import pytest

import oracle_py as O
import slat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


def btree(o: O.Csr, ctx):
    rp, col, val = o.arrays()
    return slat.CsrBTreeMatrix.from_flat(o.n, rp, col, val, ctx)


def test_torus_chain_matches_oracle(ctx):
    a = O.torus_thinned(20, 3.0, O.Rng())
    ba = btree(a, ctx)
    p, bp = a, ba
    for k in range(2, 6):
        p = O.matmul_seq(p, a)
        bp = bp.matmul_par(ba)
        rp, col, val = p.arrays()
        assert bp.nnz() == p.nnz, f"A^{k} nnz"
        np.testing.assert_array_equal(bp.data_start, rp)
        got_cols = np.concatenate([bp.data(r) for r in range(bp.n)]) if p.nnz else np.zeros(0, np.uint32)
        np.testing.assert_array_equal(got_cols, col, err_msg=f"A^{k} columns")
        np.testing.assert_array_equal(bp.values, val, err_msg=f"A^{k} values")


def test_long_rows_and_saturation(ctx):
    # rows longer than one separator stride (many separators), values whose products saturate u32
    rng = np.random.default_rng(3)
    n = 3000
    rows = np.concatenate([np.zeros(900, np.int64), rng.integers(0, n, 20000)])
    cols = np.concatenate([rng.choice(n, 900, replace=False), rng.integers(0, n, 20000)])
    vals = rng.integers(1, 1 << 20, len(rows))
    a = O.from_coo(n, rows, cols, vals, O.U32)
    got = btree(a, ctx).matmul_par_csr(btree(a, ctx)).host()
    rp, col, val = O.matmul_seq(a, a).arrays()
    np.testing.assert_array_equal(got.row_ptr, rp)
    np.testing.assert_array_equal(got.col_idx, col)
    np.testing.assert_array_equal(got.values, val)
    assert (val == 0xFFFFFFFF).any()


def test_empty_rows_and_identity(ctx):
    n = 50
    eye = O.from_coo(n, np.arange(n), np.arange(n), np.ones(n), O.U32)
    e = btree(O.from_coo(n, [], [], [], O.U32), ctx)
    assert e.matmul_par(btree(eye, ctx)).nnz() == 0
    a = O.torus_thinned(5, 3.0, O.Rng())
    got = btree(a, ctx).matmul_par(btree(O.from_coo(a.n, np.arange(a.n), np.arange(a.n), np.ones(a.n), O.U32), ctx))
    rp, col, val = a.arrays()
    np.testing.assert_array_equal(got.data_start, rp)
    np.testing.assert_array_equal(got.values, val)


def test_malformed_layouts_are_refused(ctx):
    a = O.torus_thinned(5, 3.0, O.Rng())
    good = btree(a, ctx)
    bad_col = btree(a, ctx)
    bad_col.nodes = bad_col.nodes.copy()
    bad_col.nodes[int(bad_col.data_off[3])] = a.n  # a column id == n_cols
    with pytest.raises(slat.SlatError) as e:
        bad_col.matmul_par_csr(good)
    assert e.value.status == 1
    bad_off = btree(a, ctx)
    bad_off.data_off = bad_off.data_off.copy()
    bad_off.data_off[7] = len(bad_off.nodes)  # the row's slice runs past nodes
    with pytest.raises(slat.SlatError):
        good.matmul_par_csr(bad_off)
    # the context still works afterwards
    assert good.matmul_par(good).nnz() == O.matmul_seq(a, a).nnz
