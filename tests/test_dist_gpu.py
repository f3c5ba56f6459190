"""The multi-GPU row-block path through libslat's C ABI on one GPU: device cuts
equal the numpy restatement of the flops-balanced rule; a one-rank RCCL communicator's broadcast and
allgatherv return the matrix they were given (row_ptr rebased, including a block given as a view
with absolute offsets); the allgatherv's assembly (offset tables, relative row ends, the k_rebase
kernel) over many blocks through slat_concat_rows. Multi-rank RCCL needs one GPU per rank: the
driver's 8-GPU run covers it, and bench.py checks that run's gathered product against the golden
digests."""
import ctypes as C
import os
import socket

import numpy as np
import pytest

import oracle_py as O
import slat
from slat import _lib as L
from slat import dist as D

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return slat.default_context(0)


@pytest.fixture(scope="module")
def group():
    import torch.distributed as dist
    if not dist.is_initialized():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    yield None


def _same(a, b):
    ha, hb = a.host(), b.host()
    np.testing.assert_array_equal(ha.row_ptr, hb.row_ptr)
    np.testing.assert_array_equal(ha.col_idx, hb.col_idx)
    np.testing.assert_array_equal(ha.values, hb.values)


@pytest.mark.parametrize("parts", [1, 2, 3, 4, 7, 8])
def test_device_cuts_match_host_rule(ctx, parts):
    A = slat.CsrMatrix.from_host(slat.torus_thinned(20, 3.0, slat.StdRng()), ctx)
    P = A.matmul(A).matmul(A)
    h, a = P.host(), A.host()
    assert D.device_cuts(P, A, parts) == D.flops_balanced_cuts(h.row_ptr, h.col_idx, a.row_ptr, parts)
    r = slat.CsrF64.from_host(slat.host_rmat(12, 8 << 12), ctx)  # skewed rows
    hr = r.host()
    assert D.device_cuts(r, r, parts) == D.flops_balanced_cuts(hr.row_ptr, hr.col_idx, hr.row_ptr, parts)


def test_device_cuts_no_products(ctx):
    e = slat.CsrMatrix.new(10)
    assert D.device_cuts(e, e, 4) == [0, 2, 5, 7, 10]


def test_row_blocks_concatenate_to_product(ctx):
    A = slat.CsrMatrix.from_host(slat.torus_thinned(20, 3.0, slat.StdRng()), ctx)
    P = A.matmul(A)
    cuts = D.device_cuts(P, A, 4)
    full = P.matmul(A).host()
    rows, cols = [], []
    for r in range(4):
        b = P.matmul_rowblock(cuts[r], cuts[r + 1], A).host()
        s, e = int(full.row_ptr[cuts[r]]), int(full.row_ptr[cuts[r + 1]])
        np.testing.assert_array_equal(b.row_ptr, full.row_ptr[cuts[r]:cuts[r + 1] + 1] - full.row_ptr[cuts[r]])
        np.testing.assert_array_equal(b.col_idx, full.col_idx[s:e])
        np.testing.assert_array_equal(b.values, full.values[s:e])


@pytest.mark.parametrize("cls", [slat.CsrMatrix, slat.MagnusMatrix, slat.CsrF64])
def test_one_rank_rccl_bcast_and_allgather(ctx, group, cls):
    comm = D.Comm(ctx)
    try:
        o = O.torus_thinned(10, 3.0, O.Rng())
        rp, col, val = o.arrays()
        dt = cls.DTYPE
        M = cls.from_host(slat.HostCsr(o.n, rp, col, val, slat.U32).astype(dt), ctx)
        B = comm.bcast(M, cls)
        _same(B, M)
        C2 = M._spgemm(M)
        blk = M.matmul_rowblock(100, 700, M)
        got = comm.allgather_rows(blk)
        _same(got, blk)
        assert got.nnz() == blk.nnz() and got.max_row_nnz == blk.max_row_nnz
        # a block given as a view into a larger matrix (absolute row_ptr offsets)
        v = C2.view()
        v.row_ptr = v.row_ptr + 8 * 100
        v.n_rows = 600
        v.nnz = int(C2.host().row_ptr[700] - C2.host().row_ptr[100])
        out = L.CsrOwned()
        L.check(L.lib().slat_allgather_rows(ctx.ptr, comm._p, C.byref(v), C.byref(out)), ctx.ptr)
        g2 = cls(out, ctx)
        _same(g2, blk)
    finally:
        comm.close()


@pytest.mark.parametrize("cls", [slat.CsrMatrix, slat.MagnusMatrix, slat.CsrF64])
@pytest.mark.parametrize("parts", [1, 2, 5, 8])
def test_concat_row_blocks_equals_product(ctx, cls, parts):
    """Flops-balanced row blocks of (A^2)·A computed apart, stacked by the rebase path: the full
    product, bit for bit (several blocks, empty ones included when parts exceed the busy rows)."""
    o = O.torus_thinned(20, 3.0, O.Rng())
    rp, col, val = o.arrays()
    A = cls.from_host(slat.HostCsr(o.n, rp, col, val, slat.U32).astype(cls.DTYPE), ctx)
    P = A._spgemm(A)
    full = P._spgemm(A)
    cuts = D.device_cuts(P, A, parts)
    blocks = [P.matmul_rowblock(cuts[r], cuts[r + 1], A) for r in range(parts)]
    got = D.concat_rows(blocks)
    _same(got, full)
    assert got.nnz() == full.nnz() and got.max_row_nnz == full.max_row_nnz
    # blocks given as views with absolute offsets into the full product, plus an empty block
    h = full.host()
    edges = [0, 1, 1, 2000, 4000, 4001, 8000, o.n]
    views = []
    for a, b in zip(edges[:-1], edges[1:]):
        v = full.view()
        v.row_ptr = v.row_ptr + 8 * a
        v.n_rows = b - a
        v.nnz = int(h.row_ptr[b] - h.row_ptr[a])
        views.append(v)
    _same(D.concat_rows([full] * len(views), views), full)


def test_concat_rows_refuses_mixed_blocks(ctx):
    a = slat.CsrMatrix.from_host(slat.torus_thinned(5, 3.0, slat.StdRng()), ctx)
    b = slat.CsrF64.from_host(slat.torus_thinned(5, 3.0, slat.StdRng()).astype(slat.F64), ctx)
    with pytest.raises(slat.SlatError):
        D.concat_rows([a, b])
