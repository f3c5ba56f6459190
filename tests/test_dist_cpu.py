"""Multi-GPU layout on CPU (gloo, world size 2): flops-balanced 1-D row blocks of A
and the allgatherv assembly of the distributed C row blocks. The per-rank products are computed with
the oracle here (the HIP row-block path itself is covered by tests/test_spgemm_gpu.py); what is under
test is the partition and the cross-rank assembly, which bench.py runs over RCCL on GPUs."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle_py as O
from helpers import digest
from slat import dist as D


def _torus(side=12, epn=3.0):
    return O.torus_thinned(side, epn, O.Rng())


def test_row_flops_matches_oracle():
    a = _torus()
    p = O.matmul_seq(a, a)
    prp, pcol, _ = p.arrays()
    arp, _, _ = a.arrays()
    assert int(D.row_flops(prp, pcol, arp).sum()) == O.flops(p, a)


@pytest.mark.parametrize("parts", [1, 2, 3, 4, 8])
def test_flops_balanced_cuts(parts):
    a = _torus()
    p = O.matmul_seq(O.matmul_seq(a, a), a)
    prp, pcol, _ = p.arrays()
    arp, _, _ = a.arrays()
    cuts = D.flops_balanced_cuts(prp, pcol, arp, parts)
    f = D.row_flops(prp, pcol, arp)
    assert cuts[0] == 0 and cuts[-1] == p.n and len(cuts) == parts + 1
    assert all(x <= y for x, y in zip(cuts[:-1], cuts[1:]))
    per = [int(f[lo:hi].sum()) for lo, hi in zip(cuts[:-1], cuts[1:])]
    assert sum(per) == int(f.sum())
    assert max(per) - int(f.sum()) / parts <= int(f.max())  # within one row of the ideal split


def test_cuts_degenerate_inputs():
    assert D.flops_balanced_cuts(np.zeros(1, np.uint64), np.zeros(0, np.uint32), np.zeros(1, np.uint64), 4) == [0] * 5
    rp = np.array([0, 0, 0, 0], np.uint64)  # 3 empty rows, no products: split by rows
    assert D.flops_balanced_cuts(rp, np.zeros(0, np.uint32), rp, 3) == [0, 1, 2, 3]


def _block_rows(m: O.Csr, lo: int, hi: int):
    rp, col, val = m.arrays()
    s, e = int(rp[lo]), int(rp[hi])
    return (rp[lo:hi + 1] - rp[lo]).astype(np.uint64), col[s:e], val[s:e]


def test_rowblock_product_is_row_slice():
    # rows [lo, hi) of A·B equal (A with the other rows emptied)·B restricted to [lo, hi)
    a = _torus()
    p = O.matmul_seq(a, a)
    full = O.matmul_seq(p, a)
    lo, hi = 300, 1100
    rp, col, val = p.arrays()
    keep = np.zeros(p.n + 1, np.uint64)
    keep[lo + 1:hi + 1] = rp[lo + 1:hi + 1] - rp[lo]
    keep[hi + 1:] = rp[hi] - rp[lo]
    masked = O.from_arrays(keep, col[int(rp[lo]):int(rp[hi])], val[int(rp[lo]):int(rp[hi])], O.U32)
    got = O.matmul_seq(masked, a)
    g_rp, g_col, g_val = _block_rows(got, lo, hi)
    w_rp, w_col, w_val = _block_rows(full, lo, hi)
    np.testing.assert_array_equal(g_rp, w_rp)
    np.testing.assert_array_equal(g_col, w_col)
    np.testing.assert_array_equal(g_val, w_val)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, dtype, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a = O.convert(_torus(10, 4.0), dtype)
        p = O.matmul_seq(a, a)
        full = O.matmul_seq(p, a)
        prp, pcol, _ = p.arrays()
        arp, _, _ = a.arrays()
        cuts = D.flops_balanced_cuts(prp, pcol, arp, world)
        lrp, lcol, lval = _block_rows(full, cuts[rank], cuts[rank + 1])  # this rank's C row block
        rp, col, val = D.gather_blocks(lrp, lcol, lval)
        f_rp, f_col, f_val = full.arrays()
        same = val.dtype == f_val.dtype and digest(rp, col, val, val.dtype.str) == digest(f_rp, f_col, f_val, f_val.dtype.str)
        q.put((rank, same, len(rp) - 1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dtype", [O.U32, O.SAT64, O.F64])
def test_gather_blocks_gloo_world2(dtype):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, dtype, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in procs]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert sorted(r for r, _, _ in res) == [0, 1]
    assert all(ok for _, ok, _ in res), res
    assert all(n == 1000 for _, _, n in res)
