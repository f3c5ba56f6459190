"""Two ranks through the HIP row-block path: two processes share the one GPU, each
computes its flops-balanced row block of C on the device (slat_rowblock_cuts, a prepared B,
slat_spgemm_rowblock_prepared), and the blocks are assembled over gloo (slat.dist.gather_blocks, the
host twin of the RCCL allgatherv, which needs one GPU per rank). Bar: the assembled C equals the
oracle's product bit for bit (f64: the reference's fold order), for a single-window product (the
30^3 chain's shape) and a wide one (more columns than one LDS window, config C4's shape), every value
type. tests/test_dist_cpu.py covers the cut rule and the assembly with oracle blocks; this file runs
the blocks on the device."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, side, dtype, q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "sparse-linear-algebra-tests_amd"), os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "tests")]
    import numpy as np
    import torch.distributed as dist

    import oracle_py as O
    import slat
    from helpers import digest
    from slat import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cls = {"u32": slat.CsrMatrix, "sat64": slat.MagnusMatrix, "f64": slat.CsrF64}[dtype]
        odt = {"u32": O.U32, "sat64": O.SAT64, "f64": O.F64}[dtype]
        a = O.convert(O.torus_thinned(side, 3.0, O.Rng()), odt)
        if dtype == "f64":  # values whose sums depend on the order
            rp, col, _ = a.arrays()
            a = O.from_arrays(rp, col, np.random.default_rng(5).uniform(0.5, 1.5, len(col)), O.F64)
        p = O.matmul_seq(a, a)
        want = O.matmul_seq(p, a)

        def dev(o):
            rp, col, val = o.arrays()
            return cls.from_host(slat.HostCsr(o.n, rp, col, val, cls.DTYPE))
        da, dp = dev(a), dev(p)
        cuts = D.device_cuts(dp, da, world)
        blk = dp.matmul_rowblock(cuts[rank], cuts[rank + 1], da.prepare())
        h = blk.host()
        rp, col, val = D.gather_blocks(h.row_ptr, h.col_idx, h.values)
        w_rp, w_col, w_val = want.arrays()
        same = digest(rp, col, val, val.dtype.str) == digest(w_rp, w_col, w_val, w_val.dtype.str)
        q.put((rank, same, cuts))
    except Exception as e:  # reported to the parent instead of a hang
        q.put((rank, repr(e), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("side,dtype", [(16, "u32"), (16, "sat64"), (16, "f64"), (41, "u32"), (41, "f64")])
def test_two_ranks_hip_blocks_assemble_to_product(side, dtype):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, side, dtype, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=110) for _ in procs]
    for pr in procs:
        pr.join(timeout=30)
        assert pr.exitcode == 0
    assert sorted(r for r, _, _ in res) == [0, 1]
    assert all(ok is True for _, ok, _ in res), res
    cuts = res[0][2]
    assert cuts[0] == 0 and 0 < cuts[1] < cuts[2] == side ** 3
