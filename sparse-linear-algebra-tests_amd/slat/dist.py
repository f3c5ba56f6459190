"""Multi-GPU layout of C = A·B: 1-D row blocks of the left operand.

Every output row depends on one row of A and the B rows it names, so the path shards by rows with no
data-path collective: rank r computes C[cuts[r]:cuts[r+1]] = A[cuts[r]:cuts[r+1]] · B with B
replicated (`slat_spgemm_rowblock`). Cuts are balanced by scalar products (flops), not row counts,
so skewed (power-law) inputs split evenly. The reference has no multi-process path; its `matmul_par`
(src/graph_csr.rs:350-484) splits rows across rayon threads the same way, dynamically.

On the GPUs everything runs through libslat's C ABI over RCCL (`Comm`): the cuts on the device
(`slat_rowblock_cuts`), the replicated operand from rank 0 (`slat_bcast_csr`), and the optional
assembly of the distributed row blocks into one CSR on every rank (`slat_allgather_rows`: one
ncclBroadcast per root and array, u32 columns and native-width values, row_ptr rebased on the device).
The host functions below restate the cut rule and the assembly in numpy for the CPU (gloo) rehearsal
of the multi-rank flow and its tests; `gather_blocks` is that rehearsal's allgatherv.
"""
from __future__ import annotations

import numpy as np


def row_flops(a_rp: np.ndarray, a_col: np.ndarray, b_rp: np.ndarray) -> np.ndarray:
    """Scalar products of each row of A·B: sum over k in row i of A of nnz(B row k)."""
    a_rp = np.asarray(a_rp, dtype=np.int64)
    blen = np.diff(np.asarray(b_rp, dtype=np.int64))
    per_entry = blen[np.asarray(a_col, dtype=np.int64)]
    csum = np.concatenate([[0], np.cumsum(per_entry)])
    return csum[a_rp[1:]] - csum[a_rp[:-1]]


def flops_balanced_cuts(a_rp: np.ndarray, a_col: np.ndarray, b_rp: np.ndarray, parts: int) -> list[int]:
    """Row boundaries [0, c1, ..., n] giving each of `parts` blocks about 1/parts of the products
    (no products at all: equal row counts). The rule slat_rowblock_cuts applies on the device."""
    if parts < 1:
        raise ValueError("parts must be >= 1")
    n = len(a_rp) - 1
    f = row_flops(a_rp, a_col, b_rp)
    cum = np.cumsum(f).astype(object) * parts  # exact: cut r = first row with cum * parts >= total * r
    total = int(cum[-1]) // parts if n else 0
    cuts = [0]
    for r in range(1, parts):
        c = int(np.searchsorted(cum, total * r, side="left")) if total else (n * r) // parts
        cuts.append(min(max(c, cuts[-1]), n))
    cuts.append(n)
    return cuts


class Comm:
    """An RCCL communicator of libslat (slat_comm): one rank per GPU, the unique id shared over the
    torch.distributed group that launched the ranks."""

    def __init__(self, ctx, group=None):
        import ctypes as C

        import torch.distributed as dist

        from . import _lib as L
        self._ctx = ctx
        self.rank, self.size = dist.get_rank(group), dist.get_world_size(group)
        uid = (C.c_uint8 * 128)()
        if self.rank == 0:
            L.check(L.lib().slat_comm_id(uid))
        box = [bytes(uid)]
        dist.broadcast_object_list(box, src=0, group=group)
        uid = (C.c_uint8 * 128).from_buffer_copy(box[0])
        self._p = C.c_void_p()
        L.check(L.lib().slat_comm_create(ctx.ptr, self.size, self.rank, uid, C.byref(self._p)), ctx.ptr)

    def close(self):
        from . import _lib as L
        if self._p:
            L.lib().slat_comm_destroy(self._p)
            self._p = None

    def bcast(self, m, cls, root: int = 0):
        """The root's device matrix on every rank (others pass None)."""
        import ctypes as C

        from . import _lib as L
        out = m._m if m is not None else L.CsrOwned()
        L.check(L.lib().slat_bcast_csr(self._ctx.ptr, self._p, C.byref(out), root), self._ctx.ptr)
        if m is not None:
            return m
        return cls(out, self._ctx)

    def allgather_rows(self, block):
        """C's row blocks of all ranks, in rank order, as one device matrix on every rank."""
        import ctypes as C

        from . import _lib as L
        v = block.view()
        out = L.CsrOwned()
        L.check(L.lib().slat_allgather_rows(self._ctx.ptr, self._p, C.byref(v), C.byref(out)), self._ctx.ptr)
        return type(block)(out, self._ctx)


def device_cuts(A, B, parts: int) -> list[int]:
    """flops_balanced_cuts computed on the device (slat_rowblock_cuts)."""
    import ctypes as C

    from . import _lib as L
    cuts = (C.c_uint64 * (parts + 1))()
    a, b = A.view(), B.view()
    L.check(L.lib().slat_rowblock_cuts(A._ctx.ptr, C.byref(a), C.byref(b), parts, cuts), A._ctx.ptr)
    return [int(c) for c in cuts]


def concat_rows(blocks, views=None):
    """Row blocks living on one device stacked into one matrix (slat_concat_rows): the allgatherv's
    assembly (offset tables, row ends taken relative to each block's first entry, rebase kernel)
    without the transport. `views` may replace the blocks' own views (views into larger matrices)."""
    import ctypes as C

    from . import _lib as L
    vs = views if views is not None else [b.view() for b in blocks]
    arr = (L.CsrView * len(vs))(*vs)
    out = L.CsrOwned()
    ctx = blocks[0]._ctx
    L.check(L.lib().slat_concat_rows(ctx.ptr, arr, len(vs), C.byref(out)), ctx.ptr)
    return type(blocks[0])(out, ctx)


def _to_i64(a: np.ndarray) -> np.ndarray:
    """Bit-preserving int64 view for transport (u32 widened, u64 / f64 reinterpreted)."""
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint32:
        return a.astype(np.int64)
    if a.dtype.itemsize == 8:
        return a.view(np.int64)
    raise TypeError(f"unsupported dtype {a.dtype}")


def _from_i64(a: np.ndarray, dtype) -> np.ndarray:
    dtype = np.dtype(dtype)
    if dtype == np.uint32:
        return a.astype(np.uint32)
    return a.view(dtype)


def gather_blocks(row_ptr: np.ndarray, col_idx: np.ndarray, values: np.ndarray, group=None, device=None):
    """Assemble the ranks' row blocks (in rank order) into the full CSR on every rank.

    row_ptr is the block's local row pointer (starting at 0). Returns (row_ptr, col_idx, values) of
    the concatenation, row_ptr rebased with the exclusive prefix of the blocks' nnz.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rp = np.asarray(row_ptr, dtype=np.int64)
    nrows, nnz = len(rp) - 1, int(rp[-1])
    meta = torch.tensor([nrows, nnz], dtype=torch.int64, device=device)
    metas = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    rows = [int(m[0]) for m in metas]
    nnzs = [int(m[1]) for m in metas]
    mr, mn = max(max(rows), 1), max(max(nnzs), 1)

    def allgather_padded(x: np.ndarray, pad_to: int):
        t = torch.zeros(pad_to, dtype=torch.int64, device=device)
        if len(x):
            t[: len(x)] = torch.from_numpy(_to_i64(x)).to(device)
        outs = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(outs, t, group=group)
        return [o.cpu().numpy() for o in outs]

    lens = allgather_padded(np.diff(rp), mr)
    cols = allgather_padded(np.asarray(col_idx, dtype=np.uint32), mn)
    vals = allgather_padded(np.asarray(values), mn)
    row_len = np.concatenate([lens[r][: rows[r]] for r in range(world)])
    out_rp = np.concatenate([[0], np.cumsum(row_len)]).astype(np.uint64)
    out_col = np.concatenate([cols[r][: nnzs[r]] for r in range(world)]).astype(np.uint32)
    out_val = np.concatenate([_from_i64(vals[r][: nnzs[r]], np.asarray(values).dtype) for r in range(world)])
    return out_rp, out_col, out_val
