// slat_dist.hip — the multi-GPU row-block layout of C = A·B, device-resident.
//
// The reference's only parallelism is matmul_par's split of output rows over rayon threads
// (src/graph_csr.rs:350-484); here the rows split over GPUs, one process per GPU:
//   * slat_rowblock_cuts — flops-balanced 1-D row cuts computed on the device: per-row products
//     sum_k nnz(B row k) over A's row (a kernel), their prefix (k_scan_rows), a binary search per cut;
//   * slat_spgemm_rowblock (slat_api.hip) — one rank's rows, B replicated;
//   * slat_bcast_csr — the replicated operand from one root over RCCL (one ncclBroadcast per array);
//   * slat_allgather_rows — the allgatherv of the ranks' C row blocks, in rank order, over RCCL: the
//     blocks' (rows, nnz, max row) by ncclAllGather, then one ncclBroadcast per root and array inside
//     one group (RCCL has no allgatherv), col_idx at 4 B and values at their native width, row_ptr
//     rebased on the device. Payload = nnz(C) * (4 + sizeof value) + rows * 8 bytes.
// RCCL over xGMI is point-to-point: the per-root broadcasts let RCCL route each block on its own
// rings/trees instead of padding every block to the largest one.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "slat.h"
#include "slat_internal.hpp"

struct slat_comm {
    ncclComm_t nc = nullptr;
    int nranks = 1, rank = 0, device = 0;
};

namespace {

constexpr int kB = 256;

#define SLAT_NCCL(ctx, expr)                                                                           \
    do {                                                                                               \
        ncclResult_t r_ = (expr);                                                                      \
        if (r_ != ncclSuccess) {                                                                       \
            (ctx)->err = std::string(#expr) + ": " + ncclGetErrorString(r_);                           \
            return SLAT_EHIP;                                                                          \
        }                                                                                              \
    } while (0)

unsigned grid_for(const slat_ctx *ctx, uint64_t n) {
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + kB - 1) / kB, (uint64_t)ctx->cu_count * 8));
}

// products of each row of A*B: sum over the row's entries k of nnz(B row k) (ids >= b_nrows: none)
__global__ __launch_bounds__(kB) void k_row_flops(const uint64_t *a_rp, const uint32_t *a_col, uint64_t nrows,
                                                   const uint64_t *b_rp, uint64_t b_nrows, uint64_t *flops) {
    for (uint64_t r = (uint64_t)blockIdx.x * kB + threadIdx.x; r < nrows; r += (uint64_t)gridDim.x * kB) {
        uint64_t f = 0;
        for (uint64_t i = a_rp[r], e = a_rp[r + 1]; i < e; ++i) {
            const uint32_t k = a_col[i];
            if (k < b_nrows) f += b_rp[k + 1] - b_rp[k];
        }
        flops[r] = f;
    }
}

// cut r (0 < r < parts) = the first row i with prefix[i + 1] * parts >= total * r (prefix[0] = 0,
// prefix[n] = total): block r - 1 ends before the row that reaches the r-th share of the products
// (slat.dist.flops_balanced_cuts restates the rule in numpy)
__global__ void k_cuts(const uint64_t *prefix, uint64_t n, uint32_t parts, uint64_t *cuts) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r > parts) return;
    if (r == 0 || r == parts) {
        cuts[r] = r == 0 ? 0 : n;
        return;
    }
    if (prefix[n] == 0) {  // no products at all: equal row counts
        cuts[r] = (uint64_t)((unsigned __int128)n * r / parts);
        return;
    }
    const unsigned __int128 target = (unsigned __int128)prefix[n] * r;
    uint64_t lo = 0, hi = n;  // first i in [0, n) with prefix[i + 1] * parts >= target, else n
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if ((unsigned __int128)prefix[mid + 1] * parts >= target)
            hi = mid;
        else
            lo = mid + 1;
    }
    cuts[r] = lo;
}

// full.row_ptr rows of block b: the broadcast local ends + the block's nnz offset
__global__ __launch_bounds__(kB) void k_rebase(uint64_t *rp, const uint64_t *row_off, const uint64_t *nnz_off,
                                                int nblocks) {
    if (blockIdx.x == 0 && threadIdx.x == 0) rp[0] = 0;
    for (int b = 0; b < nblocks; ++b) {
        const uint64_t r0 = row_off[b], r1 = row_off[b + 1], add = nnz_off[b];
        if (!add) continue;
        for (uint64_t i = r0 + (uint64_t)blockIdx.x * kB + threadIdx.x; i < r1; i += (uint64_t)gridDim.x * kB)
            rp[1 + i] += add;
    }
}

// ends[i] = rp[1 + i] - first: a view's row ends relative to its first entry
__global__ __launch_bounds__(kB) void k_rel_ends(const uint64_t *rp, uint64_t n, uint64_t first, uint64_t *ends) {
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kB) ends[i] = rp[1 + i] - first;
}

ncclDataType_t value_type(int32_t dt) {
    return dt == SLAT_U32 ? ncclUint32 : dt == SLAT_SAT64 ? ncclUint64 : ncclFloat64;
}

}  // namespace

extern "C" slat_status slat_comm_id(uint8_t id[128]) {
    if (!id) return SLAT_EINVAL;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return SLAT_EHIP;
    static_assert(sizeof u == 128, "RCCL unique id size");
    std::memcpy(id, &u, sizeof u);
    return SLAT_OK;
}

extern "C" slat_status slat_comm_create(slat_ctx *ctx, int nranks, int rank, const uint8_t id[128], slat_comm **out) {
    if (!ctx || !out || !id || nranks < 1 || rank < 0 || rank >= nranks) return SLAT_EINVAL;
    *out = nullptr;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    slat_comm *c = new slat_comm();
    c->nranks = nranks;
    c->rank = rank;
    c->device = ctx->device;
    const ncclResult_t r = ncclCommInitRank(&c->nc, nranks, u, rank);
    if (r != ncclSuccess) {
        ctx->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
        delete c;
        return SLAT_EHIP;
    }
    *out = c;
    return SLAT_OK;
}

extern "C" slat_status slat_comm_destroy(slat_comm *comm) {
    if (!comm) return SLAT_EINVAL;
    if (comm->nc) (void)ncclCommDestroy(comm->nc);
    delete comm;
    return SLAT_OK;
}

extern "C" slat_status slat_rowblock_cuts(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B, uint32_t parts,
                                          uint64_t *cuts) {
    if (!ctx || !cuts || parts < 1) return SLAT_EINVAL;
    slat_status st;
    if ((st = slat_check_view(ctx, A, "A")) || (st = slat_check_view(ctx, B, "B"))) return st;
    if (A->residency != SLAT_DEVICE || B->residency != SLAT_DEVICE) return fail(ctx, SLAT_EINVAL, "device views only");
    if (A->n_cols != B->n_rows) return fail(ctx, SLAT_EDIM, "A.n_cols != B.n_rows");
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    const hipStream_t s = ctx->stream;
    const uint64_t n = A->n_rows;
    uint8_t *blk = nullptr;  // flops [n] | prefix [n + 1] | cuts [parts + 1]
    const size_t fb = std::max<uint64_t>(n, 1) * 8, pb = (n + 1) * 8;
    SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&blk, fb + pb + (parts + 1) * 8, s));
    uint64_t *fl = (uint64_t *)blk, *pre = (uint64_t *)(blk + fb), *dc = (uint64_t *)(blk + fb + pb);
    if (n) {
        hipLaunchKernelGGL(k_row_flops, dim3(grid_for(ctx, n)), dim3(kB), 0, s, A->row_ptr, A->col_idx, n, B->row_ptr,
                           B->n_rows, fl);
        SLAT_HIP(ctx, hipGetLastError());
        if ((st = slat_launch_scan(ctx, fl, n, pre, s))) {
            slat_dev_free(ctx, blk, s);
            return st;
        }
    } else {
        SLAT_HIP(ctx, hipMemsetAsync(pre, 0, 8, s));
    }
    hipLaunchKernelGGL(k_cuts, dim3((parts + 1 + 63) / 64), dim3(64), 0, s, pre, n, parts, dc);
    SLAT_HIP(ctx, hipGetLastError());
    SLAT_HIP(ctx, hipMemcpyAsync(cuts, dc, (parts + 1) * 8, hipMemcpyDeviceToHost, s));
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    slat_dev_free(ctx, blk, s);
    // monotonic (a cut never passes the next one)
    for (uint32_t r = 1; r <= parts; ++r) cuts[r] = std::max(cuts[r], cuts[r - 1]);
    return SLAT_OK;
}

extern "C" slat_status slat_bcast_csr(slat_ctx *ctx, slat_comm *comm, slat_csr *m, int root) {
    if (!ctx || !comm || !m || root < 0 || root >= comm->nranks) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    const hipStream_t s = ctx->stream;
    // shape first: (rows, cols, nnz, dtype, max row) from the root
    uint64_t meta[5] = {m->n_rows, m->n_cols, m->nnz, (uint64_t)m->dtype, m->max_row_nnz};
    uint64_t *dmeta = nullptr;
    SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&dmeta, sizeof meta, s));
    SLAT_HIP(ctx, hipMemcpyAsync(dmeta, meta, sizeof meta, hipMemcpyHostToDevice, s));
    SLAT_NCCL(ctx, ncclBroadcast(dmeta, dmeta, 5, ncclUint64, root, comm->nc, s));
    SLAT_HIP(ctx, hipMemcpyAsync(meta, dmeta, sizeof meta, hipMemcpyDeviceToHost, s));
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    slat_dev_free(ctx, dmeta, s);
    const int32_t dt = (int32_t)meta[3];
    if (dt < SLAT_U32 || dt > SLAT_F64) return fail(ctx, SLAT_EINVAL, "broadcast matrix: bad dtype");
    if (comm->rank != root) {
        std::memset(m, 0, sizeof *m);
        SLAT_HIP(ctx, alloc_joint(ctx, m, meta[0], meta[2], vsize(dt), s));
        m->n_rows = meta[0];
        m->n_cols = meta[1];
        m->nnz = meta[2];
        m->capacity = meta[2];
        m->dtype = dt;
        m->max_row_nnz = meta[4];
        m->device = ctx->device;
    }
    SLAT_NCCL(ctx, ncclGroupStart());
    SLAT_NCCL(ctx, ncclBroadcast(m->row_ptr, m->row_ptr, m->n_rows + 1, ncclUint64, root, comm->nc, s));
    if (m->nnz) {
        SLAT_NCCL(ctx, ncclBroadcast(m->col_idx, m->col_idx, m->nnz, ncclUint32, root, comm->nc, s));
        SLAT_NCCL(ctx, ncclBroadcast(m->values, m->values, m->nnz, value_type(dt), root, comm->nc, s));
    }
    SLAT_NCCL(ctx, ncclGroupEnd());
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    return SLAT_OK;
}

extern "C" slat_status slat_allgather_rows(slat_ctx *ctx, slat_comm *comm, const slat_csr_view *block, slat_csr *full) {
    if (!ctx || !comm || !block || !full) return SLAT_EINVAL;
    slat_status st;
    if ((st = slat_check_view(ctx, block, "block"))) return st;
    if (block->residency != SLAT_DEVICE) return fail(ctx, SLAT_EINVAL, "device views only");
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    const hipStream_t s = ctx->stream;
    const int P = comm->nranks;
    const int32_t dt = block->dtype;
    // every block's (rows, nnz, max row, dtype, first row_ptr entry); a block's row_ptr may be a view
    // into a larger matrix (absolute offsets), so its entries are relative to row_ptr[0]
    uint64_t first = 0;
    if (block->n_rows) SLAT_HIP(ctx, hipMemcpyAsync(&first, block->row_ptr, 8, hipMemcpyDeviceToHost, s));
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    const uint64_t mine[4] = {block->n_rows, block->nnz, block->max_row_nnz, (uint64_t)dt};
    std::vector<uint64_t> all((size_t)4 * P);
    uint64_t *dm = nullptr;
    SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&dm, (size_t)(4 + 4 * P) * 8, s));
    SLAT_HIP(ctx, hipMemcpyAsync(dm, mine, sizeof mine, hipMemcpyHostToDevice, s));
    SLAT_NCCL(ctx, ncclAllGather(dm, dm + 4, 4, ncclUint64, comm->nc, s));
    SLAT_HIP(ctx, hipMemcpyAsync(all.data(), dm + 4, all.size() * 8, hipMemcpyDeviceToHost, s));
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    slat_dev_free(ctx, dm, s);
    std::vector<uint64_t> row_off(P + 1, 0), nnz_off(P + 1, 0);
    uint64_t maxrow = 0;
    for (int r = 0; r < P; ++r) {
        if ((int32_t)all[4 * r + 3] != dt) return fail(ctx, SLAT_EINVAL, "ranks' blocks differ in value type");
        row_off[r + 1] = row_off[r] + all[4 * r];
        nnz_off[r + 1] = nnz_off[r] + all[4 * r + 1];
        maxrow = std::max(maxrow, all[4 * r + 2]);
    }
    std::memset(full, 0, sizeof *full);
    SLAT_HIP(ctx, alloc_joint(ctx, full, row_off[P], nnz_off[P], vsize(dt), s));
    full->n_rows = row_off[P];
    full->n_cols = block->n_cols;
    full->nnz = nnz_off[P];
    full->capacity = std::max<uint64_t>(nnz_off[P], 1);
    full->dtype = dt;
    full->max_row_nnz = maxrow;
    full->device = ctx->device;
    // the blocks' row ends (local, rebased below), columns and values: one broadcast per root and array
    const bool me_rel = first == 0;
    uint64_t *my_ends = nullptr;  // this block's row_ptr[1..] relative to its first entry
    if (!me_rel && block->n_rows) {
        SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&my_ends, block->n_rows * 8, s));
        hipLaunchKernelGGL(k_rel_ends, dim3(grid_for(ctx, block->n_rows)), dim3(kB), 0, s, block->row_ptr, block->n_rows,
                           first, my_ends);
        SLAT_HIP(ctx, hipGetLastError());
    }
    const uint8_t *my_col = (const uint8_t *)block->col_idx + first * 4;
    const uint8_t *my_val = (const uint8_t *)block->values + first * vsize(dt);
    SLAT_NCCL(ctx, ncclGroupStart());
    for (int r = 0; r < P; ++r) {
        const uint64_t rows = all[4 * r], nz = all[4 * r + 1];
        const bool me = r == comm->rank;
        if (rows)
            SLAT_NCCL(ctx, ncclBroadcast(me ? (const void *)(me_rel ? block->row_ptr + 1 : my_ends) : nullptr,
                                         full->row_ptr + 1 + row_off[r], rows, ncclUint64, r, comm->nc, s));
        if (nz) {
            SLAT_NCCL(ctx, ncclBroadcast(me ? (const void *)my_col : nullptr, full->col_idx + nnz_off[r], nz, ncclUint32,
                                         r, comm->nc, s));
            SLAT_NCCL(ctx, ncclBroadcast(me ? (const void *)my_val : nullptr,
                                         (uint8_t *)full->values + nnz_off[r] * vsize(dt), nz, value_type(dt), r,
                                         comm->nc, s));
        }
    }
    SLAT_NCCL(ctx, ncclGroupEnd());
    // rebase: block r's (relative) row ends + nnz_off[r]
    std::vector<uint64_t> add(P + 1, 0);
    for (int r = 0; r < P; ++r) add[r] = nnz_off[r];
    uint64_t *tab = nullptr;
    SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&tab, (size_t)(2 * P + 2) * 8, s));
    SLAT_HIP(ctx, hipMemcpyAsync(tab, row_off.data(), (P + 1) * 8, hipMemcpyHostToDevice, s));
    SLAT_HIP(ctx, hipMemcpyAsync(tab + P + 1, add.data(), (P + 1) * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_rebase, dim3(grid_for(ctx, std::max<uint64_t>(row_off[P], 1))), dim3(kB), 0, s, full->row_ptr,
                       tab, tab + P + 1, P);
    SLAT_HIP(ctx, hipGetLastError());
    if (my_ends) slat_dev_free(ctx, my_ends, s);
    slat_dev_free(ctx, tab, s);
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    return SLAT_OK;
}
