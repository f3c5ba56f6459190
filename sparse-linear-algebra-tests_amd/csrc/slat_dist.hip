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
    // device words of the collectives' own metadata, allocated with the communicator so no rank can
    // fail an allocation between entering a call and reaching its first collective:
    // [0, 8) status agreement and broadcast shape, [8, 8 + 5 (P + 1)) the allgather's block metadata
    uint64_t *scratch = nullptr;
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
    if (hipMalloc((void **)&c->scratch, (size_t)(8 + 5 * (nranks + 1)) * 8) != hipSuccess) {
        delete c;
        return fail(ctx, SLAT_EOOM, "communicator scratch allocation failed");
    }
    const ncclResult_t r = ncclCommInitRank(&c->nc, nranks, u, rank);
    if (r != ncclSuccess) {
        ctx->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
        (void)hipFree(c->scratch);
        delete c;
        return SLAT_EHIP;
    }
    *out = c;
    return SLAT_OK;
}

extern "C" slat_status slat_comm_destroy(slat_comm *comm) {
    if (!comm) return SLAT_EINVAL;
    if (comm->nc) (void)ncclCommDestroy(comm->nc);
    if (comm->scratch) (void)hipFree(comm->scratch);
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

// RCCL calls whose failure must not strand the other ranks: the first error is kept and the caller
// still reaches ncclGroupEnd / the status agreement
#define SLAT_NCCL_KEEP(ctx, st, expr)                                                                  \
    do {                                                                                               \
        ncclResult_t r_ = (expr);                                                                      \
        if (r_ != ncclSuccess && (st) == SLAT_OK) {                                                    \
            (ctx)->err = std::string(#expr) + ": " + ncclGetErrorString(r_);                           \
            (st) = SLAT_EHIP;                                                                          \
        }                                                                                              \
    } while (0)

namespace {

// every rank's status agreed on (the max over ranks) before data moves: a rank that failed to
// allocate must not leave the others blocked inside broadcasts it never joins
slat_status agree(slat_ctx *ctx, slat_comm *comm, slat_status mine) {
    const hipStream_t s = ctx->stream;
    uint32_t *w = (uint32_t *)comm->scratch;  // allocated with the communicator: no failure here
    uint32_t v = (uint32_t)mine, got = 0;
    slat_status st = SLAT_OK;
    if (hipMemcpyAsync(w, &v, 4, hipMemcpyHostToDevice, s) != hipSuccess) st = SLAT_EHIP;
    SLAT_NCCL_KEEP(ctx, st, ncclAllReduce(w, w + 1, 1, ncclUint32, ncclMax, comm->nc, s));
    if (hipMemcpyAsync(&got, w + 1, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        st = SLAT_EHIP;
    if (st != SLAT_OK) return st;
    if (got != SLAT_OK && mine == SLAT_OK) return fail(ctx, (slat_status)got, "another rank failed");
    return (slat_status)got;
}

// The row-block assembly shared by slat_allgather_rows (blocks from every rank over RCCL) and
// slat_concat_rows (blocks on this device): block r's rows land at row_off[r], its entries at
// nnz_off[r]; its row ends are copied relative to its own first entry and rebased on the device.
struct Assembly {
    std::vector<uint64_t> row_off, nnz_off;
    uint64_t maxrow = 0;
    uint64_t *tab = nullptr;  // device: row_off [P + 1] | nnz_off [P + 1]
};

// offsets from every block's (rows, nnz, max row, dtype); C's arrays and the device offset table
slat_status assembly_plan(slat_ctx *ctx, const uint64_t *meta, int P, int32_t dt, uint64_t n_cols, Assembly &a,
                          slat_csr *full) {
    a.row_off.assign(P + 1, 0);
    a.nnz_off.assign(P + 1, 0);
    for (int r = 0; r < P; ++r) {
        if ((int32_t)meta[4 * r + 3] != dt) return fail(ctx, SLAT_EINVAL, "the row blocks differ in value type");
        a.row_off[r + 1] = a.row_off[r] + meta[4 * r];
        a.nnz_off[r + 1] = a.nnz_off[r] + meta[4 * r + 1];
        a.maxrow = std::max(a.maxrow, meta[4 * r + 2]);
    }
    const hipStream_t s = ctx->stream;
    std::memset(full, 0, sizeof *full);
    if (alloc_joint(ctx, full, a.row_off[P], a.nnz_off[P], vsize(dt), s) != hipSuccess)
        return fail(ctx, SLAT_EOOM, "assembled matrix allocation failed");
    full->n_rows = a.row_off[P];
    full->n_cols = n_cols;
    full->nnz = a.nnz_off[P];
    full->capacity = std::max<uint64_t>(a.nnz_off[P], 1);
    full->dtype = dt;
    full->max_row_nnz = a.maxrow;
    full->device = ctx->device;
    if (slat_dev_alloc(ctx, (void **)&a.tab, (size_t)(2 * P + 2) * 8, s) != hipSuccess) {
        slat_csr_free(ctx, full);
        return fail(ctx, SLAT_EOOM, "offset table allocation failed");
    }
    if (hipMemcpyAsync(a.tab, a.row_off.data(), (P + 1) * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(a.tab + P + 1, a.nnz_off.data(), (P + 1) * 8, hipMemcpyHostToDevice, s) != hipSuccess) {
        slat_dev_free(ctx, a.tab, s);
        a.tab = nullptr;
        slat_csr_free(ctx, full);
        return fail(ctx, SLAT_EHIP, "offset table upload failed");
    }
    return SLAT_OK;
}

// full.row_ptr[0] = 0 and block r's row ends + nnz_off[r], then the stream drained
slat_status assembly_finish(slat_ctx *ctx, Assembly &a, slat_csr *full, int P) {
    const hipStream_t s = ctx->stream;
    hipLaunchKernelGGL(k_rebase, dim3(grid_for(ctx, std::max<uint64_t>(a.row_off[P], 1))), dim3(kB), 0, s, full->row_ptr,
                       a.tab, a.tab + P + 1, P);
    const hipError_t e = hipGetLastError();
    slat_dev_free(ctx, a.tab, s);
    a.tab = nullptr;
    SLAT_HIP(ctx, e);
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    return SLAT_OK;
}

// a block's row ends relative to its first entry: the view's own row_ptr + 1 when it starts at 0,
// else a temporary (*tmp, freed by the caller) filled by k_rel_ends
slat_status rel_ends(slat_ctx *ctx, const slat_csr_view *b, uint64_t first, const uint64_t **ends, uint64_t **tmp) {
    *tmp = nullptr;
    *ends = b->row_ptr + 1;
    if (first == 0 || b->n_rows == 0) return SLAT_OK;
    const hipStream_t s = ctx->stream;
    if (slat_dev_alloc(ctx, (void **)tmp, b->n_rows * 8, s) != hipSuccess) return fail(ctx, SLAT_EOOM, "row-end scratch");
    hipLaunchKernelGGL(k_rel_ends, dim3(grid_for(ctx, b->n_rows)), dim3(kB), 0, s, b->row_ptr, b->n_rows, first, *tmp);
    SLAT_HIP(ctx, hipGetLastError());
    *ends = *tmp;
    return SLAT_OK;
}

}  // namespace

extern "C" slat_status slat_bcast_csr(slat_ctx *ctx, slat_comm *comm, slat_csr *m, int root) {
    if (!ctx || !comm || !m || root < 0 || root >= comm->nranks) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    const hipStream_t s = ctx->stream;
    // shape first: (rows, cols, nnz, dtype, max row) from the root
    uint64_t meta[5] = {m->n_rows, m->n_cols, m->nnz, (uint64_t)m->dtype, m->max_row_nnz};
    uint64_t *dmeta = comm->scratch + 2;  // words 2..6 (0..1: the status agreement)
    slat_status st = SLAT_OK;
    if (hipMemcpyAsync(dmeta, meta, sizeof meta, hipMemcpyHostToDevice, s) != hipSuccess) st = fail(ctx, SLAT_EHIP, "meta upload");
    SLAT_NCCL_KEEP(ctx, st, ncclBroadcast(dmeta, dmeta, 5, ncclUint64, root, comm->nc, s));
    if (hipMemcpyAsync(meta, dmeta, sizeof meta, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        if (st == SLAT_OK) st = fail(ctx, SLAT_EHIP, "meta read-back");
    if (st != SLAT_OK) return st;
    const int32_t dt = (int32_t)meta[3];
    if (dt < SLAT_U32 || dt > SLAT_F64) return fail(ctx, SLAT_EINVAL, "broadcast matrix: bad dtype");  // on every rank
    slat_status mine = SLAT_OK;
    if (comm->rank != root) {
        std::memset(m, 0, sizeof *m);
        if (alloc_joint(ctx, m, meta[0], meta[2], vsize(dt), s) != hipSuccess) {
            std::memset(m, 0, sizeof *m);
            mine = fail(ctx, SLAT_EOOM, "broadcast matrix allocation failed");
        } else {
            m->n_rows = meta[0];
            m->n_cols = meta[1];
            m->nnz = meta[2];
            m->capacity = meta[2];
            m->dtype = dt;
            m->max_row_nnz = meta[4];
            m->device = ctx->device;
        }
    }
    if ((st = agree(ctx, comm, mine)) != SLAT_OK) {
        if (comm->rank != root && m->row_ptr) slat_csr_free(ctx, m);
        return st;
    }
    SLAT_NCCL_KEEP(ctx, st, ncclGroupStart());
    SLAT_NCCL_KEEP(ctx, st, ncclBroadcast(m->row_ptr, m->row_ptr, meta[0] + 1, ncclUint64, root, comm->nc, s));
    if (meta[2]) {
        SLAT_NCCL_KEEP(ctx, st, ncclBroadcast(m->col_idx, m->col_idx, meta[2], ncclUint32, root, comm->nc, s));
        SLAT_NCCL_KEEP(ctx, st, ncclBroadcast(m->values, m->values, meta[2], value_type(dt), root, comm->nc, s));
    }
    SLAT_NCCL_KEEP(ctx, st, ncclGroupEnd());
    if (st != SLAT_OK) return st;
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    return SLAT_OK;
}

extern "C" slat_status slat_allgather_rows(slat_ctx *ctx, slat_comm *comm, const slat_csr_view *block, slat_csr *full) {
    if (!ctx || !comm || !block || !full) return SLAT_EINVAL;
    std::memset(full, 0, sizeof *full);
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    // a malformed block is not returned on at once: every rank must reach the metadata gather, so
    // the block travels as an invalid dtype and every rank refuses the assembly together
    slat_status vst = slat_check_view(ctx, block, "block");
    if (vst == SLAT_OK && block->residency != SLAT_DEVICE) vst = fail(ctx, SLAT_EINVAL, "device views only");
    const hipStream_t s = ctx->stream;
    const int P = comm->nranks;
    const int32_t dt = vst == SLAT_OK ? block->dtype : -1;
    // every block's (rows, nnz, max row, dtype); a block's row_ptr may be a view into a larger matrix
    // (absolute offsets), so its entries are taken relative to row_ptr[0]
    // (a failed read of it also travels as an invalid dtype: no rank returns before the gather)
    uint64_t first = 0;
    if (vst == SLAT_OK && block->n_rows &&
        (hipMemcpyAsync(&first, block->row_ptr, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
         hipStreamSynchronize(s) != hipSuccess))
        vst = fail(ctx, SLAT_EHIP, "block row_ptr read-back");
    const int32_t dtm = vst == SLAT_OK ? dt : -1;
    // (rows, nnz, max row, dtype, columns) of every block: the columns must agree on every rank
    const uint64_t mine[5] = {vst == SLAT_OK ? block->n_rows : 0, vst == SLAT_OK ? block->nnz : 0,
                              vst == SLAT_OK ? block->max_row_nnz : 0, (uint64_t)(int64_t)dtm,
                              vst == SLAT_OK ? block->n_cols : 0};
    std::vector<uint64_t> all5((size_t)5 * P), all((size_t)4 * P);
    uint64_t *dm = comm->scratch + 8;  // allocated with the communicator
    slat_status st = SLAT_OK;
    if (hipMemcpyAsync(dm, mine, sizeof mine, hipMemcpyHostToDevice, s) != hipSuccess) st = fail(ctx, SLAT_EHIP, "meta upload");
    SLAT_NCCL_KEEP(ctx, st, ncclAllGather(dm, dm + 5, 5, ncclUint64, comm->nc, s));
    if ((hipMemcpyAsync(all5.data(), dm + 5, all5.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
         hipStreamSynchronize(s) != hipSuccess) && st == SLAT_OK)
        st = fail(ctx, SLAT_EHIP, "meta read-back");
    if (st != SLAT_OK) return st;
    for (int r = 0; r < P; ++r) {
        for (int k = 0; k < 4; ++k) all[4 * r + k] = all5[5 * r + k];
        if ((int32_t)all5[5 * r + 3] < SLAT_U32 || (int32_t)all5[5 * r + 3] > SLAT_F64)
            return vst != SLAT_OK ? vst : fail(ctx, SLAT_EINVAL, "another rank's block is malformed");
    }
    for (int r = 0; r < P; ++r)  // the same verdict on every rank: every rank saw the same words
        if ((int32_t)all5[5 * r + 3] != (int32_t)all5[3] || all5[5 * r + 4] != all5[4])
            return fail(ctx, SLAT_EDIM, "the row blocks differ in value type or columns");
    // every allocation before the data moves, then one agreed status
    Assembly a;
    uint64_t *my_ends_tmp = nullptr;
    const uint64_t *my_ends = nullptr;
    slat_status mine_st = assembly_plan(ctx, all.data(), P, dt, block->n_cols, a, full);  // same verdict on every rank
    if (mine_st == SLAT_OK) mine_st = rel_ends(ctx, block, first, &my_ends, &my_ends_tmp);
    auto cleanup = [&]() {
        if (my_ends_tmp) slat_dev_free(ctx, my_ends_tmp, s);
        if (a.tab) slat_dev_free(ctx, a.tab, s);
        a.tab = nullptr;
    };
    if ((st = agree(ctx, comm, mine_st)) != SLAT_OK) {
        cleanup();
        if (full->row_ptr) slat_csr_free(ctx, full);
        return st;
    }
    // the blocks' row ends (relative, rebased below), columns and values: one broadcast per root and
    // array, inside one group that is always closed
    const uint8_t *my_col = (const uint8_t *)block->col_idx + first * 4;
    const uint8_t *my_val = (const uint8_t *)block->values + first * vsize(dt);
    SLAT_NCCL_KEEP(ctx, st, ncclGroupStart());
    // every rank issues the same sequence of broadcasts whatever happened locally (an enqueue error
    // is kept, the rest still issued, then the ranks agree): stopping early would leave the peers
    // blocked inside broadcasts this rank never joined
    for (int r = 0; r < P; ++r) {
        const uint64_t rows = all[4 * r], nz = all[4 * r + 1];
        const bool me = r == comm->rank;
        if (rows)
            SLAT_NCCL_KEEP(ctx, st, ncclBroadcast(me ? (const void *)my_ends : nullptr, full->row_ptr + 1 + a.row_off[r],
                                                  rows, ncclUint64, r, comm->nc, s));
        if (nz) {
            SLAT_NCCL_KEEP(ctx, st, ncclBroadcast(me ? (const void *)my_col : nullptr, full->col_idx + a.nnz_off[r], nz,
                                                  ncclUint32, r, comm->nc, s));
            SLAT_NCCL_KEEP(ctx, st, ncclBroadcast(me ? (const void *)my_val : nullptr,
                                                  (uint8_t *)full->values + a.nnz_off[r] * vsize(dt), nz, value_type(dt),
                                                  r, comm->nc, s));
        }
    }
    SLAT_NCCL_KEEP(ctx, st, ncclGroupEnd());
    if (st == SLAT_OK) st = assembly_finish(ctx, a, full, P);
    st = agree(ctx, comm, st);
    cleanup();
    if (st != SLAT_OK && full->row_ptr) {
        (void)hipStreamSynchronize(s);
        slat_csr_free(ctx, full);
    }
    return st;
}

extern "C" slat_status slat_concat_rows(slat_ctx *ctx, const slat_csr_view *blocks, uint32_t nblocks, slat_csr *full) {
    if (!ctx || !full || (nblocks && !blocks)) return SLAT_EINVAL;
    std::memset(full, 0, sizeof *full);
    if (nblocks == 0) return fail(ctx, SLAT_EINVAL, "no blocks");
    slat_status st;
    for (uint32_t r = 0; r < nblocks; ++r) {
        if ((st = slat_check_view(ctx, &blocks[r], "block"))) return st;
        if (blocks[r].residency != SLAT_DEVICE) return fail(ctx, SLAT_EINVAL, "device views only");
        if (blocks[r].n_cols != blocks[0].n_cols) return fail(ctx, SLAT_EDIM, "the row blocks differ in columns");
    }
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    const hipStream_t s = ctx->stream;
    const int P = (int)nblocks;
    const int32_t dt = blocks[0].dtype;
    std::vector<uint64_t> meta((size_t)4 * P), first(P, 0);
    for (int r = 0; r < P; ++r) {
        if (blocks[r].n_rows) SLAT_HIP(ctx, hipMemcpyAsync(&first[r], blocks[r].row_ptr, 8, hipMemcpyDeviceToHost, s));
        meta[4 * r] = blocks[r].n_rows;
        meta[4 * r + 1] = blocks[r].nnz;
        meta[4 * r + 2] = blocks[r].max_row_nnz;
        meta[4 * r + 3] = (uint64_t)blocks[r].dtype;
    }
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    Assembly a;
    if ((st = assembly_plan(ctx, meta.data(), P, dt, blocks[0].n_cols, a, full))) return st;
    const size_t vs = vsize(dt);
    std::vector<uint64_t *> tmps;
    for (int r = 0; r < P && st == SLAT_OK; ++r) {
        const slat_csr_view &b = blocks[r];
        const uint64_t *ends = nullptr;
        uint64_t *tmp = nullptr;
        st = rel_ends(ctx, &b, first[r], &ends, &tmp);
        if (tmp) tmps.push_back(tmp);  // freed below, also when rel_ends failed after allocating it
        if (st) break;
        hipError_t e = hipSuccess;
        if (b.n_rows)
            e = hipMemcpyAsync(full->row_ptr + 1 + a.row_off[r], ends, b.n_rows * 8, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess && b.nnz)
            e = hipMemcpyAsync(full->col_idx + a.nnz_off[r], (const uint8_t *)b.col_idx + first[r] * 4, b.nnz * 4,
                               hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess && b.nnz)
            e = hipMemcpyAsync((uint8_t *)full->values + a.nnz_off[r] * vs, (const uint8_t *)b.values + first[r] * vs,
                               b.nnz * vs, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) st = fail(ctx, SLAT_EHIP, std::string("block copy: ") + hipGetErrorString(e));
    }
    if (st == SLAT_OK) st = assembly_finish(ctx, a, full, P);
    if (a.tab) slat_dev_free(ctx, a.tab, s);
    for (uint64_t *t : tmps) slat_dev_free(ctx, t, s);
    if (st != SLAT_OK) {
        (void)hipStreamSynchronize(s);
        slat_csr_free(ctx, full);
    }
    return st;
}
