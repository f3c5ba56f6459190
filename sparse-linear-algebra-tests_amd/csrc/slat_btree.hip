// slat_btree.hip — CsrBTreeMatrix in its own layout.
//
// The reference's CsrBTreeMatrix (src/graph_csr_btree.rs:44-52) keeps each row's columns as a dense
// B-tree: DenseBTreeList (src/dense_btree.rs:269-330) packs every row as [internal separator nodes |
// sorted data] into one flat `nodes` Vec, with a NodeEntry per row {offset, internal_len, total_len,
// data_start}; the values are one flat Vec indexed by data_start, so data_start is a CSR row_ptr
// over the values while the columns sit at a per-row shift inside `nodes`. matmul_par (:350-479) is
// the CSR two-pass product over those slices and ends in from_flat(n, row_ptr, col_idx, values)
// (:99), which builds the output's trees on the host.
//
// slat_spgemm_btree takes that layout as it lies in the Rust Vecs: one kernel gathers every row's
// data slice out of `nodes` into CSR order (a wave per row, coalesced), the u32 SpGEMM of
// slat_api.hip runs on (data_start, gathered columns, values), and C comes back as CSR: the arrays the
// reference hands to from_flat. The separator nodes are never read.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "slat.h"
#include "slat_internal.hpp"

namespace {

constexpr int kB = 256;

// cols[data_start[r] + i] = nodes[data_off[r] + i] for every row; a slice past n_nodes or nnz, a
// column >= n_cols or a decreasing data_start sets *bad (the gathered column is then not used)
__global__ __launch_bounds__(kB) void k_gather_btree_cols(const uint64_t *data_start, const uint64_t *data_off,
                                                          const uint32_t *nodes, uint64_t n_rows, uint64_t n_nodes,
                                                          uint64_t nnz, uint64_t n_cols, uint32_t *cols,
                                                          unsigned int *bad) {
    const int lane = threadIdx.x & 63;
    const uint64_t waves = (uint64_t)gridDim.x * (kB / 64);
    bool b = false;
    for (uint64_t r = (uint64_t)blockIdx.x * (kB / 64) + threadIdx.x / 64; r < n_rows; r += waves) {
        const uint64_t s = data_start[r], e = data_start[r + 1], off = data_off[r];
        if (e < s || e > nnz || off > n_nodes || e - s > n_nodes - off) {
            b = true;
            continue;
        }
        for (uint64_t i = lane; i < e - s; i += 64) {
            const uint32_t c = nodes[off + i];
            b |= c >= n_cols;
            cols[s + i] = c;
        }
    }
    if (__any(b) && lane == 0) atomicOr(bad, 1u);
}

unsigned grid_for(const slat_ctx *ctx, uint64_t rows) {
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((rows + 3) / 4, (uint64_t)ctx->cu_count * 8));
}

// a device u32 CSR view of m: its data_start as row_ptr, the columns gathered into `*cols`, its
// values; host views are copied up first into one block `*stage`
slat_status gather_view(slat_ctx *ctx, const slat_btree_view *m, const char *name, slat_csr_view *out, uint32_t **cols,
                        uint8_t **stage, unsigned int *bad) {
    const std::string nm(name);
    if (!m) return fail(ctx, SLAT_EINVAL, nm + " is null");
    if (!m->data_start || (m->n_rows && !m->data_off)) return fail(ctx, SLAT_EINVAL, nm + ": null row arrays");
    if (m->nnz && (!m->nodes || !m->values)) return fail(ctx, SLAT_EINVAL, nm + ": null arrays");
    if (m->n_cols > 0xFFFFFFFFull || m->n_rows > 0xFFFFFFFFull)
        return fail(ctx, SLAT_ENOTSUP, nm + ": dims exceed NodeId (u32)");
    const hipStream_t s = ctx->stream;
    const uint64_t *ds = m->data_start, *off = m->data_off;
    const uint32_t *nodes = m->nodes, *val = m->values;
    if (m->residency == SLAT_HOST) {
        // one device block: data_start | data_off | nodes | values
        auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
        const size_t ds_b = up((m->n_rows + 1) * 8), off_b = up(std::max<uint64_t>(m->n_rows, 1) * 8),
                     nd_b = up(std::max<uint64_t>(m->n_nodes, 1) * 4), v_b = up(std::max<uint64_t>(m->nnz, 1) * 4);
        SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)stage, ds_b + off_b + nd_b + v_b, s));
        uint8_t *blk = *stage;
        SLAT_HIP(ctx, hipMemcpyAsync(blk, ds, (m->n_rows + 1) * 8, hipMemcpyHostToDevice, s));
        if (m->n_rows) SLAT_HIP(ctx, hipMemcpyAsync(blk + ds_b, off, m->n_rows * 8, hipMemcpyHostToDevice, s));
        if (m->n_nodes)
            SLAT_HIP(ctx, hipMemcpyAsync(blk + ds_b + off_b, nodes, m->n_nodes * 4, hipMemcpyHostToDevice, s));
        if (m->nnz) SLAT_HIP(ctx, hipMemcpyAsync(blk + ds_b + off_b + nd_b, val, m->nnz * 4, hipMemcpyHostToDevice, s));
        ds = (const uint64_t *)blk;
        off = (const uint64_t *)(blk + ds_b);
        nodes = (const uint32_t *)(blk + ds_b + off_b);
        val = (const uint32_t *)(blk + ds_b + off_b + nd_b);
    }
    SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)cols, std::max<uint64_t>(m->nnz, 1) * 4, s));
    if (m->n_rows) {
        hipLaunchKernelGGL(k_gather_btree_cols, dim3(grid_for(ctx, m->n_rows)), dim3(kB), 0, s, ds, off, nodes,
                           m->n_rows, m->n_nodes, m->nnz, m->n_cols, *cols, bad);
        SLAT_HIP(ctx, hipGetLastError());
    }
    std::memset(out, 0, sizeof *out);
    out->n_rows = m->n_rows;
    out->n_cols = m->n_cols;
    out->nnz = m->nnz;
    out->row_ptr = ds;
    out->col_idx = *cols;
    out->values = val;
    out->dtype = SLAT_U32;
    out->residency = SLAT_DEVICE;
    out->max_row_nnz = m->max_row_nnz;
    return SLAT_OK;
}

}  // namespace

extern "C" slat_status slat_spgemm_btree(slat_ctx *ctx, const slat_btree_view *A, const slat_btree_view *B,
                                         slat_csr *C, uint32_t flags) {
    if (!ctx || !C) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    std::memset(C, 0, sizeof *C);
    // assert_eq!(self.n, other.n) (src/graph_csr_btree.rs:351): square matrices of one size
    if (A && B && (A->n_cols != B->n_rows)) return fail(ctx, SLAT_EDIM, "A.n_cols != B.n_rows");
    const hipStream_t s = ctx->stream;
    unsigned int *bad = (unsigned int *)(ctx->d_words + 4);  // context scratch word, cleared on the stream
    SLAT_HIP(ctx, hipMemsetAsync(bad, 0, 4, s));
    slat_csr_view va, vb;
    uint32_t *ca = nullptr, *cb = nullptr;
    uint8_t *sa = nullptr, *sb = nullptr;
    auto release = [&]() {
        for (void *p : {(void *)ca, (void *)cb, (void *)sa, (void *)sb})
            if (p) slat_dev_free(ctx, p, s);
    };
    slat_status st = gather_view(ctx, A, "A", &va, &ca, &sa, bad);
    if (!st) st = gather_view(ctx, B, "B", &vb, &cb, &sb, bad);
    if (st) {
        release();
        return st;
    }
    // the gathers' verdict before the product reads their columns
    unsigned int hbad = 0;
    SLAT_HIP(ctx, hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    if (hbad) {
        release();
        return fail(ctx, SLAT_EINVAL, "a row slice lies outside nodes, or a column id is >= n_cols");
    }
    st = slat_spgemm_csr_u32(ctx, &va, &vb, C, flags);  // synchronous
    release();
    return st;
}
