// slat_magnus.hip — MagnusMatrix with its own column type.
//
// The reference's MagnusMatrix wraps magnus::SparseMatrixCSR<Sat64>, whose col_idx is Vec<usize>
// (src/graph_magnus.rs:11-14, built by from_coo :34-76), i.e. 8-byte column ids. These entry points
// take and return that layout, so a Rust caller hands its Vecs over without narrowing or widening
// them on the host. Inside, the column ids are narrowed to u32 on the device (n_cols < 2^32 is
// checked there), the Sat64 SpGEMM of slat_api.hip runs, and C's columns are widened back to u64
// into their own block; C's row_ptr and values stay in the SpGEMM's output block.
#include <hip/hip_runtime.h>

#include <cstring>

#include "slat.h"
#include "slat_internal.hpp"

namespace {

constexpr int kB = 256;

// u64 -> u32 column ids; a column >= 2^32 (or >= n_cols) sets *bad
__global__ __launch_bounds__(kB) void k_narrow_cols(const uint64_t *src, uint64_t n, uint64_t n_cols, uint32_t *dst,
                                                     unsigned int *bad) {
    bool b = false;
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kB) {
        const uint64_t c = src[i];
        b |= c >= n_cols;
        dst[i] = (uint32_t)c;
    }
    if (__any(b) && (threadIdx.x & 63) == 0) atomicOr(bad, 1u);
}

// u32 -> u64 column ids, two per thread (8-byte loads, 16-byte stores)
__global__ __launch_bounds__(kB) void k_widen_cols(const uint32_t *src, uint64_t n, uint64_t *dst) {
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; 2 * i < n; i += (uint64_t)gridDim.x * kB) {
        if (2 * i + 1 < n) {
            const uint2 v = *(const uint2 *)(src + 2 * i);
            *(ulonglong2 *)(dst + 2 * i) = make_ulonglong2(v.x, v.y);
        } else {
            dst[2 * i] = src[2 * i];
        }
    }
}

unsigned grid_for(const slat_ctx *ctx, uint64_t n) {
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + kB - 1) / kB, (uint64_t)ctx->cu_count * 8));
}

// a device Sat64 CSR view of m with u32 columns in `tmp` (narrowed on the device); host views are
// copied up first into `stage`
slat_status narrow_view(slat_ctx *ctx, const slat_magnus_view *m, const char *name, slat_csr_view *out, uint32_t **tmp,
                        slat_csr *stage, unsigned int *bad) {
    if (!m) return fail(ctx, SLAT_EINVAL, std::string(name) + " is null");
    if (m->n_rows && !m->row_ptr) return fail(ctx, SLAT_EINVAL, std::string(name) + ": null row_ptr");
    if (m->nnz && (!m->col_idx || !m->values)) return fail(ctx, SLAT_EINVAL, std::string(name) + ": null arrays");
    if (m->n_cols > 0xFFFFFFFFull || m->n_rows > 0xFFFFFFFFull)
        return fail(ctx, SLAT_ENOTSUP, std::string(name) + ": dims exceed the engine's u32 ids");
    const hipStream_t s = ctx->stream;
    const uint64_t *rp = m->row_ptr, *col = m->col_idx, *val = m->values;
    std::memset(stage, 0, sizeof *stage);
    if (m->residency == SLAT_HOST) {
        // one device block: row_ptr | u64 cols | values
        const size_t rp_b = (m->n_rows + 1) * 8, z = std::max<uint64_t>(m->nnz, 1) * 8;
        uint8_t *blk = nullptr;
        SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&blk, rp_b + 2 * z, s));
        stage->row_ptr = (uint64_t *)blk;
        stage->alloc = kAllocJoint;
        SLAT_HIP(ctx, hipMemcpyAsync(blk, rp, rp_b, hipMemcpyHostToDevice, s));
        if (m->nnz) {
            SLAT_HIP(ctx, hipMemcpyAsync(blk + rp_b, col, m->nnz * 8, hipMemcpyHostToDevice, s));
            SLAT_HIP(ctx, hipMemcpyAsync(blk + rp_b + z, val, m->nnz * 8, hipMemcpyHostToDevice, s));
        }
        rp = (const uint64_t *)blk;
        col = (const uint64_t *)(blk + rp_b);
        val = (const uint64_t *)(blk + rp_b + z);
    }
    SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)tmp, std::max<uint64_t>(m->nnz, 1) * 4, s));
    if (m->nnz) {
        hipLaunchKernelGGL(k_narrow_cols, dim3(grid_for(ctx, m->nnz)), dim3(kB), 0, s, col, m->nnz, m->n_cols, *tmp, bad);
        SLAT_HIP(ctx, hipGetLastError());
    }
    std::memset(out, 0, sizeof *out);
    out->n_rows = m->n_rows;
    out->n_cols = m->n_cols;
    out->nnz = m->nnz;
    out->row_ptr = rp;
    out->col_idx = *tmp;
    out->values = val;
    out->dtype = SLAT_SAT64;
    out->residency = SLAT_DEVICE;
    out->max_row_nnz = m->max_row_nnz;
    return SLAT_OK;
}

// The MagnusMatrix operations in its own layout: the inputs' u64 column ids are narrowed on the
// device (an id >= n_cols refused before anything runs), `op` runs on the u32-column Sat64 views,
// and its result's columns are widened back into *C (row_ptr and values stay in op's block).
template <typename Op>
slat_status magnus_op(slat_ctx *ctx, const slat_magnus_view *A, const slat_magnus_view *B, slat_magnus *C, Op &&op) {
    const hipStream_t s = ctx->stream;
    // the narrowing kernels' error word: a context scratch word, cleared on the stream
    unsigned int *bad = (unsigned int *)(ctx->d_words + 4);
    SLAT_HIP(ctx, hipMemsetAsync(bad, 0, 4, s));
    slat_csr_view va, vb;
    uint32_t *ta = nullptr, *tb = nullptr;
    slat_csr sa = {}, sb = {};
    auto release = [&]() {
        if (ta) slat_dev_free(ctx, ta, s);
        if (tb) slat_dev_free(ctx, tb, s);
        if (sa.row_ptr) slat_csr_free(ctx, &sa);
        if (sb.row_ptr) slat_csr_free(ctx, &sb);
    };
    slat_status st = narrow_view(ctx, A, "A", &va, &ta, &sa, bad);
    if (!st && B) st = narrow_view(ctx, B, "B", &vb, &tb, &sb, bad);
    if (st) {
        release();
        return st;
    }
    // the narrowing verdict before the operation: an id >= n_cols (or >= 2^32, which would wrap to
    // a valid-looking u32) must never reach the kernels' LDS bitmaps and composite keys
    unsigned int hbad = 0;
    SLAT_HIP(ctx, hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    if (hbad) {
        release();
        return fail(ctx, SLAT_EINVAL, "a column id is >= n_cols");
    }
    slat_csr c32 = {};
    st = op(&va, B ? &vb : nullptr, &c32);  // synchronous
    if (st) {
        release();
        return st;
    }
    if (!C) {  // no matrix result (connected components)
        release();
        if (c32.row_ptr) slat_csr_free(ctx, &c32);
        return SLAT_OK;
    }
    uint64_t *c64 = nullptr;
    if (slat_dev_alloc(ctx, (void **)&c64, std::max<uint64_t>(c32.nnz, 1) * 8, s) != hipSuccess) {
        slat_csr_free(ctx, &c32);
        release();
        return fail(ctx, SLAT_EOOM, "C column allocation failed");
    }
    if (c32.nnz) hipLaunchKernelGGL(k_widen_cols, dim3(grid_for(ctx, c32.nnz / 2 + 1)), dim3(kB), 0, s, c32.col_idx, c32.nnz, c64);
    release();
    SLAT_HIP(ctx, hipGetLastError());
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    C->n_rows = c32.n_rows;
    C->n_cols = c32.n_cols;
    C->nnz = c32.nnz;
    C->capacity = c32.nnz;
    C->max_row_nnz = c32.max_row_nnz;
    C->row_ptr = c32.row_ptr;
    C->col_idx = c64;
    C->values = (uint64_t *)c32.values;
    C->device = ctx->device;
    static_assert(sizeof(slat_csr) <= sizeof(C->_owner), "slat_magnus owner slot too small");
    std::memcpy(C->_owner, &c32, sizeof c32);
    return SLAT_OK;
}

}  // namespace

extern "C" slat_status slat_magnus_matmul(slat_ctx *ctx, const slat_magnus_view *A, const slat_magnus_view *B,
                                          slat_magnus *C, uint32_t flags) {
    if (!ctx || !C) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    std::memset(C, 0, sizeof *C);
    if (!B) return fail(ctx, SLAT_EINVAL, "B is null");
    if (A && A->n_cols != B->n_rows) return fail(ctx, SLAT_EDIM, "A.n_cols != B.n_rows");
    return magnus_op(ctx, A, B, C, [&](const slat_csr_view *a, const slat_csr_view *b, slat_csr *c) {
        return slat_spgemm_csr_sat64(ctx, a, b, c, flags);
    });
}

extern "C" slat_status slat_magnus_add(slat_ctx *ctx, const slat_magnus_view *A, const slat_magnus_view *B,
                                       slat_magnus *C) {
    if (!ctx || !C) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    std::memset(C, 0, sizeof *C);
    if (!B) return fail(ctx, SLAT_EINVAL, "B is null");
    // assert_eq!(self.n, other.n) (src/graph_magnus.rs:246)
    if (A && (A->n_rows != B->n_rows || A->n_cols != B->n_cols)) return fail(ctx, SLAT_EDIM, "A and B differ in shape");
    return magnus_op(ctx, A, B, C, [&](const slat_csr_view *a, const slat_csr_view *b, slat_csr *c) {
        return slat_csr_add(ctx, a, b, c);
    });
}

extern "C" slat_status slat_magnus_reachability_sum(slat_ctx *ctx, const slat_magnus_view *A, slat_magnus *sum,
                                                    uint64_t *k) {
    if (!ctx || !sum || !k) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    std::memset(sum, 0, sizeof *sum);
    return magnus_op(ctx, A, nullptr, sum, [&](const slat_csr_view *a, const slat_csr_view *, slat_csr *c) {
        return slat_reachability_sum(ctx, a, c, k);
    });
}

extern "C" slat_status slat_magnus_power_until_stable(slat_ctx *ctx, const slat_magnus_view *A, slat_magnus *out,
                                                      uint64_t *k) {
    if (!ctx || !out || !k) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    std::memset(out, 0, sizeof *out);
    return magnus_op(ctx, A, nullptr, out, [&](const slat_csr_view *a, const slat_csr_view *, slat_csr *c) {
        return slat_power_until_stable(ctx, a, c, k);
    });
}

extern "C" slat_status slat_magnus_connected_components(slat_ctx *ctx, const slat_magnus_view *A, uint64_t *component) {
    if (!ctx || !component) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    return magnus_op(ctx, A, nullptr, nullptr, [&](const slat_csr_view *a, const slat_csr_view *, slat_csr *) {
        return slat_connected_components(ctx, a, component);
    });
}

extern "C" slat_status slat_magnus_free(slat_ctx *ctx, slat_magnus *m) {
    if (!ctx || !m) return SLAT_EINVAL;
    (void)hipSetDevice(ctx->device);
    slat_csr c32;
    std::memcpy(&c32, m->_owner, sizeof c32);
    if (c32.row_ptr) slat_csr_free(ctx, &c32);
    if (m->col_idx) slat_dev_free(ctx, m->col_idx, ctx->stream);
    std::memset(m, 0, sizeof *m);
    return SLAT_OK;
}

extern "C" slat_status slat_magnus_to_host(slat_ctx *ctx, const slat_magnus *m, uint64_t *row_ptr, uint64_t *col_idx,
                                           uint64_t *values) {
    if (!ctx || !m) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    const hipStream_t s = ctx->stream;
    if (row_ptr && m->row_ptr)
        SLAT_HIP(ctx, hipMemcpyAsync(row_ptr, m->row_ptr, (m->n_rows + 1) * 8, hipMemcpyDeviceToHost, s));
    if (m->nnz && col_idx) SLAT_HIP(ctx, hipMemcpyAsync(col_idx, m->col_idx, m->nnz * 8, hipMemcpyDeviceToHost, s));
    if (m->nnz && values) SLAT_HIP(ctx, hipMemcpyAsync(values, m->values, m->nnz * 8, hipMemcpyDeviceToHost, s));
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    return SLAT_OK;
}

extern "C" slat_magnus_view slat_magnus_view_of(const slat_magnus *m) {
    slat_magnus_view v;
    std::memset(&v, 0, sizeof v);
    if (!m) return v;
    v.n_rows = m->n_rows;
    v.n_cols = m->n_cols;
    v.nnz = m->nnz;
    v.row_ptr = m->row_ptr;
    v.col_idx = m->col_idx;
    v.values = m->values;
    v.residency = SLAT_DEVICE;
    v.max_row_nnz = m->max_row_nnz;
    return v;
}
