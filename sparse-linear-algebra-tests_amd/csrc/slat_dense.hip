// slat_dense.hip — sparse x sparse with a dense output: the Sparse2D
// driver einsum_sparse_driven (einsum-dyn/src/sparse.rs:70-148), spec "ab,bc->ac" (or "->ca").
// The reference keeps a dense row accumulator and writes every touched column of the output row,
// leaving untouched entries as they were. Here one wavefront owns an output row: pass 1 stores 0
// at every touched column, pass 2 adds the products in place. Integer T (plain u32: the einsum
// tests' T, wrapping `+=` / `*` of a release build) adds with atomics, since wrapping sums are
// order-free. f64 keeps the reference's left fold: the A entries of the row in order, each a
// read-modify-write of distinct columns (one B row), the next step issued after the stores land.
#include <hip/hip_runtime.h>

#include <cstring>

#include "slat.h"
#include "slat_internal.hpp"

namespace {

constexpr int kB = 256, kW = 64;

template <typename T, bool ORDERED>
__global__ __launch_bounds__(kB) void k_dense_out(const uint64_t *arp, const uint32_t *acol, const T *aval,
                                                  const uint64_t *brp, const uint32_t *bcol, const T *bval,
                                                  uint64_t nrows, uint64_t bn, T *out, uint64_t ld, int trans) {
    const int lane = threadIdx.x & (kW - 1);
    const uint64_t waves = (uint64_t)gridDim.x * (kB / kW);
    for (uint64_t i = (uint64_t)blockIdx.x * (kB / kW) + threadIdx.x / kW; i < nrows; i += waves) {
        const uint64_t a0 = arp[i], a1 = arp[i + 1];
        auto at = [&](uint32_t j) -> T * { return trans ? out + (uint64_t)j * ld + i : out + i * ld + j; };
        // pass 1: the touched columns start from T::default()
        for (uint64_t e = a0; e < a1; ++e) {
            const uint32_t k = acol[e];
            if (k >= bn) continue;  // malformed input: no such B row
            for (uint64_t t = brp[k] + lane; t < brp[k + 1]; t += kW) *at(bcol[t]) = T(0);
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        // pass 2: acc[j] += a * b in A-row order, then B-row order
        for (uint64_t e = a0; e < a1; ++e) {
            const uint32_t k = acol[e];
            if (k >= bn) continue;
            const T a = aval[e];
            for (uint64_t t = brp[k] + lane; t < brp[k + 1]; t += kW) {
                T *p = at(bcol[t]);
                if constexpr (ORDERED) {
                    const T v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(p, __dadd_rn(v, __dmul_rn(a, bval[t])), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    atomicAdd(p, (T)(a * bval[t]));
                }
            }
            if constexpr (ORDERED) __builtin_amdgcn_s_waitcnt(0);  // the next entry may hit these columns
        }
    }
}

}  // namespace

extern "C" slat_status slat_spgemm_dense(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B, void *out,
                                         uint64_t ld, int32_t transpose, int32_t out_residency) {
    if (!ctx || (!out && A && A->n_rows && B && B->n_cols)) return SLAT_EINVAL;
    slat_status st;
    if ((st = slat_check_view(ctx, A, "A")) || (st = slat_check_view(ctx, B, "B"))) return st;
    if (A->dtype != B->dtype) return fail(ctx, SLAT_EINVAL, "A and B value types differ");
    if (A->dtype == SLAT_SAT64) return fail(ctx, SLAT_ENOTSUP, "dense output: u32 (wrapping) or f64 values");
    if (A->n_cols != B->n_rows) return fail(ctx, SLAT_EDIM, "A.n_cols != B.n_rows");
    if (A->residency != SLAT_DEVICE || B->residency != SLAT_DEVICE)
        return fail(ctx, SLAT_EINVAL, "dense output takes device-resident A and B");
    const uint64_t orows = transpose ? B->n_cols : A->n_rows, ocols = transpose ? A->n_rows : B->n_cols;
    if (ld < ocols) return fail(ctx, SLAT_EINVAL, "ld smaller than the output row length");
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t vs = vsize(A->dtype), bytes = orows * ld * vs;
    void *dout = out;
    if (out_residency != SLAT_DEVICE && bytes) {
        SLAT_HIP(ctx, slat_dev_alloc(ctx, &dout, bytes, s));
        SLAT_HIP(ctx, hipMemcpyAsync(dout, out, bytes, hipMemcpyHostToDevice, s));
    }
    if (A->n_rows) {
        const unsigned g = (unsigned)std::min<uint64_t>((A->n_rows + kB / kW - 1) / (kB / kW), (uint64_t)ctx->cu_count * 32);
        if (A->dtype == SLAT_F64)
            hipLaunchKernelGGL((k_dense_out<double, true>), dim3(g), dim3(kB), 0, s, A->row_ptr, A->col_idx,
                               (const double *)A->values, B->row_ptr, B->col_idx, (const double *)B->values, A->n_rows,
                               B->n_rows, (double *)dout, ld, transpose);
        else
            hipLaunchKernelGGL((k_dense_out<uint32_t, false>), dim3(g), dim3(kB), 0, s, A->row_ptr, A->col_idx,
                               (const uint32_t *)A->values, B->row_ptr, B->col_idx, (const uint32_t *)B->values,
                               A->n_rows, B->n_rows, (uint32_t *)dout, ld, transpose);
        if (hipGetLastError() != hipSuccess) {
            if (dout != out) slat_dev_free(ctx, dout, s);
            return fail(ctx, SLAT_EHIP, "dense output launch failed");
        }
    }
    if (dout != out) {
        SLAT_HIP(ctx, hipMemcpyAsync(out, dout, bytes, hipMemcpyDeviceToHost, s));
        slat_dev_free(ctx, dout, s);
    }
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    return SLAT_OK;
}

// device buffers for dense operands (from the context's block cache) and their host copies
extern "C" slat_status slat_device_alloc(slat_ctx *ctx, uint64_t bytes, void **p) {
    if (!ctx || !p) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    if (slat_dev_alloc(ctx, p, bytes, ctx->stream) != hipSuccess) return fail(ctx, SLAT_EOOM, "device buffer");
    return SLAT_OK;
}
extern "C" slat_status slat_device_free(slat_ctx *ctx, void *p) {
    if (!ctx) return SLAT_EINVAL;
    if (p) slat_dev_free(ctx, p, ctx->stream);
    return SLAT_OK;
}
extern "C" slat_status slat_device_copy(slat_ctx *ctx, void *dst, const void *src, uint64_t bytes, int32_t to_host) {
    if (!ctx || (bytes && (!dst || !src))) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    if (bytes)
        SLAT_HIP(ctx, hipMemcpyAsync(dst, src, bytes, to_host ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice,
                                     ctx->stream));
    SLAT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return SLAT_OK;
}
