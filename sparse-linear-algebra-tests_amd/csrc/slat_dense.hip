// slat_dense.hip — sparse x sparse with a dense output: the Sparse2D
// driver einsum_sparse_driven (einsum-dyn/src/sparse.rs:70-148), spec "ab,bc->ac" (or "->ca").
//
// The reference keeps a dense row accumulator `acc` and lists column j in `nz_cols` every time
// acc[j] reads T::default() before an add (sparse.rs:126-129); afterwards it writes acc[j] and
// clears it once per listing, in listing order (:137-143). A column listed once ends at its sum
// (0 + p1 + p2 + ... in visiting order); a column listed again — its running sum passed through 0
// after the first add: a u32 product that wraps to 0, an exact f64 cancellation — is written a
// second time after the clear, so it ends at 0. Untouched columns keep their content.
//
// Here one wavefront owns an output row and walks its products in the reference's order (A row
// entries ascending, then each B row; the lanes spread over one B row, whose columns are
// distinct). Per column window it keeps two LDS bitmaps: `seen` (touched before in this row) and
// `dead` (listed twice: the output is 0, later adds change nothing). A first touch stores 0 + p;
// a later touch reads the running sum from the output, marks the column dead if it is 0 (and
// stores 0), else stores sum + p. The next A entry waits for these stores (it may hit the same
// columns). T is plain u32 (the einsum tests' T, wrapping `+=` / `*` of a release build) or f64
// (`__dmul_rn` / `__dadd_rn`, no FMA: Rust never fuses).
#include <hip/hip_runtime.h>

#include <cstring>

#include "slat.h"
#include "slat_internal.hpp"

namespace {

constexpr int kB = 256, kW = 64, kWpb = kB / kW;
constexpr uint32_t kMaxWinBits = 1u << 16;  // columns per window (2 x 8 KB of bitmaps per wave)

template <typename T>
__device__ __forceinline__ T dmul(T a, T b) {
    if constexpr (sizeof(T) == 8) return __dmul_rn(a, b); else return a * b;
}
template <typename T>
__device__ __forceinline__ T dadd(T a, T b) {
    if constexpr (sizeof(T) == 8) return __dadd_rn(a, b); else return a + b;
}

template <typename T>
__global__ __launch_bounds__(kB) void k_dense_out(const uint64_t *arp, const uint32_t *acol, const T *aval,
                                                  const uint64_t *brp, const uint32_t *bcol, const T *bval,
                                                  uint64_t nrows, uint64_t bn, uint64_t ncols, uint32_t win,
                                                  T *out, uint64_t ld, int trans) {
    extern __shared__ uint32_t sm[];
    const int lane = threadIdx.x & (kW - 1);
    const uint32_t words = win / 32;
    uint32_t *seen = sm + (threadIdx.x / kW) * 2 * words, *dead = seen + words;
    for (uint32_t w = lane; w < 2 * words; w += kW) seen[w] = 0;
    __builtin_amdgcn_wave_barrier();
    const uint64_t waves = (uint64_t)gridDim.x * kWpb;
    for (uint64_t i = (uint64_t)blockIdx.x * kWpb + threadIdx.x / kW; i < nrows; i += waves) {
        const uint64_t a0 = arp[i], a1 = arp[i + 1];
        auto at = [&](uint32_t j) -> T * { return trans ? out + (uint64_t)j * ld + i : out + i * ld + j; };
        for (uint64_t wlo = 0; wlo < ncols; wlo += win) {
            for (uint64_t e = a0; e < a1; ++e) {
                const uint32_t k = acol[e];
                if (k >= bn) continue;  // malformed input: no such B row
                const T a = aval[e];
                for (uint64_t t = brp[k] + lane; t < brp[k + 1]; t += kW) {
                    const uint32_t j = bcol[t];
                    const uint64_t off = (uint64_t)j - wlo;
                    if (off >= win) continue;
                    const uint32_t w = (uint32_t)off >> 5, bit = 1u << (off & 31);
                    const T p = dmul(a, bval[t]);
                    T *q = at(j);
                    if (!(seen[w] & bit)) {
                        __hip_atomic_store(q, dadd(T(0), p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        atomicOr(&seen[w], bit);
                    } else if (!(dead[w] & bit)) {
                        const T v = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (v == T(0)) {  // listed again: the second write (of 0) wins
                            __hip_atomic_store(q, T(0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            atomicOr(&dead[w], bit);
                        } else {
                            __hip_atomic_store(q, dadd(v, p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                }
                __builtin_amdgcn_s_waitcnt(0);  // the next entry may hit these columns (stores and bits)
                __builtin_amdgcn_wave_barrier();
            }
            // clear the bits this row set (the same walk)
            for (uint64_t e = a0; e < a1; ++e) {
                const uint32_t k = acol[e];
                if (k >= bn) continue;
                for (uint64_t t = brp[k] + lane; t < brp[k + 1]; t += kW) {
                    const uint64_t off = (uint64_t)bcol[t] - wlo;
                    if (off < win) {
                        seen[off >> 5] = 0;
                        dead[off >> 5] = 0;
                    }
                }
            }
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
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
    if (A->n_rows && B->n_cols) {
        // window: all columns when they fit kMaxWinBits, rounded to whole 64-word blocks
        const uint64_t cols = std::min<uint64_t>(B->n_cols, kMaxWinBits);
        const uint32_t win = (uint32_t)((cols + 2047) / 2048 * 2048);
        const size_t lds = (size_t)kWpb * 2 * (win / 32) * 4;
        const unsigned g = (unsigned)std::min<uint64_t>((A->n_rows + kWpb - 1) / kWpb, (uint64_t)ctx->cu_count * 8);
        if (A->dtype == SLAT_F64)
            hipLaunchKernelGGL((k_dense_out<double>), dim3(g), dim3(kB), lds, s, A->row_ptr, A->col_idx,
                               (const double *)A->values, B->row_ptr, B->col_idx, (const double *)B->values, A->n_rows,
                               B->n_rows, B->n_cols, win, (double *)dout, ld, transpose);
        else
            hipLaunchKernelGGL((k_dense_out<uint32_t>), dim3(g), dim3(kB), lds, s, A->row_ptr, A->col_idx,
                               (const uint32_t *)A->values, B->row_ptr, B->col_idx, (const uint32_t *)B->values,
                               A->n_rows, B->n_rows, B->n_cols, win, (uint32_t *)dout, ld, transpose);
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
