// slat_graph.hip — C ABI of the reference's SpGEMM consumers, all
// device-resident: CsrMatrix::add / identity and the iterated drivers reachability_sum,
// power_until_stable and connected_components (src/graph_csr.rs:68-80, 487-603; the MagnusMatrix
// twins at src/graph_magnus.rs:245-360 on Sat64). Every product goes through slat_spgemm, every
// sum through k_add; only the loop decisions (nnz, pattern equality) come back to the host.
#include <hip/hip_runtime.h>

#include <cstring>

#include "graph_kernels.hpp"
#include "slat.h"
#include "slat_internal.hpp"

using namespace slat;

namespace {

dim3 wave_grid(const slat_ctx *ctx, uint64_t rows) {
    const uint64_t blocks = (rows + kBlock / kWave - 1) / (kBlock / kWave);
    return dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)ctx->cu_count * 16)));
}
dim3 flat_grid(const slat_ctx *ctx, uint64_t items) {
    const uint64_t blocks = (items + kBlock - 1) / kBlock;
    return dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)ctx->cu_count * 8)));
}

// a device-resident copy of a host view (owned in *tmp), or the view itself
slat_status on_device(slat_ctx *ctx, const slat_csr_view *v, slat_csr *tmp, slat_csr_view *dv,
                      const slat_csr_view **out) {
    if (v->residency == SLAT_DEVICE) {
        *out = v;
        return SLAT_OK;
    }
    slat_status st = slat_csr_create(ctx, v, tmp);
    if (st) return st;
    *dv = slat_csr_view_of(tmp);
    *out = dv;
    return SLAT_OK;
}

template <typename S>
slat_status add_typed(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B, slat_csr *C) {
    hipStream_t s = ctx->stream;
    const uint64_t n = A->n_rows;
    slat_status st = slat_ensure_ws(ctx, std::max<uint64_t>(n, 1) * 8);
    if (st) return st;
    uint64_t *counts = (uint64_t *)ctx->ws;
    SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&C->row_ptr, (n + 1) * 8, s));
    C->alloc = kAllocSeparate;
    const dim3 g = wave_grid(ctx, n);
    hipLaunchKernelGGL((k_add<S, true>), g, dim3(kBlock), 0, s, A->row_ptr, A->col_idx, (const S *)A->values,
                       B->row_ptr, B->col_idx, (const S *)B->values, n, counts, nullptr, nullptr, nullptr);
    SLAT_HIP(ctx, hipGetLastError());
    ctx->h_out[0] = ctx->h_out[1] = 0;
    if ((st = slat_launch_scan(ctx, counts, n, C->row_ptr, s))) return st;
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    const uint64_t nnz = ctx->h_out[0];
    C->nnz = nnz;
    C->capacity = std::max<uint64_t>(nnz, 1);
    C->max_row_nnz = ctx->h_out[1];
    SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&C->col_idx, C->capacity * 4, s));
    SLAT_HIP(ctx, slat_dev_alloc(ctx, &C->values, C->capacity * sizeof(S), s));
    hipLaunchKernelGGL((k_add<S, false>), g, dim3(kBlock), 0, s, A->row_ptr, A->col_idx, (const S *)A->values,
                       B->row_ptr, B->col_idx, (const S *)B->values, n, nullptr, C->row_ptr, C->col_idx,
                       (S *)C->values);
    SLAT_HIP(ctx, hipGetLastError());
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    return SLAT_OK;
}

slat_status square_check(slat_ctx *ctx, const slat_csr_view *A) {
    slat_status st = slat_check_view(ctx, A, "A");
    if (st) return st;
    if (A->n_rows != A->n_cols) return fail(ctx, SLAT_EDIM, "matrix is not square");
    return SLAT_OK;
}

}  // namespace

extern "C" slat_status slat_csr_add(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B, slat_csr *C) {
    if (!ctx || !C) return SLAT_EINVAL;
    slat_status st;
    if ((st = slat_check_view(ctx, A, "A")) || (st = slat_check_view(ctx, B, "B"))) return st;
    if (A->dtype != B->dtype) return fail(ctx, SLAT_EINVAL, "A and B value types differ");
    if (A->n_rows != B->n_rows || A->n_cols != B->n_cols)
        return fail(ctx, SLAT_EDIM, "A and B shapes differ");  // assert_eq!(self.n, other.n)
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    slat_csr ta = {}, tb = {};
    slat_csr_view va, vb;
    const slat_csr_view *pa, *pb;
    if ((st = on_device(ctx, A, &ta, &va, &pa))) return st;
    if ((st = on_device(ctx, B, &tb, &vb, &pb))) {
        slat_csr_free(ctx, &ta);
        return st;
    }
    std::memset(C, 0, sizeof *C);
    C->n_rows = A->n_rows;
    C->n_cols = A->n_cols;
    C->dtype = A->dtype;
    C->device = ctx->device;
    if (A->dtype == SLAT_U32)
        st = add_typed<uint32_t>(ctx, pa, pb, C);
    else if (A->dtype == SLAT_SAT64)
        st = add_typed<unsigned long long>(ctx, pa, pb, C);
    else
        st = add_typed<double>(ctx, pa, pb, C);
    if (st) slat_csr_free(ctx, C);
    if (ta.row_ptr) slat_csr_free(ctx, &ta);
    if (tb.row_ptr) slat_csr_free(ctx, &tb);
    return st;
}

extern "C" slat_status slat_csr_identity(slat_ctx *ctx, uint64_t n, int32_t dtype, slat_csr *out) {
    if (!ctx || !out || dtype < SLAT_U32 || dtype > SLAT_F64) return SLAT_EINVAL;
    if (n > 0xFFFFFFFFull) return fail(ctx, SLAT_EINVAL, "n exceeds u32 ids");
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    std::memset(out, 0, sizeof *out);
    hipStream_t s = ctx->stream;
    SLAT_HIP(ctx, alloc_joint(ctx, out, n, n, vsize(dtype), s));
    const dim3 g = flat_grid(ctx, n + 1);
    if (dtype == SLAT_U32)
        hipLaunchKernelGGL(k_identity<uint32_t>, g, dim3(kBlock), 0, s, n, out->row_ptr, out->col_idx, (uint32_t *)out->values);
    else if (dtype == SLAT_SAT64)
        hipLaunchKernelGGL(k_identity<unsigned long long>, g, dim3(kBlock), 0, s, n, out->row_ptr, out->col_idx,
                           (unsigned long long *)out->values);
    else
        hipLaunchKernelGGL(k_identity<double>, g, dim3(kBlock), 0, s, n, out->row_ptr, out->col_idx, (double *)out->values);
    SLAT_HIP(ctx, hipGetLastError());
    out->n_rows = out->n_cols = out->nnz = n;
    out->capacity = std::max<uint64_t>(n, 1);
    out->max_row_nnz = n ? 1 : 0;
    out->dtype = dtype;
    out->device = ctx->device;
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    return SLAT_OK;
}

extern "C" slat_status slat_csr_pattern_equal(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B,
                                              int32_t *equal) {
    if (!ctx || !equal) return SLAT_EINVAL;
    slat_status st;
    if ((st = slat_check_view(ctx, A, "A")) || (st = slat_check_view(ctx, B, "B"))) return st;
    if (A->residency != SLAT_DEVICE || B->residency != SLAT_DEVICE)
        return fail(ctx, SLAT_EINVAL, "pattern_equal takes device-resident views");
    *equal = 0;
    if (A->n_rows != B->n_rows || A->nnz != B->nnz) return SLAT_OK;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    ctx->h_out[3] = 0;
    hipLaunchKernelGGL(k_diff<uint64_t>, flat_grid(ctx, A->n_rows + 1), dim3(kBlock), 0, s, A->row_ptr, B->row_ptr,
                       A->n_rows + 1, ctx->h_out_dev + 3);
    SLAT_HIP(ctx, hipGetLastError());
    if (A->nnz) {
        hipLaunchKernelGGL(k_diff<uint32_t>, flat_grid(ctx, A->nnz), dim3(kBlock), 0, s, A->col_idx, B->col_idx, A->nnz,
                           ctx->h_out_dev + 3);
        SLAT_HIP(ctx, hipGetLastError());
    }
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    *equal = ctx->h_out[3] == 0 ? 1 : 0;
    return SLAT_OK;
}

extern "C" slat_status slat_power_until_stable(slat_ctx *ctx, const slat_csr_view *A, slat_csr *out, uint64_t *k) {
    if (!ctx || !out || !k) return SLAT_EINVAL;
    slat_status st = square_check(ctx, A);
    if (st) return st;
    std::memset(out, 0, sizeof *out);
    slat_csr cur = {};
    if ((st = slat_csr_create(ctx, A, &cur))) return st;  // current = self.clone()
    *k = 0;
    for (;;) {
        slat_csr next = {};
        slat_csr_view vc = slat_csr_view_of(&cur);
        if ((st = slat_spgemm(ctx, &vc, &vc, &next, 0))) break;
        *k += 1;
        slat_csr_view vn = slat_csr_view_of(&next);
        int32_t eq = 0;
        if ((st = slat_csr_pattern_equal(ctx, &vn, &vc, &eq))) {
            slat_csr_free(ctx, &next);
            break;
        }
        slat_csr_free(ctx, &cur);
        cur = next;
        if (eq) {
            *out = cur;
            return SLAT_OK;
        }
    }
    slat_csr_free(ctx, &cur);
    return st;
}

extern "C" slat_status slat_reachability_sum(slat_ctx *ctx, const slat_csr_view *A, slat_csr *out, uint64_t *k) {
    if (!ctx || !out || !k) return SLAT_EINVAL;
    slat_status st = square_check(ctx, A);
    if (st) return st;
    std::memset(out, 0, sizeof *out);
    slat_csr base = {}, power = {}, sum = {};
    if ((st = slat_csr_create(ctx, A, &base)) || (st = slat_csr_create(ctx, A, &power)) ||
        (st = slat_csr_create(ctx, A, &sum))) {
        for (slat_csr *m : {&base, &power, &sum})
            if (m->row_ptr) slat_csr_free(ctx, m);
        return st;
    }
    slat_csr_view vb = slat_csr_view_of(&base);
    *k = 1;
    for (;;) {
        slat_csr np = {}, ns = {};
        slat_csr_view vp = slat_csr_view_of(&power);
        if ((st = slat_spgemm(ctx, &vp, &vb, &np, 0))) break;  // power = power.matmul(self)
        slat_csr_free(ctx, &power);
        power = np;
        *k += 1;
        slat_csr_view vs = slat_csr_view_of(&sum), vp2 = slat_csr_view_of(&power);
        if ((st = slat_csr_add(ctx, &vs, &vp2, &ns))) break;  // new_sum = sum.add(&power)
        const bool done = ns.nnz == sum.nnz;
        slat_csr_free(ctx, &sum);
        sum = ns;
        if (done) break;
    }
    slat_csr_free(ctx, &base);
    slat_csr_free(ctx, &power);
    if (st) {
        slat_csr_free(ctx, &sum);
        return st;
    }
    *out = sum;
    return SLAT_OK;
}

extern "C" slat_status slat_connected_components(slat_ctx *ctx, const slat_csr_view *A, uint64_t *component) {
    if (!ctx) return SLAT_EINVAL;
    slat_status st = square_check(ctx, A);
    if (st) return st;
    const uint64_t n = A->n_rows;
    if (n == 0) return SLAT_OK;
    if (!component) return SLAT_EINVAL;
    slat_csr id = {}, with_id = {}, closure = {};
    uint64_t k = 0;
    if ((st = slat_csr_identity(ctx, n, A->dtype, &id))) return st;
    slat_csr_view vid = slat_csr_view_of(&id);
    st = slat_csr_add(ctx, A, &vid, &with_id);  // self.add(&Self::identity(self.n))
    slat_csr_free(ctx, &id);
    if (st) return st;
    slat_csr_view vw = slat_csr_view_of(&with_id);
    st = slat_power_until_stable(ctx, &vw, &closure, &k);
    slat_csr_free(ctx, &with_id);
    if (st) return st;
    // workspace: low u32[n] | root u64[n] | ids u64[n+1] | comp u64[n]
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_root = up(n * 4), o_ids = o_root + up(n * 8), o_comp = o_ids + up((n + 1) * 8);
    if ((st = slat_ensure_ws(ctx, o_comp + n * 8))) {
        slat_csr_free(ctx, &closure);
        return st;
    }
    uint8_t *ws = (uint8_t *)ctx->ws;
    uint32_t *low = (uint32_t *)ws;
    uint64_t *root = (uint64_t *)(ws + o_root), *ids = (uint64_t *)(ws + o_ids), *comp = (uint64_t *)(ws + o_comp);
    hipStream_t s = ctx->stream;
    hipLaunchKernelGGL(k_cc_low, wave_grid(ctx, n), dim3(kBlock), 0, s, closure.row_ptr, closure.col_idx, n, low, root);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && !(st = slat_launch_scan(ctx, root, n, ids, s))) {
        hipLaunchKernelGGL(k_cc_label, flat_grid(ctx, n), dim3(kBlock), 0, s, low, ids, n, comp);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(component, comp, n * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
    }
    slat_csr_free(ctx, &closure);
    if (st) return st;
    if (e != hipSuccess) return fail(ctx, SLAT_EHIP, std::string("connected_components: ") + hipGetErrorString(e));
    return SLAT_OK;
}

// bench_diameter's algorithm (src/graph_csr.rs:1228-1319) as a device-resident driver: R0 = A + I of
// the undirected graph (R[i][j] > 0 iff dist(i, j) <= 1); phase 1 squares until the pattern stops
// changing (reach doubles each time), phase 2 multiplies the last power before stabilisation by R0
// until its pattern stops changing. Loop decisions (pattern equality) are the only host round trips.
extern "C" slat_status slat_diameter(slat_ctx *ctx, const slat_csr_view *A, uint64_t *diameter, uint64_t *squarings,
                                     uint64_t *refinements) {
    if (!ctx || !diameter) return SLAT_EINVAL;
    slat_status st = square_check(ctx, A);
    if (st) return st;
    slat_csr id = {}, r0 = {};
    if ((st = slat_csr_identity(ctx, A->n_rows, A->dtype, &id))) return st;
    slat_csr_view vi = slat_csr_view_of(&id);
    st = slat_csr_add(ctx, A, &vi, &r0);
    slat_csr_free(ctx, &id);
    if (st) return st;
    slat_csr_view vr0 = slat_csr_view_of(&r0);
    uint64_t sq = 0, rf = 0, prev_reach = 0, reach = 1;
    slat_csr current = {}, prev_saved = {};
    if ((st = slat_csr_create(ctx, &vr0, &current))) {
        slat_csr_free(ctx, &r0);
        return st;
    }
    auto cleanup = [&]() {
        if (current.row_ptr) slat_csr_free(ctx, &current);
        if (prev_saved.row_ptr) slat_csr_free(ctx, &prev_saved);
        slat_csr_free(ctx, &r0);
    };
    for (;;) {  // phase 1: repeated squaring
        slat_csr next = {};
        slat_csr_view vc = slat_csr_view_of(&current);
        if ((st = slat_spgemm(ctx, &vc, &vc, &next, 0))) break;
        ++sq;
        slat_csr_view vn = slat_csr_view_of(&next);
        int32_t eq = 0;
        if ((st = slat_csr_pattern_equal(ctx, &vn, &vc, &eq))) {
            slat_csr_free(ctx, &next);
            break;
        }
        if (eq) {  // stabilised: diameter in (prev_reach, 2 * reach]
            slat_csr_free(ctx, &next);
            break;
        }
        if (prev_saved.row_ptr) slat_csr_free(ctx, &prev_saved);
        prev_saved = current;
        prev_reach = reach;
        current = next;
        reach *= 2;
    }
    if (st) {
        cleanup();
        return st;
    }
    uint64_t d = 1;  // stabilised on the first squaring: R0 is its own closure (diameter <= 1)
    if (prev_reach != 0) {  // phase 2: linear refinement from the power covering <= prev_reach
        slat_csr refine = prev_saved;
        prev_saved = {};
        d = prev_reach;
        for (;;) {
            slat_csr next = {};
            slat_csr_view vf = slat_csr_view_of(&refine);
            if ((st = slat_spgemm(ctx, &vf, &vr0, &next, 0))) break;
            ++rf;
            ++d;
            slat_csr_view vn = slat_csr_view_of(&next);
            int32_t eq = 0;
            st = slat_csr_pattern_equal(ctx, &vn, &vf, &eq);
            slat_csr_free(ctx, &refine);
            refine = next;
            if (st) break;
            if (eq) {
                d -= 1;
                break;
            }
        }
        slat_csr_free(ctx, &refine);
    }
    cleanup();
    if (st) return st;
    *diameter = d;
    if (squarings) *squarings = sq;
    if (refinements) *refinements = rf;
    return SLAT_OK;
}
