// slat_api.hip — C ABI (include/slat.h) over the gfx950 SpGEMM kernels.
//
// Orchestration of one C = A·B call on the context's stream:
//   1. C.row_ptr, C.col and C.val in pieces of the context's device memory (slat_dev_alloc). By
//      default col/val are sized by the exact upper bound nnz(A)·max_row_nnz(B) (clamped to
//      rows·cols), so no host round trip is needed between the symbolic and numeric passes; at the
//      end both are trimmed to nnz(C) and the tails return to the context's cache.
//      SLAT_FLAG_EXACT_ALLOC (or a bound above 4 GiB / the budget) takes the reference's
//      exact-size path instead: sync after the scan, allocate nnz(C).
//   2. k_symbolic -> k_scan_rows (single-pass look-back scan) -> k_numeric, all stream-ordered.
//   3. One D2H of the 64 status shards (nnz, max row nnz, dropped-zero rows) + stream sync.
//   4. Rare: k_compact when explicit zeros were dropped.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "slat.h"
#include "slat_internal.hpp"
#include "spgemm_kernels.hpp"
#include "slat_launch.hpp"
#include "slat_fat.hpp"  // the fat-row category (a workgroup and a dense LDS accumulator per row)

using namespace slat;

// max(B) for the CSR walk too (SLAT_NO_NARROW_CSR=1: the u64 slots of before, for A/B runs)
static const bool kNarrowCsr = slat_ab_knob("SLAT_NO_NARROW_CSR") == nullptr;
static void dev_release_all(slat_ctx *ctx);

extern "C" {

const char *slat_status_string(slat_status s) {
    switch (s) {
    case SLAT_OK: return "ok";
    case SLAT_EINVAL: return "invalid argument";
    case SLAT_EDIM: return "dimension mismatch";
    case SLAT_EOOM: return "out of memory";
    case SLAT_EHIP: return "HIP error";
    case SLAT_ENOTSUP: return "not supported";
    case SLAT_ENODEV: return "no gfx950 device";
    }
    return "unknown";
}

const char *slat_last_error(slat_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

slat_status slat_ctx_create(int device, slat_ctx **out) {
    if (!out) return SLAT_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return SLAT_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return SLAT_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SLAT_ENODEV;
    if (const char *e_ = slat_ab_knob("SLAT_SPIN"))  // experiment: spin-wait stream syncs
        if (std::atoi(e_)) {
            (void)hipSetDevice(device);
            (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
        }
    slat_ctx *ctx = new slat_ctx();
    ctx->device = device;
    ctx->cu_count = prop.multiProcessorCount;
    ctx->lds_per_block_max = prop.sharedMemPerBlock;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return SLAT_EHIP;
    }
    ctx->stream = ctx->own_stream;
    if (hipHostMalloc((void **)&ctx->h_shards, sizeof(unsigned long long) * kShards * kShardStride) != hipSuccess) {
        (void)hipStreamDestroy(ctx->own_stream);
        delete ctx;
        return SLAT_EOOM;
    }
    if (hipMalloc((void **)&ctx->d_words, 128) != hipSuccess || hipMemset(ctx->d_words, 0, 128) != hipSuccess ||
        hipMalloc((void **)&ctx->d_done, kDoneBytes + kMaxwBytes) != hipSuccess ||
        hipMemset(ctx->d_done, 0, kDoneBytes + kMaxwBytes) != hipSuccess ||
        hipHostMalloc((void **)&ctx->h_out, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void **)&ctx->h_out_dev, ctx->h_out, 0) != hipSuccess) {
        (void)hipHostFree(ctx->h_shards);
        (void)hipStreamDestroy(ctx->own_stream);
        delete ctx;
        return SLAT_EOOM;
    }
    std::memset(ctx->h_out, 0, 64);  // [7] must not match the first call's sequence number
    ctx->d_vmax = ctx->d_words;
    ctx->d_maxw = ctx->d_done + kDoneBytes / 8;  // (the one-kernel paths' max row words)
    for (auto &e : ctx->ev) (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);  // timing only
    *out = ctx;
    return SLAT_OK;
}

slat_status slat_ctx_destroy(slat_ctx *ctx) {
    if (!ctx) return SLAT_EINVAL;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->ws) (void)hipFree(ctx->ws);
    slat_hostio_destroy(ctx);
    dev_release_all(ctx);
    if (ctx->h_shards) (void)hipHostFree(ctx->h_shards);
    if (ctx->d_words) (void)hipFree(ctx->d_words);
    if (ctx->d_done) (void)hipFree(ctx->d_done);
    if (ctx->h_out) (void)hipHostFree(ctx->h_out);
    for (auto &e : ctx->ev) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return SLAT_OK;
}

slat_status slat_ctx_set_stream(slat_ctx *ctx, void *s) {
    if (!ctx) return SLAT_EINVAL;
    ctx->stream = s ? (hipStream_t)s : ctx->own_stream;
    return SLAT_OK;
}

void *slat_ctx_stream(slat_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

slat_status slat_sync(slat_ctx *ctx) {
    if (!ctx) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return SLAT_OK;
}

static std::atomic<int> g_progress{std::getenv("SLAT_MATMUL_PROGRESS") ? 1 : 0};

extern "C" int slat_set_matmul_progress(int on) { return g_progress.exchange(on ? 1 : 0, std::memory_order_relaxed); }

slat_status slat_get_stats(slat_ctx *ctx, slat_stats *out) {
    if (!ctx || !out) return SLAT_EINVAL;
    *out = ctx->stats;
    return SLAT_OK;
}

slat_csr_view slat_csr_view_of(const slat_csr *m) {
    slat_csr_view v;
    std::memset(&v, 0, sizeof v);
    if (!m) return v;
    v.n_rows = m->n_rows;
    v.n_cols = m->n_cols;
    v.nnz = m->nnz;
    v.row_ptr = m->row_ptr;
    v.col_idx = m->col_idx;
    v.values = m->values;
    v.dtype = m->dtype;
    v.residency = SLAT_DEVICE;
    v.max_row_nnz = m->max_row_nnz;
    return v;
}

slat_status slat_host_alloc(uint64_t bytes, void **p) {
    if (!p) return SLAT_EINVAL;
    *p = nullptr;
    return hipHostMalloc(p, std::max<uint64_t>(bytes, 1), hipHostMallocDefault) == hipSuccess ? SLAT_OK : SLAT_EOOM;
}

slat_status slat_host_free(void *p) {
    if (!p) return SLAT_OK;
    return hipHostFree(p) == hipSuccess ? SLAT_OK : SLAT_EINVAL;
}

slat_status slat_csr_free(slat_ctx *ctx, slat_csr *m) {
    if (!ctx || !m) return SLAT_EINVAL;
    (void)hipSetDevice(ctx->device);
    if (m->alloc == kAllocJoint) {
        if (m->row_ptr) slat_dev_free(ctx, m->row_ptr, ctx->stream);
    } else {
        if (m->row_ptr) slat_dev_free(ctx, m->row_ptr, ctx->stream);
        if (m->col_idx) slat_dev_free(ctx, m->col_idx, ctx->stream);
        if (m->values) slat_dev_free(ctx, m->values, ctx->stream);
    }
    std::memset(m, 0, sizeof *m);
    return SLAT_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Device memory (slat_internal.hpp): hipMalloc'd chunks carved into pieces. Sizes round to 4 KiB (to
// 2 MiB above 1 MiB) so repeated calls of similar size find their piece; a request takes the best-fit
// free piece and splits off a remainder of 1 MiB or more; freed pieces merge with their free
// neighbours; slat_dev_shrink hands the tail of a live piece back (C trimmed to nnz(C)).
// Measured reason for not using hipMallocAsync (ROCm 7.2 image): after a thin call freed pool
// blocks, a 324 MB lattice allocation read back zeros for a 26 MiB range of k_lattice's row writes
// (the column writes of the same threads, in another range, were intact); with the default release
// threshold a later scan spun forever on status words it had written. hipMalloc: correct.
static size_t round_block(size_t b) {
    const size_t g = b > ((size_t)1 << 20) ? ((size_t)2 << 20) : 4096;
    return (std::max<size_t>(b, 1) + g - 1) / g * g;
}
static constexpr size_t kCacheMax = (size_t)32 << 30;  // cached bytes kept at most (of 288 GB)
static constexpr size_t kSplitMin = (size_t)1 << 20;   // smallest remainder kept as a piece of its own

// a free piece into the cache, merged with the free neighbours of its chunk on the same stream
static void cache_put(slat_ctx *ctx, slat_ctx::Block b) {
    ctx->cache_bytes += b.bytes;
    for (size_t i = 0; i < ctx->cache.size();) {
        const auto &c = ctx->cache[i];
        if (c.chunk == b.chunk && c.s == b.s &&
            ((uint8_t *)c.p + c.bytes == (uint8_t *)b.p || (uint8_t *)b.p + b.bytes == (uint8_t *)c.p)) {
            if (c.p < b.p) b.p = c.p;
            b.bytes += c.bytes;
            ctx->cache.erase(ctx->cache.begin() + (std::ptrdiff_t)i);
            i = 0;  // the grown piece may now touch another
            continue;
        }
        ++i;
    }
    ctx->cache.push_back(b);
}

static bool whole_chunk(const slat_ctx *ctx, const slat_ctx::Block &b) {
    auto it = ctx->chunks.find(b.p);
    return b.p == b.chunk && it != ctx->chunks.end() && it->second == b.bytes;
}

hipError_t slat_dev_alloc(slat_ctx *ctx, void **p, size_t bytes, hipStream_t s) {
    const size_t r = round_block(bytes);
    // best fit on this stream: an exact-ish piece, or a larger one split (remainder >= kSplitMin)
    size_t best = SIZE_MAX;
    for (size_t i = 0; i < ctx->cache.size(); ++i) {
        const auto &c = ctx->cache[i];
        if (c.s != s || c.bytes < r) continue;
        if (c.bytes / 4 > r && c.bytes - r < kSplitMin) continue;
        if (best == SIZE_MAX || c.bytes < ctx->cache[best].bytes) best = i;
    }
    if (best != SIZE_MAX) {
        slat_ctx::Block c = ctx->cache[best];
        ctx->cache.erase(ctx->cache.begin() + (std::ptrdiff_t)best);
        ctx->cache_bytes -= c.bytes;
        if (c.bytes - r >= kSplitMin) {
            ctx->cache_bytes += c.bytes - r;
            ctx->cache.push_back({(uint8_t *)c.p + r, c.bytes - r, s, c.chunk});
            c.bytes = r;
        }
        *p = c.p;
        ctx->live[c.p] = c;
        return hipSuccess;
    }
    hipError_t e = hipMalloc(p, r);
    if (e == hipErrorOutOfMemory && !ctx->cache.empty()) {
        (void)hipGetLastError();
        slat_dev_trim(ctx);
        e = hipMalloc(p, r);
    }
    if (e == hipSuccess) {
        ctx->live[*p] = {*p, r, s, *p};
        ctx->chunks[*p] = r;
        ctx->mem_changed = true;
    }
    return e;
}

void slat_dev_free(slat_ctx *ctx, void *p, hipStream_t s) {
    auto it = ctx->live.find(p);
    if (it == ctx->live.end()) return;  // not ours (or freed already)
    slat_ctx::Block b = it->second;
    ctx->live.erase(it);
    for (auto *tab : {ctx->lane_miss, ctx->list_miss})
        for (int i = 0; i < 8; ++i)
            if (tab[i].a_rp == p || tab[i].a_col == p || tab[i].b_rp == p || tab[i].b_col == p) tab[i] = {};
    b.s = s;
    cache_put(ctx, b);
    if (ctx->cache_bytes > kCacheMax) {
        (void)hipDeviceSynchronize();  // the evicted chunks may still be read by queued work
        for (size_t i = 0; i < ctx->cache.size() && ctx->cache_bytes > kCacheMax / 2;) {
            if (whole_chunk(ctx, ctx->cache[i])) {
                ctx->cache_bytes -= ctx->cache[i].bytes;
                ctx->chunks.erase(ctx->cache[i].p);
                (void)hipFree(ctx->cache[i].p);
                ctx->mem_changed = true;
                ctx->cache.erase(ctx->cache.begin() + (std::ptrdiff_t)i);
            } else {
                ++i;
            }
        }
    }
}

void slat_dev_shrink(slat_ctx *ctx, void *p, size_t bytes) {
    auto it = ctx->live.find(p);
    if (it == ctx->live.end()) return;
    const size_t r = round_block(bytes);
    slat_ctx::Block &b = it->second;
    if (b.bytes < r + kSplitMin) return;  // not worth a piece
    // the tail is free on the piece's stream from here on: work queued later on that stream runs
    // after the work that wrote the kept head
    cache_put(ctx, {(uint8_t *)p + r, b.bytes - r, b.s, b.chunk});
    b.bytes = r;
}

void slat_dev_trim(slat_ctx *ctx) {
    if (ctx->cache.empty()) return;
    (void)hipDeviceSynchronize();
    for (size_t i = 0; i < ctx->cache.size();) {
        if (whole_chunk(ctx, ctx->cache[i])) {
            ctx->cache_bytes -= ctx->cache[i].bytes;
            ctx->chunks.erase(ctx->cache[i].p);
            (void)hipFree(ctx->cache[i].p);
            ctx->mem_changed = true;
            ctx->cache.erase(ctx->cache.begin() + (std::ptrdiff_t)i);
        } else {
            ++i;  // part of a chunk that still holds live pieces
        }
    }
}

// context teardown: every chunk back to the driver, live pieces included
static void dev_release_all(slat_ctx *ctx) {
    (void)hipDeviceSynchronize();
    for (auto &c : ctx->chunks) (void)hipFree(c.first);
    ctx->chunks.clear();
    ctx->cache.clear();
    ctx->live.clear();
    ctx->cache_bytes = 0;
}

slat_status slat_ensure_ws(slat_ctx *ctx, size_t bytes) {
    if (bytes <= ctx->ws_bytes) return SLAT_OK;
    SLAT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->ws) SLAT_HIP(ctx, hipFree(ctx->ws));
    ctx->ws = nullptr;
    ctx->ws_bytes = 0;
    size_t nb = std::max(bytes, (size_t)1 << 20);
    nb = std::max(nb, ctx->ws_bytes * 2);
    if (hipMalloc(&ctx->ws, nb) != hipSuccess) return fail(ctx, SLAT_EOOM, "workspace allocation failed");
    ctx->ws_bytes = nb;
    return SLAT_OK;
}

slat_status slat_check_view(slat_ctx *ctx, const slat_csr_view *v, const char *name) {
    if (!v) return fail(ctx, SLAT_EINVAL, std::string(name) + " is null");
    if (v->dtype < SLAT_U32 || v->dtype > SLAT_F64) return fail(ctx, SLAT_EINVAL, std::string(name) + ": bad dtype");
    if (v->n_rows && !v->row_ptr) return fail(ctx, SLAT_EINVAL, std::string(name) + ": null row_ptr");
    if (v->nnz && (!v->col_idx || !v->values)) return fail(ctx, SLAT_EINVAL, std::string(name) + ": null arrays");
    if (v->n_cols > 0xFFFFFFFFull || v->n_rows > 0xFFFFFFFFull) return fail(ctx, SLAT_EINVAL, std::string(name) + ": dims exceed u32 ids");
    return SLAT_OK;
}

extern "C" slat_status slat_csr_create(slat_ctx *ctx, const slat_csr_view *src, slat_csr *out) {
    if (!ctx || !out) return SLAT_EINVAL;
    slat_status st = slat_check_view(ctx, src, "src");
    if (st) return st;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    std::memset(out, 0, sizeof *out);
    const size_t vs = vsize(src->dtype);
    SLAT_HIP(ctx, alloc_joint(ctx, out, src->n_rows, src->nnz, vs, ctx->stream));
    if (!src->n_rows) SLAT_HIP(ctx, hipMemsetAsync(out->row_ptr, 0, 8, ctx->stream));
    if (src->residency == SLAT_HOST) {
        // host arrays (the drop-in's Vecs): the staging ring for pageable memory (slat_hostio.hip)
        const slat_hostseg segs[3] = {{(void *)src->row_ptr, out->row_ptr, src->n_rows ? (src->n_rows + 1) * 8 : 0},
                                      {(void *)src->col_idx, out->col_idx, src->nnz * 4},
                                      {(void *)src->values, out->values, src->nnz * vs}};
        if ((st = slat_copy_h2d(ctx, segs, 3))) {
            slat_csr_free(ctx, out);
            return st;
        }
    } else {
        const hipMemcpyKind kind = hipMemcpyDeviceToDevice;
        if (src->n_rows)
            SLAT_HIP(ctx, hipMemcpyAsync(out->row_ptr, src->row_ptr, (src->n_rows + 1) * 8, kind, ctx->stream));
        if (src->nnz) {
            SLAT_HIP(ctx, hipMemcpyAsync(out->col_idx, src->col_idx, src->nnz * 4, kind, ctx->stream));
            SLAT_HIP(ctx, hipMemcpyAsync(out->values, src->values, src->nnz * vs, kind, ctx->stream));
        }
    }
    out->n_rows = src->n_rows;
    out->n_cols = src->n_cols;
    out->nnz = src->nnz;
    out->capacity = src->nnz;
    out->dtype = src->dtype;
    out->device = ctx->device;
    uint64_t mr = src->max_row_nnz;
    if (mr == 0 && src->n_rows) {
        if (src->residency == SLAT_HOST) {
            for (uint64_t i = 0; i < src->n_rows; ++i) mr = std::max(mr, src->row_ptr[i + 1] - src->row_ptr[i]);
        } else {
            slat_csr_view v = slat_csr_view_of(out);
            st = slat_csr_max_row_nnz(ctx, &v, &mr);
            if (st) return st;
        }
    }
    out->max_row_nnz = mr;
    SLAT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return SLAT_OK;
}

extern "C" slat_status slat_csr_to_host(slat_ctx *ctx, const slat_csr_view *src, uint64_t *row_ptr, uint32_t *col,
                                        void *vals) {
    if (!ctx) return SLAT_EINVAL;
    slat_status st = slat_check_view(ctx, src, "src");
    if (st) return st;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    if (src->residency != SLAT_HOST) {
        // device -> the caller's host arrays: the staging ring for pageable memory (slat_hostio.hip)
        const slat_hostseg segs[3] = {{row_ptr, (void *)src->row_ptr, row_ptr ? (src->n_rows + 1) * 8 : 0},
                                      {col, (void *)src->col_idx, col ? src->nnz * 4 : 0},
                                      {vals, (void *)src->values, vals ? src->nnz * vsize(src->dtype) : 0}};
        return slat_copy_d2h(ctx, segs, 3);
    }
    const hipMemcpyKind kind = hipMemcpyHostToHost;
    if (row_ptr) SLAT_HIP(ctx, hipMemcpyAsync(row_ptr, src->row_ptr, (src->n_rows + 1) * 8, kind, ctx->stream));
    if (src->nnz && col) SLAT_HIP(ctx, hipMemcpyAsync(col, src->col_idx, src->nnz * 4, kind, ctx->stream));
    if (src->nnz && vals) SLAT_HIP(ctx, hipMemcpyAsync(vals, src->values, src->nnz * vsize(src->dtype), kind, ctx->stream));
    SLAT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return SLAT_OK;
}

extern "C" slat_status slat_csr_max_row_nnz(slat_ctx *ctx, const slat_csr_view *m, uint64_t *out) {
    if (!ctx || !m || !out) return SLAT_EINVAL;
    *out = 0;
    if (m->n_rows == 0) return SLAT_OK;
    if (m->residency == SLAT_HOST) {
        uint64_t mr = 0;
        for (uint64_t i = 0; i < m->n_rows; ++i) mr = std::max(mr, m->row_ptr[i + 1] - m->row_ptr[i]);
        *out = mr;
        return SLAT_OK;
    }
    slat_status st = slat_ensure_ws(ctx, 4096);
    if (st) return st;
    unsigned long long *shards = (unsigned long long *)ctx->ws;
    SLAT_HIP(ctx, hipMemsetAsync(shards, 0, sizeof(unsigned long long) * kShards * kShardStride, ctx->stream));
    const uint64_t blocks = std::min<uint64_t>((m->n_rows + kBlock - 1) / kBlock, 1024);
    hipLaunchKernelGGL(k_max_row, dim3((unsigned)blocks), dim3(kBlock), 0, ctx->stream, m->row_ptr, m->n_rows, shards);
    SLAT_HIP(ctx, hipGetLastError());
    SLAT_HIP(ctx, hipMemcpyAsync(ctx->h_shards, shards, sizeof(unsigned long long) * kShards * kShardStride,
                                 hipMemcpyDeviceToHost, ctx->stream));
    SLAT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    uint64_t mr = 0;
    for (int s = 0; s < kShards; ++s) mr = std::max<uint64_t>(mr, ctx->h_shards[s * kShardStride + 1]);
    *out = mr;
    return SLAT_OK;
}

// ---------------------------------------------------------------------------------------------
// launch helpers (templated over semiring and traversal modes)
// ---------------------------------------------------------------------------------------------
// blocks of k_build_ell (each stores one B-value partial for k_scan_rows when u32)
static uint32_t build_ell_blocks(const slat_csr_view *B, uint32_t wq) {
    return (uint32_t)std::max<uint64_t>(std::min<uint64_t>((B->n_rows * wq + kBlock - 1) / kBlock, 4096), 1);
}

template <typename S>
static hipError_t launch_build_ell(hipStream_t s, const slat_csr_view *B, uint32_t wq, uint32_t *ecol, void *eval,
                                   uint8_t *eng, unsigned long long *part) {
    hipLaunchKernelGGL(k_build_ell<S>, dim3(build_ell_blocks(B, wq)), dim3(kBlock), 0, s, B->row_ptr, B->col_idx,
                       (const S *)B->values, (uint32_t)B->n_rows, wq, ecol, (S *)eval, eng, part);
    return hipGetLastError();
}

template <typename Sem>
static hipError_t launch_compact(dim3 grid, hipStream_t s, const uint64_t *orp, const uint64_t *nrp, uint64_t n,
                                 const uint32_t *oc, const void *ov, uint32_t *nc, void *nv) {
    using S = typename Sem::S;
    hipLaunchKernelGGL(k_compact<Sem>, grid, dim3(kBlock), 0, s, orp, nrp, n, oc, (const S *)ov, nc, (S *)nv);
    return hipGetLastError();
}

// row_ptr[0..n] of a count vector: k_scan_rows (one kernel); the total and the max count land in
// ctx->h_out[0], [1] once the stream reaches that point
uint32_t slat_next_scan_epoch(slat_ctx *ctx, hipStream_t s) {
    if (++ctx->scan_epoch >= (1u << 22)) {  // tag wrap: clear every tagged word once
        if (ctx->d_status) (void)hipMemsetAsync(ctx->d_status, 0, ctx->status_cap * 8, s);
        (void)hipMemsetAsync(ctx->d_maxw, 0, kMaxwBytes, s);
        ctx->scan_epoch = 1;
    }
    return ctx->scan_epoch;
}

// the look-back status words for `tiles` tiles (k_scan_rows, k_tiny)
static slat_status ensure_status(slat_ctx *ctx, uint64_t tiles, hipStream_t s) {
    if (tiles > ctx->status_cap) {
        if (ctx->d_status) slat_dev_free(ctx, ctx->d_status, s);
        ctx->d_status = nullptr;
        const uint64_t cap = std::max<uint64_t>(tiles, 1024);
        SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&ctx->d_status, cap * 8, s));
        SLAT_HIP(ctx, hipMemsetAsync(ctx->d_status, 0, cap * 8, s));
        ctx->status_cap = cap;
    }
    return SLAT_OK;
}

slat_status slat_launch_scan(slat_ctx *ctx, const uint64_t *counts, uint64_t n, uint64_t *rp, hipStream_t s,
                             const unsigned long long *bpart, uint32_t nbpart, uint32_t vepoch, const uint32_t *bmax,
                             uint32_t nbmax, unsigned int *zero_word) {
    const uint64_t tiles = std::max<uint64_t>((n + kScanTile - 1) / kScanTile, 1);
    slat_status st;
    if ((st = ensure_status(ctx, tiles, s))) return st;
    const uint32_t epoch = slat_next_scan_epoch(ctx, s);
    // At most one block per CU, each taking its tiles in order (k_scan_rows: block b walks tiles b,
    // b + G, ...). Block 0's second tile looks back on tile G - 1, so when tiles > G forward progress
    // assumes all G blocks are resident at once. G <= the CU count, and one CU holds several of these
    // blocks (256 threads, a few hundred bytes of LDS), so they co-reside unless another process
    // holds every CU for the whole kernel; two ranks sharing one GPU (tests/test_dist_hip_gpu.py)
    // time-slice, and their kernels retire. Earlier tiles' blocks never wait on later ones.
    const uint64_t grid = std::min<uint64_t>(tiles, (uint64_t)ctx->cu_count);
    hipLaunchKernelGGL(k_scan_rows, dim3((unsigned)grid), dim3(kScanThreads), 0, s, counts, n, rp, ctx->d_status, epoch,
                       ctx->d_maxw, ctx->h_out_dev, bpart, nbpart, ctx->d_vmax, vepoch, bmax, nbmax, zero_word);
    SLAT_HIP(ctx, hipGetLastError());
    return SLAT_OK;
}


// Window geometry: ww bitmap words, a multiple of 64 (words are handled in 64-word blocks, one word
// per lane) and at most max_ww (u16 column offsets need 32 * ww <= 65536; the touched-block mask
// needs ww / 64 <= 32). `wide` = one window does not cover all columns.
static void pick_window(uint64_t ncols, uint32_t threads, uint32_t max_ww, uint32_t &ww, uint32_t &wide) {
    const uint64_t words = std::max<uint64_t>((ncols + 31) / 32, 1);
    uint64_t blocks = (words + threads - 1) / threads;
    const uint64_t max_blocks = max_ww / threads;
    wide = 0;
    if (blocks > max_blocks) {
        blocks = max_blocks;
        wide = 1;
    }
    ww = (uint32_t)(blocks * threads);
}

// End of a call: poll the stream instead of a blocking sync, whose wake-up adds microseconds to
// every call (SLAT_BLOCKING_SYNC=1 restores the blocking wait)
// diagnostics (SLAT_HOST_CLOCK=1): host time of each part of a call, printed every 256 calls:
// [0] checks and hipSetDevice, [1] launch geometry, [2] workspace, [3] the ELL build's launch, [4] C's
// allocation, [5] the symbolic launches, [6] the scan / numeric launches, [7] waiting for them,
// [8] the rest
struct HostClock {
    static constexpr int kN = 9;
    static bool on() {
        static const bool e = slat_ab_knob("SLAT_HOST_CLOCK") != nullptr;
        return e;
    }
    std::chrono::steady_clock::time_point t;
    void start() {
        if (on()) t = std::chrono::steady_clock::now();
    }
    void mark(int i) {
        if (!on()) return;
        static thread_local double acc[kN];
        static thread_local long calls = 0;  // the first 64 calls (one-time costs: code object loads,
                                             // occupancy queries) are not counted
        const auto now = std::chrono::steady_clock::now();
        if (calls >= 64) acc[i] += std::chrono::duration<double, std::micro>(now - t).count();
        t = now;
        if (i == kN - 1 && ++calls > 64 && (calls - 64) % 256 == 0) {
            std::fprintf(stderr,
                         "host us/call: checks %.2f geometry %.2f workspace %.2f ell %.2f alloc %.2f symbolic %.2f "
                         "scan+numeric %.2f wait %.2f finish %.2f\n",
                         acc[0] / 256, acc[1] / 256, acc[2] / 256, acc[3] / 256, acc[4] / 256, acc[5] / 256,
                         acc[6] / 256, acc[7] / 256, acc[8] / 256);
            for (double &x : acc) x = 0;
        }
    }
};

// relaxed: the call's results are read through stream-ordered copies, and the mapped words the host
// reads (nnz, max row, rows with zeros) were stored by earlier kernels, which completed their stores
// before this one started. A release here wrote back the L2 and took 4 us.
__global__ void k_signal(unsigned long long *word, unsigned long long v) {
    __hip_atomic_store(word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wait for the call's kernels. Default: a one-thread kernel queued after them stores a sequence
// number into the context's mapped host words, and the host spins on that word. Measured on this
// runtime (tools/repro/launch_latency.hip, 4 small kernels per call): 15.2 us per call, against 17.6
// for hipStreamSynchronize and 27.6 for a hipStreamQuery spin (each query slows the runtime down).
// Every 2^16 polls the stream is queried, so a faulted kernel surfaces as an error, not a hang.
// SLAT_WAIT=sync | query selects the other two, SLAT_WAIT=write stores the word with
// hipStreamWriteValue64 instead of k_signal (A/B only).
static int wait_mode() {
    static const int mode = [] {
        const char *e = slat_ab_knob("SLAT_WAIT");
        if (slat_ab_knob("SLAT_BLOCKING_SYNC") || (e && !std::strcmp(e, "sync"))) return 1;
        if (e && !std::strcmp(e, "write")) return 3;  // the sequence word stored by a stream write op
        return e && !std::strcmp(e, "query") ? 2 : 0;
    }();
    return mode;
}
// signalled != 0: the call's last kernel stores that sequence number itself (signal_done)
static hipError_t wait_stream(slat_ctx *ctx, hipStream_t s, unsigned long long signalled = 0) {
    const int mode = wait_mode();
    hipError_t e;
    if (mode == 1) return hipStreamSynchronize(s);
    if (mode == 2) {
        while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
        }
        return e;
    }
    const unsigned long long seq = signalled ? signalled : ++ctx->done_seq;
    if (signalled) {
    } else if (mode == 3) {
        if ((e = hipStreamWriteValue64(s, ctx->h_out_dev + 7, seq, 0)) != hipSuccess) return e;
    } else {
        hipLaunchKernelGGL(k_signal, dim3(1), dim3(1), 0, s, ctx->h_out_dev + 7, seq);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const volatile unsigned long long *w = ctx->h_out + 7;
    for (uint32_t i = 1; *w != seq; ++i)
        if ((i & 0xFFFFu) == 0) {
            e = hipStreamQuery(s);
            if (e == hipSuccess) return *w == seq ? hipSuccess : hipStreamSynchronize(s);
            if (e != hipErrorNotReady) return e;
        }
    // the runtime learns of completed work only through its own calls: let it retire the queue now
    // and then (event timestamps are read after a hipEventSynchronize of their own)
    if ((seq & 63) == 0 && (e = hipStreamQuery(s)) != hipSuccess && e != hipErrorNotReady) return e;
    return hipSuccess;
}

// B's padded ELL image applies: short rows (<= 32 entries), a bounded blow-up, 24-bit row indices and
// 31-bit byte offsets in the kernels
static bool ell_fits(const slat_csr_view *B, uint64_t maxrow_b, size_t vs) {
    const uint64_t q = (maxrow_b + 3) / 4;
    const uint64_t bytes = B->n_rows * q * 4 * (4 + vs);
    return maxrow_b <= 32 && bytes <= std::max<uint64_t>(64ull << 20, 8 * B->nnz * (4 + vs)) &&
           B->n_rows < (1ull << 24) && B->n_rows * q * 16 * (vs / 4) < (1ull << 31);
}

static slat_status rowblock_impl(slat_ctx *ctx, const slat_csr_view *A, uint64_t row_begin, uint64_t row_end,
                                 const slat_csr_view *B, const slat_bprep *prep, slat_csr *C, uint32_t flags);

extern "C" slat_status slat_spgemm_rowblock(slat_ctx *ctx, const slat_csr_view *A, uint64_t row_begin,
                                            uint64_t row_end, const slat_csr_view *B, slat_csr *C, uint32_t flags) {
    return rowblock_impl(ctx, A, row_begin, row_end, B, nullptr, C, flags);
}

extern "C" slat_status slat_spgemm_rowblock_prepared(slat_ctx *ctx, const slat_csr_view *A, uint64_t row_begin,
                                                     uint64_t row_end, const slat_bprep *B, slat_csr *C, uint32_t flags) {
    if (!ctx || !B) return SLAT_EINVAL;
    if (B->device != ctx->device) return fail(ctx, SLAT_EINVAL, "prepared B belongs to another device");
    if (B->owner != ctx) return fail(ctx, SLAT_EINVAL, "prepared B belongs to another context");
    return rowblock_impl(ctx, A, row_begin, row_end, &B->b, B, C, flags);
}

static slat_status rowblock_impl(slat_ctx *ctx, const slat_csr_view *A, uint64_t row_begin, uint64_t row_end,
                                 const slat_csr_view *B, const slat_bprep *prep, slat_csr *C, uint32_t flags) {
    if (!ctx || !C) return SLAT_EINVAL;
    HostClock hc;
    hc.start();
    slat_status st;
    if ((st = slat_check_view(ctx, A, "A")) || (st = slat_check_view(ctx, B, "B"))) return st;
    if (A->dtype != B->dtype) return fail(ctx, SLAT_EINVAL, "A and B value types differ");
    if (A->n_cols != B->n_rows) return fail(ctx, SLAT_EDIM, "A.n_cols != B.n_rows");
    if (B->n_cols > 0xFFFFFFFFull - (1ull << 17))  // column ids are u32; the top 2^17 values stay free
        return fail(ctx, SLAT_ENOTSUP, "n_cols too large for u32 column ids");
    if (row_begin > row_end || row_end > A->n_rows) return fail(ctx, SLAT_EINVAL, "bad row block");
    if (A->residency != SLAT_DEVICE || B->residency != SLAT_DEVICE) {
        // host inputs: stage through owned device copies (PCIe outside the engine's hot path)
        slat_csr dA = {}, dB = {};
        const slat_csr_view *pa = A, *pb = B;
        slat_csr_view va, vb;
        if (A->residency != SLAT_DEVICE) {
            if ((st = slat_csr_create(ctx, A, &dA))) return st;
            va = slat_csr_view_of(&dA);
            pa = &va;
        }
        if (B->residency != SLAT_DEVICE) {
            if ((st = slat_csr_create(ctx, B, &dB))) {
                slat_csr_free(ctx, &dA);
                return st;
            }
            vb = slat_csr_view_of(&dB);
            pb = &vb;
        }
        st = rowblock_impl(ctx, pa, row_begin, row_end, pb, nullptr, C, flags);
        if (dA.row_ptr) slat_csr_free(ctx, &dA);
        if (dB.row_ptr) slat_csr_free(ctx, &dB);
        return st;
    }
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    hc.mark(0);
    std::memset(C, 0, sizeof *C);
    std::memset(&ctx->stats, 0, sizeof ctx->stats);
    const uint64_t n = row_end - row_begin;
    const uint64_t ncols = B->n_cols;
    const int32_t dt = A->dtype;
    const size_t vs = vsize(dt);
    // f64 in any summation order (tolerance-checked, config C5) instead of the reference's fold order
    const bool f64any = dt == SLAT_F64 && (flags & SLAT_FLAG_F64_ANY_ORDER);
    hipStream_t s = ctx->stream;
    C->n_rows = n;
    C->n_cols = ncols;
    C->dtype = dt;
    C->device = ctx->device;
    if (n == 0 || ncols == 0 || A->nnz == 0 || B->nnz == 0) {
        // empty product: all-zero row_ptr
        SLAT_HIP(ctx, alloc_joint(ctx, C, n, 0, vs, s));
        SLAT_HIP(ctx, hipMemsetAsync(C->row_ptr, 0, (n + 1) * 8, s));
        SLAT_HIP(ctx, hipStreamSynchronize(s));
        return SLAT_OK;
    }
    uint64_t maxrow_b = prep ? prep->maxrow_b : B->max_row_nnz;
    if (maxrow_b == 0 && (st = slat_csr_max_row_nnz(ctx, B, &maxrow_b))) return st;
    // C's capacity by the exact bound nnz(A block) x max row(B) (no mid-call sync) unless it exceeds
    // the budget: free device memory / 4 (re-read when this context's pool grew or shrank, else every
    // 1024 calls: the query costs tens of microseconds of host time) and at most kBoundBytes (a loose
    // bound, power-law B: nnz(A) x a hub row, would make every call allocate and release tens of GB,
    // which costs far more than the exact path's one sync). Decided before the kernel choice: the
    // one-kernel paths (tiny, lane) need the bound-sized C, so an exact call takes the pipeline with
    // its ELL image, stored bitmaps and hash batches
    if (ctx->mem_changed || ctx->free_age++ % 1024 == 0) {
        size_t total_b = 0;
        (void)hipMemGetInfo(&ctx->free_b, &total_b);
        ctx->mem_changed = false;
    }
    static const uint64_t kBoundBytes = [] {
        const char *e = slat_ab_knob("SLAT_BOUND_MAX_BYTES");
        return e ? std::strtoull(e, nullptr, 10) : (4ull << 30);
    }();
    const unsigned __int128 budget = std::min<unsigned __int128>(ctx->free_b / 4, kBoundBytes);
    // A entries of the row block: the whole A's nnz, then rows x A's max row when known (no sync);
    // only a block whose bound is still over the budget reads its two row_ptr words (one round trip,
    // which cost a row-block call ~15 us of its ~300: one rank's eighth of C4)
    uint64_t a_nnz_block = A->nnz;
    if (n < A->n_rows) {
        if (A->max_row_nnz) a_nnz_block = std::min<uint64_t>(a_nnz_block, n * A->max_row_nnz);
        if ((unsigned __int128)a_nnz_block * maxrow_b * (4 + vs) > budget) {
            SLAT_HIP(ctx, hipMemcpyAsync(ctx->h_shards, A->row_ptr + row_begin, 8, hipMemcpyDeviceToHost, ctx->stream));
            SLAT_HIP(ctx, hipMemcpyAsync(ctx->h_shards + 1, A->row_ptr + row_end, 8, hipMemcpyDeviceToHost, ctx->stream));
            SLAT_HIP(ctx, hipStreamSynchronize(ctx->stream));
            if (ctx->h_shards[1] < ctx->h_shards[0] || ctx->h_shards[1] - ctx->h_shards[0] > A->nnz)
                return fail(ctx, SLAT_EINVAL, "A.row_ptr is not monotonic over the row block");
            a_nnz_block = ctx->h_shards[1] - ctx->h_shards[0];
        }
    }
    unsigned __int128 bound128 = (unsigned __int128)a_nnz_block * maxrow_b;
    const unsigned __int128 dense = (unsigned __int128)n * ncols;
    if (bound128 > dense) bound128 = dense;
    bool exact = (flags & SLAT_FLAG_EXACT_ALLOC) || bound128 * (4 + vs) > budget;

    Args a = {};
    a.a_rp = A->row_ptr + row_begin;
    a.a_col = A->col_idx;
    a.a_val = A->values;
    a.b_rp = B->row_ptr;
    a.b_col = B->col_idx;
    a.b_val = B->values;
    a.nrows = n;
    a.ncols = ncols;
    a.b_nrows = B->n_rows;
    a.stats = (flags & SLAT_FLAG_STATS) ? 1u : 0u;

    // 32-bit offsets whenever every position fits (the common case; halves the index math)
    const bool idx32 = A->nnz < 0xFFFFFFFFull && B->nnz < 0xFFFFFFFFull && !(flags & SLAT_FLAG_IDX64);
    // environment knobs (A/B experiments only) are read once: a getenv per call is host time on
    // every call
    static const uint32_t ablate = [] {  // experiments only: never reaches the real pipeline's kernels
        const char *e = slat_ab_knob("SLAT_ABLATE");
        return e ? (uint32_t)std::atoi(e) : 0u;
    }();
    Args asym = a;
    pick_window(ncols, kWave, 1984, asym.ww, asym.wide);
    pick_window(ncols, kWave, 1984, a.ww, a.wide);
    // rank slots per wave: 896 narrow (u32 + u16) slots and MODE 4's 64 sink slots; 3 blocks/CU at the
    // 30^3 window (MODE 0 takes all 960 as slots)
    a.area = 960 * 6;
    // Wide launches (columns beyond one window): short rows take the per-wave LDS hash table
    // (MAGNUS's small-row category); the rest keep row-span windows, made small so the shared
    // region stays small: symbolic 1024 words (the hash keys' size), numeric 256 words.
    // Wide launches (columns beyond one window) split the rows by MAGNUS-style category into two
    // launches per pass: short rows in a per-wave LDS hash table (mode 1), the rest by row-span
    // windows (mode 2; numeric windows of 1024 words keep two blocks per CU).
    // padded ELL copy of B when its rows are short (bounded blow-up)
    const uint64_t wq = (maxrow_b + 3) / 4;
    // small products: the whole call in one regular launch (slat_tiny.hip) — one window of at most
    // 8192 columns, <= 2048 rows (at 3375 rows, the 15^3 cells, it measured 1-2 us slower than the
    // pipeline: profiles/r03_small_cells_tiny_abi.csv), 32-bit offsets, a wave per row with every row in flight, a product bound a wave
    // finishes in microseconds, no fat rows, and no per-pass timing or stats (those report the
    // regular pipeline's passes)
    static const bool kNoTiny = slat_ab_knob("SLAT_NO_TINY") != nullptr;
    const bool tiny = !kNoTiny && !exact && !asym.wide && ncols <= 8192 && n <= 2048 && idx32 && wait_mode() == 0 && !ablate &&
                      !(flags & (SLAT_FLAG_TIMING | SLAT_FLAG_STATS | SLAT_FLAG_NO_TINY)) &&
                      g_progress.load(std::memory_order_relaxed) == 0 &&
                      (unsigned __int128)a_nnz_block * maxrow_b <= (1u << 18) &&
                      (A->max_row_nnz ? (unsigned __int128)A->max_row_nnz * maxrow_b < slat_fat_min(false) : maxrow_b <= 32);
    // rows of at most slat_lane_cap() products: the whole call in one kernel, a row per lane
    // (slat_lane.hip: C1, the 30^3 chain's A * A, 88 -> ~25 us). Tried when the bound max row(A) x
    // max row(B) is <= 4 caps; a row past the cap sets the mapped overflow word and the call reruns
    // through the pipeline. Column ids < 2^26 - 1: the sort key (column << 6) | slot of column 2^26 - 1
    // at slot 63 would equal the padding key kSent
    static const bool kNoLane = slat_ab_knob("SLAT_NO_LANE") != nullptr;
    bool lane = !kNoLane && !exact && !tiny && idx32 && wait_mode() == 0 && !ablate && ncols < (1ull << 26) &&
                !(flags & (SLAT_FLAG_STATS | SLAT_FLAG_NO_TINY)) && g_progress.load(std::memory_order_relaxed) == 0 &&
                A->max_row_nnz && (unsigned __int128)A->max_row_nnz * maxrow_b <= 4 * slat_lane_cap();
    // (a bound above one cap may overflow: a pair that did is sent to the pipeline from then on. The
    // 30^3 sweep's e/n-4 cell overflowed on every call and paid both paths, 95 -> 149 us)
    if (lane && (unsigned __int128)A->max_row_nnz * maxrow_b > slat_lane_cap())
        for (const auto &m : ctx->lane_miss)
            if (m.a_rp == A->row_ptr && m.a_col == A->col_idx && m.b_rp == B->row_ptr && m.b_col == B->col_idx &&
                m.a_nnz == A->nnz && m.b_nnz == B->nnz && m.a_rows == A->n_rows && m.row_begin == row_begin &&
                m.row_end == row_end)
                lane = false;
    static const bool kNoEll = slat_ab_knob("SLAT_NO_ELL") != nullptr;
    const bool ell = ell_fits(B, maxrow_b, vs) && !kNoEll && !tiny && !lane;
    // a prepared B (slat_bprep_create) brings its image and value summary: no per-call build
    const bool pell = ell && prep && prep->ell && prep->wq == wq;
    // stored bitmaps (single-window launches): symbolic keeps each row's touched bitmap blocks for
    // numeric, n * ww words at most (only touched blocks are written), capped against free memory
    const uint64_t sbm_words = a.wide ? 0 : (uint64_t)n * a.ww;
    static const bool kNoSbm = slat_ab_knob("SLAT_NO_SBM") != nullptr;
    const bool sbm = !a.wide && sbm_words * 4 <= std::max<uint64_t>(256ull << 20, ctx->free_b / 16) && !kNoSbm && !tiny &&
                     !lane;
    static const bool kNoHash = slat_ab_knob("SLAT_NO_HASH") != nullptr;
    // single-window launches (the 30^3 chain, configs C1 / C2 / C3) batch their short rows the same way
    // (MAGNUS's small-row category) when the workgroup kernels take the rest: rows of <= 256 products
    // (a bound: 4 per ELL group) in symbolic, <= 256 outputs in numeric, so every row numeric lists
    // has a stored bitmap. f64 in the fold order keeps one kernel for every row
    // Off by default (SLAT_SHORT1=1: on when every row is short by the bound, A's longest row x B's
    // longest row rounded up to ELL groups <= 256; SLAT_SHORT1_ANY=1: on for any single-window launch).
    // Measured slower everywhere on the 30^3 chain: with long rows among them, MODE 2 over listed rows
    // plus the hash path for rows of ~250 outputs took A^6 * A from 0.153 to 0.363 ms
    // (profiles/r04_ab3.txt); on C1 (A * A, every row short) the 8-row hash batches cost ~56 k cycles
    // each (a chain of dependent loads, then the 256-key sort) and numeric took 110 us against the
    // window kernel's 46 (profiles/r04_inv1.txt)
    static const bool kShort1 = slat_ab_knob("SLAT_SHORT1") != nullptr;
    static const bool kShort1Any = slat_ab_knob("SLAT_SHORT1_ANY") != nullptr;
    const bool bound_short = A->max_row_nnz && maxrow_b > 0 &&
                             (unsigned __int128)A->max_row_nnz * (4 * ((maxrow_b + 3) / 4)) <= kHashT / 2;
    const bool short1 = !a.wide && ell && !tiny && !ablate && (dt != SLAT_F64 || f64any) &&
                        ((kShort1 && bound_short) || kShort1Any);
    const bool hash = (asym.wide || short1) && !kNoHash && !lane;
    if (hash) {
        if (asym.wide) a.ww = std::min<uint32_t>(a.ww, 1024);
        a.b_maxrow = asym.b_maxrow = (uint32_t)std::min<uint64_t>(maxrow_b, 0xFFFFFFFFull);
    }

    // LDS sizing and grids. The numeric grid is the kernel's resident capacity (waves stride over
    // rows; measured faster than oversubscribing); symbolic takes up to 16 blocks per CU.
    const int wpb = kBlock / kWave;
    static const int kCap = [] {  // tuning knob: rank slots per wave
        const char *e = slat_ab_knob("SLAT_CAP");
        return e ? std::max(64, std::atoi(e)) : 0;
    }();
    if (kCap) a.area = 6 * kCap;
    a.area = (a.area + 15) & ~15u;
    const size_t num_lds = (size_t)wpb * num_layout(a.ww, a.area).bytes;
    // short rows batched several per hash table (integer semirings with the ELL copy of B), else
    // one row per table; composite (row, column) keys need the column bits + 6 <= 31
    // symbolic batches for every value type (it never reads values); numeric for the integer ones
    // B in CSR form (rows past the ELL limit: power-law graphs) batches the same way, reading its
    // groups of 4 where they lie (u32 entry offsets: B of < 2^32 entries; SLAT_NO_CSR_BATCH: one
    // row per table, A/B)
    static const bool kNoBatch = slat_ab_knob("SLAT_NO_BATCH") != nullptr;
    static const bool kNoCsrBatch = slat_ab_knob("SLAT_NO_CSR_BATCH") != nullptr;
    const bool csr_batch = !ell && !kNoCsrBatch && B->nnz < 0xFFFFFFF0ull;
    const bool sym_batched = hash && (ell || csr_batch) && !kNoBatch;
    const bool batched = sym_batched && (dt != SLAT_F64 || f64any);
    if (sym_batched) {
        uint32_t cb = 1;
        while (cb < 64 && ((ncols - 1) >> cb)) ++cb;
        a.cbits = cb <= 25 ? cb : 0;
        static const uint32_t kTileRows = [] {  // A/B knob: rows per tile (8 .. 64)
            const char *e = slat_ab_knob("SLAT_TILE_ROWS");
            return e ? (uint32_t)std::min(64, std::max(2, std::atoi(e))) : 0u;
        }();
        if (asym.wide && kTileRows) a.tile_rows = asym.tile_rows = kTileRows;  // (else by occupancy, below)
        if (!asym.wide) {
            a.sym_cap = asym.sym_cap = kHashT / 2;  // every counted row fits numeric's table
            // tiles of fewer rows when 64-row tiles would leave most resident waves idle (27 000 rows:
            // 422 tiles for ~6 000 waves): about 4 tiles per CU slot of 16 waves
            const uint64_t t = (n + (uint64_t)ctx->cu_count * 16 - 1) / ((uint64_t)ctx->cu_count * 16);
            a.tile_rows = asym.tile_rows = kTileRows ? kTileRows : (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(8, t));
        }
    }
    // every row short (single-window launches): A's longest row x B's longest row rounded up to ELL
    // groups (k_symbolic_short's bound, 4 per group) fits the short tables, so the symbolic pass lists
    // no row and the window launches are skipped; numeric's short launch stores the completion word
    // (C1: A^2 of the 30^3 torus, 7 x 8 = 56 products a row)
    // (maxrow_b > 0: with an empty B the bound says nothing about a row's entry count)
    const bool all_short = sym_batched && batched && !asym.wide && bound_short;
    // speculative wide launches: the listed-row launches (symbolic and numeric window rows) are not
    // queued, as if every row were short; a short-row kernel that lists a row sets a mapped word and
    // the call reruns with them (C4 lists none: its two launches found empty lists, ~4.5 us each of a
    // row block's ~217). A triple that listed rows once is remembered and not speculated again
    // (SLAT_NO_SPEC: never, A/B)
    static const bool kNoSpec = slat_ab_knob("SLAT_NO_SPEC") != nullptr;
    auto same = [&](const slat_ctx::LaneMiss &m) {
        return m.a_rp == A->row_ptr && m.a_col == A->col_idx && m.b_rp == B->row_ptr && m.b_col == B->col_idx &&
               m.a_nnz == A->nnz && m.b_nnz == B->nnz && m.a_rows == A->n_rows && m.row_begin == row_begin &&
               m.row_end == row_end;
    };
    bool spec = sym_batched && batched && asym.wide && !kNoSpec && !(flags & kFlagNoSpec) && !exact;
    if (spec)
        for (const auto &m : ctx->list_miss)
            if (same(m)) spec = false;
    const size_t hash_lds =
        (size_t)wpb * (dt == SLAT_U32    ? (!batched ? hash_bytes<SemU32>() : short_bytes<SemU32>())
                       : dt == SLAT_SAT64 ? (!batched ? hash_bytes<SemSat64>() : short_bytes<SemSat64>())
                       : f64any ? (!batched ? hash_bytes<SemF64Any>() : short_bytes<SemF64Any>())
                                : hash_bytes<SemF64>());
    if (num_lds > ctx->lds_per_block_max) return fail(ctx, SLAT_ENOTSUP, "LDS budget too small");
    const size_t sym_lds = (size_t)wpb * asym.ww * 4, sym_hash_lds = (size_t)wpb * kSymHashT * 4;
    const uint64_t row_blocks = (n + wpb - 1) / wpb;
    // grid geometry knobs (A/B only): symbolic blocks per CU, numeric oversubscription factor
    static const uint64_t kSymBpc = [] {
        const char *e = slat_ab_knob("SLAT_SYM_BPC");
        return e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) : 16ull;
    }();
    // (the batched short-row tiles: twice the resident blocks, so blocks that drew cheap tiles
    // make room for more: C4 numeric 1.00 -> 0.91 ms, profiles/r03_ab_dyn_xlane.txt)
    static const uint64_t kNumOver = [] {
        const char *e = slat_ab_knob("SLAT_NUM_OVER");
        return e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) : 2ull;
    }();
    const dim3 sym_grid((unsigned)std::max<uint64_t>(1, std::min(row_blocks, (uint64_t)ctx->cu_count * kSymBpc)));
    const int sem = dt == SLAT_U32 ? kSemU32 : dt == SLAT_SAT64 ? kSemSat64 : f64any ? kSemF64Any : kSemF64;
    if (sym_batched && asym.wide && !a.tile_rows) {
        // Short-row tiles of the wide launches (a wave's unit of work): about three tiles per resident
        // wave W of the kernel, T = n / 3W rows (8 <= T <= 64). Small launches need the rounds: one
        // rank's eighth of C4 (125 000 rows, W ~ 5 000) took 0.216 ms in 8-row tiles, 0.249 in 24-row
        // ones (one round: every wave in the same phase at once) and 0.43 in 64-row ones; the whole
        // C4 (1 M rows) is fastest in 64-row tiles (1.226 ms; 1.315 in 8-row ones: a tile's fixed
        // cost) (profiles/r05_c4_tile_sweep.txt)
        auto rows_for = [&](uint64_t waves) {
            waves = std::max<uint64_t>(waves, 1);
            return (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(8, (n + 3 * waves - 1) / (3 * waves)));
        };
        const uint64_t cus = (uint64_t)ctx->cu_count;
        asym.tile_rows = rows_for(cus * wpb * slat_symbolic_short_blocks_per_cu(idx32, ell, (size_t)wpb * sym_short_bytes()));
        a.tile_rows = batched ? rows_for(cus * wpb * slat_numeric_blocks_per_cu(sem, 3, idx32, ell, hash_lds))
                              : asym.tile_rows;
    }
    const int hash_mode = batched ? 3 : 1;  // numeric instance of the short rows of a wide launch
    auto num_grid = [&](int mode, size_t lds) {
        const int nbpc = slat_numeric_blocks_per_cu(sem, mode, idx32, ell, lds);
        const uint64_t over = mode == 3 ? kNumOver : 1;
        return dim3((unsigned)std::max<uint64_t>(1, std::min(row_blocks, (uint64_t)ctx->cu_count * nbpc * over)));
    };
    // the single-window numeric pass over stored bitmaps with B's ELL image: MODE 4 (spgemm_stored.hpp)
    // for the semirings that add in any order (SLAT_NO_STORED_MODE: the generic MODE 0, A/B)
    static const bool kNoStored = slat_ab_knob("SLAT_NO_STORED_MODE") != nullptr;
    const int win_mode = hash ? 2 : (sbm && ell && !ablate && (dt != SLAT_F64 || f64any) && !kNoStored) ? 4 : 0;
    const dim3 grid = num_grid(win_mode, num_lds);
    const dim3 hash_grid = hash ? num_grid(hash_mode, hash_lds) : dim3(1);
    const bool progress = g_progress.load(std::memory_order_relaxed) != 0;
    const bool timing = (flags & SLAT_FLAG_TIMING) || progress;

    hc.mark(1);
    // workspace: counts [n] | ablation counts [n] | shards | scan temp | ELL cols | ELL vals | ELL groups
    auto up256 = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t counts_b = up256(n * 8);
    const size_t shards_b = 4096 + (SLAT_PHASES ? 8192 : 0);  // + phase-timing slots (diagnostic builds)
    const bool bell = ell && !pell;  // the image built by this call
    const size_t ecol_b = bell ? up256(B->n_rows * wq * 16) : 0, eval_b = bell ? up256(B->n_rows * wq * 4 * vs) : 0;
    const size_t eng_b = bell ? up256(B->n_rows) : 0;
    const size_t sbm_b = sbm ? up256(sbm_words * 4) : 0, smask_b = sbm ? up256(n * 4) : 0;
    const size_t o_abl = counts_b, o_sh = o_abl + counts_b, o_ecol = o_sh + shards_b,
                 o_eval = o_ecol + ecol_b, o_eng = o_eval + eval_b, o_sbm = o_eng + eng_b, o_smask = o_sbm + sbm_b;
    // batched wide launches: symbolic / numeric window-row lists u32[n] | their counters
    const size_t list_b = sym_batched ? up256(n * 4) : 0;
    const size_t o_l1 = o_smask + smask_b, o_l2 = o_l1 + list_b, o_lc = o_l2 + list_b, lc_b = 0;
    // fat rows (MAGNUS's dense-accumulation category) once a row can reach slat_fat_min() products:
    // max row of A x max row of B (A's max row unknown: when B has long rows)
    static const bool kNoFat = slat_ab_knob("SLAT_NO_FAT") != nullptr;
    const uint64_t maxrow_a = A->max_row_nnz;
    const uint64_t fat_min = slat_fat_min(!ell && (dt != SLAT_F64 || f64any));
    const bool fat = !kNoFat && !tiny && !lane && (maxrow_a ? (unsigned __int128)maxrow_a * maxrow_b >= fat_min : maxrow_b > 32);
    // k_build_ell's per-block B-value partials (u32), reduced by k_scan_rows
    const size_t o_part = o_lc + lc_b, part_b = (bell && dt != SLAT_F64) ? 4096 * 8 : 0;
    const size_t o_fat = o_part + part_b, fat_b = fat ? slat_fat_ws(n) : 0;
    const size_t o_bmax = o_fat + fat_b,  // per-block max counts (the symbolic grid)
        bmax_b = up256((size_t)std::max<uint64_t>(sym_grid.x, (uint64_t)ctx->cu_count * 8) * 4);
    if ((st = slat_ensure_ws(ctx, o_bmax + bmax_b))) return st;
    uint8_t *ws = (uint8_t *)ctx->ws;
    if (pell) {
        a.ell_wq = (uint32_t)wq;
        a.ell_col = prep->ecol;
        a.ell_val = prep->eval;
        a.ell_ng = prep->eng;
        if (dt != SLAT_F64) {  // the prepared summary, tagged with its own epoch
            a.b_vmax = prep->vmax;
            a.epoch = prep->epoch;
        }
    } else if (ell) {
        a.ell_wq = (uint32_t)wq;
        a.ell_col = (const uint32_t *)(ws + o_ecol);
        a.ell_val = ws + o_eval;
        a.ell_ng = ws + o_eng;
        if (dt != SLAT_F64) {  // u32 / Sat64: the clamped B-value summary for narrow slots
            a.b_vmax = ctx->d_vmax;
            a.epoch = ++ctx->epoch;
        }
    } else if (dt != SLAT_F64 && kNarrowCsr && !tiny && !lane) {
        // B walked in CSR form: k_bvmax gives the numeric pass the same max(B) (narrow slots, and
        // hub rows accumulate in C instead of one re-traversal per rank chunk)
        a.b_vmax = ctx->d_vmax;
        a.epoch = ++ctx->epoch;
    }
    a.counts = (uint64_t *)ws;
    a.shards = (unsigned long long *)(ws + o_sh);
    if (sbm) {
        a.sbm = (uint32_t *)(ws + o_sbm);
        a.smask = (uint32_t *)(ws + o_smask);
        a.nblk = a.ww / kWave;
    }
    a.host_out = ctx->h_out_dev;
    ctx->h_out[0] = ctx->h_out[1] = ctx->h_out[2] = ctx->h_out[3] = 0;  // no kernel of this context is in flight
    hc.mark(2);
    // the ELL image (or B's value summary) first: it runs while the host allocates C and queues
    // the rest, instead of after the host's setup with the GPU idle
    if (bell) {
        hipError_t be;
        if (dt == SLAT_U32)
            be = launch_build_ell<uint32_t>(s, B, a.ell_wq, (uint32_t *)a.ell_col, (void *)a.ell_val, (uint8_t *)a.ell_ng,
                                            (unsigned long long *)(ws + o_part));
        else if (dt == SLAT_SAT64)
            be = launch_build_ell<unsigned long long>(s, B, a.ell_wq, (uint32_t *)a.ell_col, (void *)a.ell_val, (uint8_t *)a.ell_ng,
                                                      (unsigned long long *)(ws + o_part));
        else
            be = launch_build_ell<double>(s, B, a.ell_wq, (uint32_t *)a.ell_col, (void *)a.ell_val, (uint8_t *)a.ell_ng, nullptr);
        SLAT_HIP(ctx, be);
    } else if (a.b_vmax && B->nnz && !pell) {
        const unsigned g = (unsigned)std::min<uint64_t>((B->nnz + kBlock - 1) / kBlock, (uint64_t)ctx->cu_count * 4);
        if (dt == SLAT_U32)
            hipLaunchKernelGGL(k_bvmax<uint32_t>, dim3(g), dim3(kBlock), 0, s, (const uint32_t *)B->values, B->nnz,
                               ctx->d_vmax, a.epoch);
        else
            hipLaunchKernelGGL(k_bvmax<unsigned long long>, dim3(g), dim3(kBlock), 0, s,
                               (const unsigned long long *)B->values, B->nnz, ctx->d_vmax, a.epoch);
        SLAT_HIP(ctx, hipGetLastError());
    }

    // wide launches with B in CSR form: B bucketed by the window passes' column chunk (32 chunks over
    // the columns, 2^chunk_shift each), so a window walks only its chunks' part of each B row
    uint32_t *wsplit = nullptr;
    static const bool kNoWinSplit = slat_ab_knob("SLAT_NO_WIN_SPLIT") != nullptr;  // A/B knob
    if (hash && !ell && !kNoWinSplit && B->nnz) {
        uint32_t csh = 0;
        while (csh < 58 && ((ncols - 1) >> (csh + 5))) ++csh;
        csh = std::max(csh, 5u);
        const uint64_t nch1 = ((ncols + (1ull << csh) - 1) >> csh) + 1;
        if (B->n_rows * nch1 * 4 <= (256ull << 20) &&
            slat_dev_alloc(ctx, (void **)&wsplit, B->n_rows * nch1 * 4, s) == hipSuccess) {
            // absolute offsets (B of < 2^32 entries): a window's walk then loads a B row's part bounds
            // from the table alone, not also the row pointer
            a.wsplit_abs = B->nnz < 0xFFFFFFFFull ? 1u : 0u;
            if (slat_launch_splits(ctx, B->row_ptr, B->col_idx, B->n_rows, (uint32_t)nch1, csh, wsplit, s, a.wsplit_abs) !=
                hipSuccess) {
                ctx->err = "slat_launch_splits failed";
                slat_dev_free(ctx, wsplit, s);
                return SLAT_EHIP;
            }
            a.wsplit = wsplit;
            a.wnch1 = (uint32_t)nch1;
        } else {
            (void)hipGetLastError();
            wsplit = nullptr;
        }
    }
    hc.mark(3);
    // capacity by the bound computed above (exact: the exact-size path)
    // C's arrays in three pieces: row_ptr, then col_idx and values sized by the bound; after the
    // call both are trimmed to nnz(C) and their tails go back to the context's cache
    SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&C->row_ptr, (n + 1) * 8, s));
    C->alloc = kAllocSeparate;
    if (!exact) {
        C->capacity = (uint64_t)std::max<unsigned __int128>(bound128, 1);
        if (slat_dev_alloc(ctx, (void **)&C->col_idx, C->capacity * 4, s) != hipSuccess ||
            slat_dev_alloc(ctx, &C->values, C->capacity * vs, s) != hipSuccess) {
            // the bound does not fit (or the cache is fragmented): the exact-size path instead
            (void)hipGetLastError();
            if (C->col_idx) slat_dev_free(ctx, C->col_idx, s);
            C->col_idx = nullptr;
            C->capacity = 0;
            exact = true;
        }
    }
    a.c_rp = C->row_ptr;
    // C's pieces are live from here: every error return frees them
    auto failc = [&](slat_status e) {
        (void)hipStreamSynchronize(s);
        slat_csr_free(ctx, C);
        if (wsplit) slat_dev_free(ctx, wsplit, s);
        return e;
    };
#define SLAT_HIPC(expr)                                                                            \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            ctx->err = std::string(#expr) + ": " + hipGetErrorString(e_);                          \
            return failc(SLAT_EHIP);                                                               \
        }                                                                                          \
    } while (0)

    hc.mark(4);
    hipError_t e;
    const bool run_tiny = tiny && !exact;
    const bool run_lane = lane && !exact;
    if (run_tiny) {
        // the whole call in one kernel: a wave per row, every block resident (<= 1024 blocks of
        // <= 30 KB LDS), block offsets by look-back; it stores the completion word itself
        a.c_col = C->col_idx;
        a.c_val = C->values;
        a.seq = ++ctx->done_seq;
        a.done = ctx->d_done;
        const uint64_t g = row_blocks;
        if ((st = ensure_status(ctx, g, s))) return failc(st);
        const uint32_t epoch = slat_next_scan_epoch(ctx, s);
        SLAT_HIPC(slat_launch_tiny(sem, dim3((unsigned)g), num_lds, s, a, ctx->d_status, epoch, ctx->d_maxw));
        hc.mark(5);
        hc.mark(6);
        SLAT_HIPC(wait_stream(ctx, s, a.seq));
    } else if (run_lane) {
        // the whole call in one kernel, a row per lane, a wave's 64 rows per block; block offsets by
        // look-back; it stores the completion word itself (timing: the kernel is the "numeric" pass)
        a.c_col = C->col_idx;
        a.c_val = C->values;
        a.seq = ++ctx->done_seq;
        a.done = ctx->d_done;
        const uint64_t g = (n + slat_lane_rows() - 1) / slat_lane_rows();
        if ((st = ensure_status(ctx, g, s))) return failc(st);
        const uint32_t epoch = slat_next_scan_epoch(ctx, s);
        if (timing)
            for (int i = 0; i < 3; ++i) SLAT_HIPC(hipEventRecord(ctx->ev[i], s));
        if (SLAT_PHASES) SLAT_HIPC(hipMemsetAsync(a.shards, 0, shards_b, s));
        SLAT_HIPC(slat_launch_lane(sem, dim3((unsigned)g), s, a, ctx->d_status, epoch, ctx->d_maxw));
        if (timing) SLAT_HIPC(hipEventRecord(ctx->ev[3], s));
        hc.mark(5);
        hc.mark(6);
        SLAT_HIPC(wait_stream(ctx, s, a.seq));
        if (ctx->h_out[3]) {
            ctx->lane_miss[ctx->lane_miss_next++ % 8] = {A->row_ptr, A->col_idx, B->row_ptr, B->col_idx, A->nnz,
                                                         B->nnz,     A->n_rows,   row_begin, row_end};
            // a row of more than slat_lane_cap() products: the call through the pipeline
            (void)failc(SLAT_OK);
            return rowblock_impl(ctx, A, row_begin, row_end, B, prep, C, flags | SLAT_FLAG_NO_TINY);
        }
    } else {
    if (a.stats || SLAT_PHASES) SLAT_HIPC(hipMemsetAsync(a.shards, 0, shards_b, s));
    asym.counts = a.counts;
    asym.shards = a.shards;
    asym.c_rp = a.c_rp;
    asym.ell_wq = a.ell_wq;
    asym.ell_col = a.ell_col;
    asym.ell_val = a.ell_val;
    asym.ell_ng = a.ell_ng;
    asym.sbm = a.sbm;
    asym.smask = a.smask;
    asym.nblk = a.nblk;
    asym.wsplit = a.wsplit;
    asym.wsplit_abs = a.wsplit_abs;
    asym.wnch1 = a.wnch1;
    slat::FatArgs fat_args = {};
    slat::FatArgs *fa = &fat_args;
    if (fat) {
        if ((st = slat_fat_select(ctx, a, ws + o_fat, fat_min, fa))) return failc(st);
        fa->buckets = (flags & SLAT_FLAG_FAT_BUCKETS) ? 1u : 0u;
        fa->split_abs = B->nnz < 0xFFFFFFFFull ? 1u : 0u;  // absolute offsets fit the split table's u32
        asym.fr_mark = a.fr_mark;
    }
    if (ablate & 7u) {
        // experiments only: an ablated symbolic pass into scratch counts, timed, then discarded
        Args abl = asym;
        abl.ablate = ablate;
        abl.counts = (uint64_t *)(ws + o_abl);
        abl.c_rp = abl.counts;  // row_ptr[0] store lands in scratch too
        SLAT_HIPC(hipEventRecord(ctx->ev[4], s));
        SLAT_HIPC(slat_launch_symbolic(0, idx32, ell, sym_grid, sym_lds, s, abl));
        SLAT_HIPC(hipEventRecord(ctx->ev[5], s));
    }
    // work distribution (tickets in d_words[5]): the rows of the wide launches' window / one-row-hash
    // passes (long, uneven rows: R-MAT 2^16 A^2 18.0 -> 15.3 ms); the single-window pass and the
    // short-row tiles keep a fixed stride (tickets measured slower there).
    // SLAT_DYN=0: no tickets (A/B knob)
    static const uint32_t kDyn = [] {
        const char *e = slat_ab_knob("SLAT_DYN");
        return e ? (uint32_t)std::atoi(e) : 2u;
    }();
    unsigned long long *tq = ctx->d_words + 5;
    // the call's last kernel stores the completion word itself unless fat rows or the stats copy
    // follow (SLAT_NO_FUSED_SIGNAL: a k_signal launch after it, A/B)
    static const bool kFusedSignal = slat_ab_knob("SLAT_NO_FUSED_SIGNAL") == nullptr;
    const bool fused = kFusedSignal && !fat && !a.stats && wait_mode() == 0;
    spec = spec && fused;  // (the short numeric kernel then ends the call)
    uint32_t sym_blocks = sym_grid.x;  // blocks of the symbolic launch whose maxima the scan reduces
    if (timing) SLAT_HIPC(hipEventRecord(ctx->ev[0], s));
    if (fat && (st = slat_fat_symbolic(ctx, *fa, asym, idx32))) return failc(st);
    unsigned int *list_next = nullptr;  // (batched wide launches) the word the scan zeroes for the next call
    if (sym_batched) {
        // MAGNUS categorisation: the short rows batched in hash tables (k_symbolic_short bounds each
        // row's products per tile, listing the rest), then the listed rows by windows
        // the lists' lengths: context words that are zero when the call starts, no memset launch:
        // the symbolic list in one of two words alternating by call (the scan of this call zeroes
        // the other one for the next call), the numeric list's word zeroed by k_symbolic_short's
        // block 0. A call that stopped between its symbolic launch and its scan leaves the words
        // dirty: the next one clears them first
        unsigned int *lc = nullptr;
        if (!all_short) {
            if (ctx->lists_dirty) SLAT_HIPC(hipMemsetAsync(ctx->d_words + 8, 0, 4 * 8, s));
            lc = (unsigned int *)(ctx->d_words + 8 + 2 * (ctx->list_parity & 1u));
            list_next = (unsigned int *)(ctx->d_words + 8 + 2 * ((ctx->list_parity + 1) & 1u));
            ++ctx->list_parity;
            ctx->lists_dirty = true;
        }
        Args h1 = asym, h2 = asym;
        h1.list_reset = all_short ? nullptr : (unsigned int *)(ctx->d_words + 12);
        h1.cbits = a.cbits;
        h1.list = h2.list = all_short ? nullptr : (uint32_t *)(ws + o_l1);
        h1.list_cnt = h2.list_cnt = lc;
        const uint64_t trows = h1.tile_rows ? h1.tile_rows : kWave;
        // (at most 10 blocks per CU, ~1.7 rounds of the 6 resident: C4 1.288 -> 1.272 ms against 16,
        // one eighth and R-MAT 2^16 A^2 within 1 %, profiles/r06_short_bpc_sweep.txt; SLAT_SHORT_BPC: A/B)
        static const uint64_t kShortBpc = [] {
            const char *e = slat_ab_knob("SLAT_SHORT_BPC");
            return e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) : 10ull;
        }();
        const dim3 g1((unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + trows - 1) / trows / wpb + 1, ctx->cu_count * kShortBpc)));
        if (spec) h1.spec_flag = ctx->h_out_dev + 3;
        SLAT_HIPC(slat_launch_symbolic_short(idx32, ell, g1, wpb * sym_short_bytes(), s, h1));
        h2.tq = (kDyn & 2u) && asym.wide ? tq : nullptr;  // (single-window rows: a fixed stride)
        if (all_short || spec) {
            // (no listed rows, or none expected: spec)
        } else {
            // the listed rows take tickets in wide launches, so a resident grid covers any list (the
            // launch is mostly its dispatch when the list is short: C4 lists none, and 4 096 blocks
            // took 4.8 us to dispatch)
            dim3 g2 = sym_grid;
            if (h2.tq)
                g2.x = (unsigned)std::min<uint64_t>(g2.x, (uint64_t)ctx->cu_count *
                                                              slat_symbolic_listed_blocks_per_cu(idx32, ell, sym_lds));
            SLAT_HIPC(slat_launch_symbolic(2, idx32, ell, g2, sym_lds, s, h2));
        }
        a.list = all_short ? nullptr : (uint32_t *)(ws + o_l2);  // the numeric pass's window rows
        a.list_cnt = all_short ? nullptr : (unsigned int *)(ctx->d_words + 12);
    } else if (hash) {
        Args h1 = asym;
        h1.tq = (kDyn & 2u) ? tq : nullptr;
        SLAT_HIPC(slat_launch_symbolic(1, idx32, ell, sym_grid, sym_hash_lds, s, h1));
        SLAT_HIPC(slat_launch_symbolic(2, idx32, ell, sym_grid, sym_lds, s, h1));
    } else {
        // single-window launch without fat rows: symbolic leaves per-block max row counts for the
        // scan's last tile (<= 16 per scan thread)
        if (!fat && sym_grid.x <= 16u * kScanThreads) asym.bmax = (uint32_t *)(ws + o_bmax);
        if (win_mode == 4)  // the stored-bitmap pair: symbolic MODE 4 (spgemm_stored.hpp)
            SLAT_HIPC(slat_launch_symbolic(4, idx32, ell, sym_grid, (size_t)wpb * sym_stored_words(asym.ww) * 4, s, asym));
        else
            SLAT_HIPC(slat_launch_symbolic(0, idx32, ell, sym_grid, sym_lds, s, asym));
    }
    hc.mark(5);
    if (timing) SLAT_HIPC(hipEventRecord(ctx->ev[1], s));
    // (u32 / Sat64 with the ELL copy: the scan also reduces k_build_ell's B-value partials for numeric)
    const bool bpart = bell && dt != SLAT_F64;
    if ((st = slat_launch_scan(ctx, a.counts, n, C->row_ptr, s,
                               bpart ? (const unsigned long long *)(ws + o_part) : nullptr,
                               bpart ? build_ell_blocks(B, a.ell_wq) : 0u, a.epoch, asym.bmax, sym_blocks, list_next)))
        return failc(st);
    if (list_next) ctx->lists_dirty = false;  // the next call's symbolic list word is zeroed in the stream
    if (timing) SLAT_HIPC(hipEventRecord(ctx->ev[2], s));

    if (exact) {
        SLAT_HIPC(hipStreamSynchronize(s));
        const uint64_t total = ctx->h_out[0];
        C->capacity = std::max<uint64_t>(total, 1);
        if (slat_dev_alloc(ctx, (void **)&C->col_idx, C->capacity * 4, s) != hipSuccess ||
            slat_dev_alloc(ctx, &C->values, C->capacity * vs, s) != hipSuccess) {
            (void)hipGetLastError();
            return failc(fail(ctx, SLAT_EOOM, "C allocation failed"));
        }
        if (timing) SLAT_HIPC(hipEventRecord(ctx->ev[2], s));
    }
    a.c_col = C->col_idx;
    a.c_val = C->values;
    auto launch_num = [&](const Args &x) { return slat_launch_numeric(sem, win_mode, idx32, ell, grid, num_lds, s, x); };
    if (ablate & ~7u) {
        // experiments only: an ablated numeric pass (writes stay inside C's row slices), timed;
        // the real numeric pass below overwrites everything it wrote
        Args abl = a;
        abl.ablate = ablate;
        abl.counts = (uint64_t *)(ws + o_abl);
        SLAT_HIPC(hipEventRecord(ctx->ev[4], s));
        SLAT_HIPC(launch_num(abl));
        SLAT_HIPC(hipEventRecord(ctx->ev[5], s));
    }
    if (hash) {
        Args h1 = a;
        if (!batched) a.list = h1.list = nullptr;  // f64: MODE 1 does not list; MODE 2 tests each row
        h1.tq = (kDyn & 2u) && hash_mode != 3 ? tq : nullptr;
        if ((all_short || spec) && fused) {
            a.seq = h1.seq = ++ctx->done_seq;
            h1.done = ctx->d_done;
        }
        if (spec) h1.spec_flag = ctx->h_out_dev + 3;
        SLAT_HIPC(slat_launch_numeric(sem, hash_mode, idx32, ell, hash_grid, hash_lds, s, h1));
    }
    a.tq = (kDyn & 2u) && hash && a.wide ? tq : nullptr;  // (single-window rows: a fixed stride)
    if (fused && !all_short && !spec) {
        a.seq = ++ctx->done_seq;
        a.done = ctx->d_done;
    }
    if (!all_short && !spec) SLAT_HIPC(launch_num(a));
    if (wsplit) slat_dev_free(ctx, wsplit, s);  // stream-ordered: reused only by later work
    if (fat && (st = slat_fat_numeric(ctx, *fa, a, dt, f64any, idx32))) return failc(st);
    if (timing) SLAT_HIPC(hipEventRecord(ctx->ev[3], s));
    if (a.stats) SLAT_HIPC(hipMemcpyAsync(ctx->h_shards, a.shards, sizeof(unsigned long long) * kShards * kShardStride,
                                             hipMemcpyDeviceToHost, s));
    hc.mark(6);
    SLAT_HIPC(wait_stream(ctx, s, a.seq));
    if (spec && ctx->h_out[3]) {
        // a short-row kernel listed a row: this call is void; again with the listed-row launches
        ctx->list_miss[ctx->list_miss_next++ % 8] = {A->row_ptr, A->col_idx, B->row_ptr, B->col_idx, A->nnz,
                                                     B->nnz,     A->n_rows,   row_begin, row_end};
        (void)failc(SLAT_OK);
        const slat_status rs = rowblock_impl(ctx, A, row_begin, row_end, B, prep, C, flags | kFlagNoSpec);
        if (rs == SLAT_OK) ctx->stats.mode |= 64u;
        return rs;
    }
    }  // regular pipeline
#undef SLAT_HIPC
    hc.mark(7);
    if (SLAT_PHASES) {
        // diagnostic build: per-phase cycles of the numeric kernel, summed over waves
        unsigned long long ph[kPhaseSlots * 64];
        SLAT_HIP(ctx, hipMemcpy(ph, a.shards + 512, sizeof ph, hipMemcpyDeviceToHost));
        double tot[kPhaseSlots] = {};
        for (int sh = 0; sh < 64; ++sh)
            for (int i = 0; i < kPhaseSlots; ++i) tot[i] += (double)ph[sh * kPhaseSlots + i];
        std::fprintf(stderr, "phases(rows=%.0f):", tot[kPhaseSlots - 1]);
        for (int i = 0; i < kPhaseSlots - 1; ++i)
            std::fprintf(stderr, " %d:%.0f", i, tot[i] / std::max(1.0, tot[kPhaseSlots - 1]));
        std::fprintf(stderr, "\n");
    }
    // totals from the mapped host words (k_scan_rows: nnz, max row; k_numeric: rows with zeros)
    uint64_t maxrow = ctx->h_out[1], drops = ctx->h_out[2], flops = 0;
    if (a.stats)
        for (int i = 0; i < kShards; ++i) flops += ctx->h_shards[i * kShardStride + 3];
    const uint64_t nnz0 = ctx->h_out[0];
    uint64_t nnz = nnz0;
    double compact_ms = 0;
    if (drops) {
        // exact zeros were dropped: rebuild row_ptr from the per-row actual counts and move rows
        uint64_t *nrp = nullptr;
        SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&nrp, (n + 1) * 8, s));
        if ((st = slat_launch_scan(ctx, a.counts, n, nrp, s))) return st;
        SLAT_HIP(ctx, hipStreamSynchronize(s));
        const uint64_t total = ctx->h_out[0];
        maxrow = ctx->h_out[1];
        uint32_t *ncol = nullptr;
        void *nval = nullptr;
        SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&ncol, std::max<uint64_t>(total, 1) * 4, s));
        SLAT_HIP(ctx, slat_dev_alloc(ctx, &nval, std::max<uint64_t>(total, 1) * vs, s));
        if (timing) SLAT_HIP(ctx, hipEventRecord(ctx->ev[4], s));
        if (dt == SLAT_U32)
            e = launch_compact<SemU32>(sym_grid, s, C->row_ptr, nrp, n, C->col_idx, C->values, ncol, nval);
        else if (dt == SLAT_SAT64)
            e = launch_compact<SemSat64>(sym_grid, s, C->row_ptr, nrp, n, C->col_idx, C->values, ncol, nval);
        else
            e = launch_compact<SemF64>(sym_grid, s, C->row_ptr, nrp, n, C->col_idx, C->values, ncol, nval);
        SLAT_HIP(ctx, e);
        if (timing) SLAT_HIP(ctx, hipEventRecord(ctx->ev[5], s));
        slat_csr old = *C;
        (void)slat_csr_free(ctx, &old);
        SLAT_HIP(ctx, hipStreamSynchronize(s));
        C->row_ptr = nrp;
        C->col_idx = ncol;
        C->values = nval;
        C->alloc = kAllocSeparate;
        C->capacity = std::max<uint64_t>(total, 1);
        nnz = total;
        if (timing) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, ctx->ev[4], ctx->ev[5]);
            compact_ms = ms;
        }
    }
    C->nnz = nnz;
    C->max_row_nnz = maxrow;
    if (C->capacity > nnz) {
        // trim the bound-sized arrays to nnz(C): the tails serve later allocations of the context
        slat_dev_shrink(ctx, C->col_idx, std::max<uint64_t>(nnz, 1) * 4);
        slat_dev_shrink(ctx, C->values, std::max<uint64_t>(nnz, 1) * vs);
        C->capacity = std::max<uint64_t>(nnz, 1);
    }

    slat_stats &S = ctx->stats;
    S.nnz = nnz;
    S.flops = flops;
    S.capacity = C->capacity;
    S.mode = (idx32 ? 1u : 0u) | (ell ? 2u : 0u) | (run_tiny ? 4u : 0u) | (run_lane ? 8u : 0u) |
             (!run_tiny && !run_lane && win_mode == 4 ? 16u : 0u) | (!run_tiny && !run_lane && spec ? 32u : 0u);
    S.window_words = a.ww;
    S.exact_alloc = exact ? 1u : 0u;
    S.dropped_rows = (uint32_t)drops;
    if (timing) {
        float ms = 0;
        SLAT_HIP(ctx, hipEventSynchronize(ctx->ev[3]));  // the wait above does not tell the runtime
        (void)hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]);
        S.symbolic_ms = ms;
        (void)hipEventElapsedTime(&ms, ctx->ev[1], ctx->ev[2]);
        S.scan_ms = ms;
        (void)hipEventElapsedTime(&ms, ctx->ev[2], ctx->ev[3]);
        S.numeric_ms = ms;
        S.compact_ms = compact_ms;
        if (ablate) {
            (void)hipEventElapsedTime(&ms, ctx->ev[4], ctx->ev[5]);
            S.compact_ms = ms;  // experiments only: the ablated pass
        }
        (void)hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[3]);
        S.total_ms = ms + compact_ms;
    }
    if (progress) {  // the reference's pass summaries (rows of this call)
        const double rows = (double)n, ts = S.symbolic_ms * 1e-3, tn = (S.numeric_ms + S.compact_ms) * 1e-3;
        std::fprintf(stderr, "\r  symbolic: done in %.1fs (%.0f rows/s)                    \n", ts, rows / std::max(ts, 1e-9));
        std::fprintf(stderr, "\r  numeric:  done in %.1fs (%.0f rows/s)                    \n", tn, rows / std::max(tn, 1e-9));
    }
    hc.mark(8);
    return SLAT_OK;
}

extern "C" slat_status slat_spgemm(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B, slat_csr *C,
                                   uint32_t flags) {
    if (!ctx || !A) return SLAT_EINVAL;
    return slat_spgemm_rowblock(ctx, A, 0, A->n_rows, B, C, flags);
}

static slat_status typed(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B, slat_csr *C, uint32_t flags,
                         int32_t dt) {
    if (!ctx || !A || !B) return SLAT_EINVAL;
    if (A->dtype != dt || B->dtype != dt) return fail(ctx, SLAT_EINVAL, "value type does not match the entry point");
    return slat_spgemm(ctx, A, B, C, flags);
}

extern "C" slat_status slat_spgemm_csr_u32(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B, slat_csr *C,
                                           uint32_t flags) {
    return typed(ctx, A, B, C, flags, SLAT_U32);
}
extern "C" slat_status slat_spgemm_csr_sat64(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B,
                                             slat_csr *C, uint32_t flags) {
    return typed(ctx, A, B, C, flags, SLAT_SAT64);
}
extern "C" slat_status slat_spgemm_csr_f64(slat_ctx *ctx, const slat_csr_view *A, const slat_csr_view *B, slat_csr *C,
                                           uint32_t flags) {
    return typed(ctx, A, B, C, flags, SLAT_F64);
}

// ---------------------------------------------------------------------------------------------
// A prepared right operand: B's padded ELL image and its clamped value summary, built once for many
// products with the same B (the replicated B of the multi-GPU row blocks, an A^k chain's A)
// ---------------------------------------------------------------------------------------------
extern "C" slat_status slat_bprep_create(slat_ctx *ctx, const slat_csr_view *B, slat_bprep **out) {
    if (!ctx || !out) return SLAT_EINVAL;
    *out = nullptr;
    slat_status st = slat_check_view(ctx, B, "B");
    if (st) return st;
    if (B->residency != SLAT_DEVICE) return fail(ctx, SLAT_EINVAL, "a prepared B must be device-resident");
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    slat_bprep *p = new slat_bprep();
    p->b = *B;
    p->device = ctx->device;
    p->owner = ctx;
    uint64_t mr = B->max_row_nnz;
    if (mr == 0 && B->n_rows && (st = slat_csr_max_row_nnz(ctx, B, &mr))) {
        delete p;
        return st;
    }
    p->maxrow_b = mr;
    p->b.max_row_nnz = mr;
    const size_t vs = vsize(B->dtype);
    p->wq = (uint32_t)((mr + 3) / 4);
    p->ell = mr > 0 && B->nnz > 0 && ell_fits(B, mr, vs);
    if (p->ell) {
        hipStream_t s = ctx->stream;
        const uint32_t nparts = build_ell_blocks(B, p->wq);
        unsigned long long *parts = nullptr;
        hipError_t e = slat_dev_alloc(ctx, (void **)&p->ecol, B->n_rows * p->wq * 16, s);
        if (e == hipSuccess) e = slat_dev_alloc(ctx, &p->eval, B->n_rows * p->wq * 4 * vs, s);
        if (e == hipSuccess) e = slat_dev_alloc(ctx, (void **)&p->eng, B->n_rows, s);
        if (e == hipSuccess) e = slat_dev_alloc(ctx, (void **)&p->vmax, 64, s);
        if (e == hipSuccess && B->dtype != SLAT_F64) e = slat_dev_alloc(ctx, (void **)&parts, (size_t)nparts * 8, s);
        if (e == hipSuccess) {
            if (B->dtype == SLAT_U32)
                e = launch_build_ell<uint32_t>(s, B, p->wq, p->ecol, p->eval, p->eng, parts);
            else if (B->dtype == SLAT_SAT64)
                e = launch_build_ell<unsigned long long>(s, B, p->wq, p->ecol, p->eval, p->eng, parts);
            else
                e = launch_build_ell<double>(s, B, p->wq, p->ecol, p->eval, p->eng, nullptr);
        }
        p->epoch = 1;
        if (e == hipSuccess && parts) {
            hipLaunchKernelGGL(k_reduce_bparts, dim3(1), dim3(kWave), 0, s, parts, nparts, p->vmax, p->epoch);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (parts) slat_dev_free(ctx, parts, s);
        if (e != hipSuccess) {
            ctx->err = std::string("slat_bprep_create: ") + hipGetErrorString(e);
            (void)slat_bprep_free(ctx, p);
            return SLAT_EHIP;
        }
    }
    *out = p;
    return SLAT_OK;
}

extern "C" slat_status slat_bprep_free(slat_ctx *ctx, slat_bprep *p) {
    if (!ctx) return SLAT_EINVAL;
    if (!p) return SLAT_OK;
    (void)hipSetDevice(ctx->device);
    for (void *q : {(void *)p->ecol, p->eval, (void *)p->eng, (void *)p->vmax})
        if (q) slat_dev_free(ctx, q, ctx->stream);
    delete p;
    return SLAT_OK;
}
