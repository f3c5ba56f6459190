// slat_coo.hip — the reference's matrix constructors on the device:
//   slat_csr_from_coo  CsrMatrix::from_coo  src/graph_csr.rs:83-129
//   slat_csr_lattice   CsrMatrix::lattice   src/graph_csr.rs:177-222
//   slat_csr_thin      CsrMatrix::thin      src/graph_csr.rs:225-247
// so a 100^3+ input never round-trips through host memory. from_coo: 64-bit (row, column) keys
// radix-sorted with their triplet index (stable: duplicates keep input order), run heads flagged
// and scanned, each run summed by its head (u32 / u64 wrapping like the reference's release
// build, f64 in input order), zeros dropped by a second scan, rows counted and scanned into
// row_ptr. thin: draw k of the reference's row-major scan is keystream words 2k, 2k+1 of ChaCha12
// (u64 draws only, so never split across refills), hence every draw is computed independently.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>
#include <hipcub/hipcub.hpp>

#include "slat.h"
#include "slat_internal.hpp"

namespace {

constexpr int kB = 256;

dim3 grid_for(const slat_ctx *ctx, uint64_t items) {
    const uint64_t blocks = (items + kB - 1) / kB;
    return dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)ctx->cu_count * 8)));
}

// value bits of a triplet (u32 zero-extended, u64 / f64 as bits)
__device__ __forceinline__ uint64_t load_bits(const void *v, uint64_t i, int dt) {
    return dt == SLAT_U32 ? (uint64_t)((const uint32_t *)v)[i] : ((const uint64_t *)v)[i];
}
__device__ __forceinline__ uint64_t add_bits(uint64_t a, uint64_t b, int dt) {
    if (dt == SLAT_F64) return __double_as_longlong(__dadd_rn(__longlong_as_double(a), __longlong_as_double(b)));
    if (dt == SLAT_U32) return (uint32_t)(a + b);  // `+=` on u32 wraps in a release build
    return a + b;
}
__device__ __forceinline__ bool zero_bits(uint64_t v, int dt) {
    return dt == SLAT_F64 ? __longlong_as_double(v) == 0.0 : v == 0;
}

// keys = row << 32 | col, idx = i; rows >= n or cols >= n set *bad (and sort last as row n), except
// row 0xFFFFFFFF when `skip` (generator slots that hold no triplet)
__global__ void k_coo_keys(const uint32_t *rows, const uint32_t *cols, uint64_t nt, uint64_t n, uint64_t *keys,
                           uint32_t *idx, unsigned long long *bad, int skip) {
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < nt; i += (uint64_t)gridDim.x * kB) {
        const uint32_t r = rows[i], c = cols[i];
        const bool ok = r < n && c < n;
        if (!ok && !(skip && r == 0xFFFFFFFFu)) __hip_atomic_store(bad, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        keys[i] = ok ? ((uint64_t)r << 32) | c : (uint64_t)n << 32;
        idx[i] = (uint32_t)i;
    }
}

// run heads of the sorted keys (entries of row n, the invalid or skipped ones, are no run)
__global__ void k_coo_heads(const uint64_t *keys, uint64_t nt, uint64_t n, uint64_t *head) {
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < nt; i += (uint64_t)gridDim.x * kB)
        head[i] = (keys[i] >> 32) < n && (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

// every head sums its run in sorted (= input) order; keep = the sum is not zero
__global__ void k_coo_runs(const uint64_t *keys, const uint32_t *idx, const void *vals, int dt, uint64_t nt,
                           const uint64_t *head, const uint64_t *upos, uint64_t *ukey, uint64_t *uval,
                           uint64_t *keep, int keep_zeros) {
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < nt; i += (uint64_t)gridDim.x * kB) {
        if (!head[i]) continue;
        const uint64_t k = keys[i];
        uint64_t v = load_bits(vals, idx[i], dt);
        for (uint64_t j = i + 1; j < nt && keys[j] == k; ++j) v = add_bits(v, load_bits(vals, idx[j], dt), dt);
        const uint64_t u = upos[i];
        if (u >= nt) continue;  // never write outside the run arrays (a scan gone wrong stays a wrong result)
        ukey[u] = k;
        uval[u] = v;
        keep[u] = keep_zeros || !zero_bits(v, dt) ? 1u : 0u;
    }
}

__global__ void k_coo_emit(const uint64_t *ukey, const uint64_t *uval, const uint64_t *keep, const uint64_t *fpos,
                           uint64_t nu, uint64_t nnz, uint64_t n, int dt, uint32_t *col, void *val,
                           unsigned long long *rowcnt) {
    for (uint64_t u = (uint64_t)blockIdx.x * kB + threadIdx.x; u < nu; u += (uint64_t)gridDim.x * kB) {
        if (!keep[u]) continue;
        const uint64_t f = fpos[u], row = ukey[u] >> 32;
        if (f >= nnz || row >= n) continue;  // bounds of C and of the row counters
        col[f] = (uint32_t)ukey[u];
        if (dt == SLAT_U32)
            ((uint32_t *)val)[f] = (uint32_t)uval[u];
        else
            ((uint64_t *)val)[f] = uval[u];
        atomicAdd(&rowcnt[row], 1ull);
    }
}

// CsrMatrix::lattice triplets: (node, offset) -> neighbor, row-major strides, base-3 offsets with
// dimension 0 least significant, self excluded, torus wrap or out-of-range dropped (-> row n)
struct LatDims {
    uint64_t dims[8], strides[8];
    int ndim;
};
__global__ void k_lattice(LatDims L, int torus, uint64_t total, uint64_t nnb, uint32_t *rows, uint32_t *cols) {
    const uint64_t nt = total * nnb;
    for (uint64_t t = (uint64_t)blockIdx.x * kB + threadIdx.x; t < nt; t += (uint64_t)gridDim.x * kB) {
        const uint64_t node = t / nnb, off = t - node * nnb;
        uint64_t tmp = off, rem = node, neighbor = 0;
        bool all_zero = true, valid = true;
        for (int d = 0; d < L.ndim; ++d) {
            const int64_t delta = (int64_t)(tmp % 3) - 1;
            tmp /= 3;
            if (delta != 0) all_zero = false;
            const uint64_t coord = (rem / L.strides[d]) % L.dims[d];
            int64_t c = (int64_t)coord + delta;
            const int64_t m = (int64_t)L.dims[d];
            if (torus) {
                c = ((c % m) + m) % m;
            } else if (c < 0 || c >= m) {
                valid = false;
            }
            neighbor += (uint64_t)(c < 0 ? 0 : c) * L.strides[d];
        }
        const bool ok = valid && !all_zero;
        rows[t] = ok ? (uint32_t)node : 0xFFFFFFFFu;  // dropped: no row (k_coo_keys maps it past row n)
        cols[t] = ok ? (uint32_t)neighbor : 0u;
    }
}

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
// keystream words w, w+1 (w even, never across a 16-word block) of ChaCha12 with `key`, stream 0
__device__ uint64_t chacha12_u64(const uint32_t *key, uint64_t w) {
    const uint64_t ctr = w >> 4;
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                      key[4], key[5], key[6], key[7], (uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u};
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = s[i];
    auto qr = [&](int a, int b, int c, int d) {
        x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16);
        x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12);
        x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8);
        x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7);
    };
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
    }
    const int o = (int)(w & 15);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 16; i += 2)
        if (i == o) {
            lo = x[i] + s[i];
            hi = x[i + 1] + s[i + 1];
        }
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

struct Key8 {
    uint32_t k[8];
};

__device__ __forceinline__ uint64_t row_of(const uint64_t *rp, uint64_t n, uint64_t i) {
    uint64_t lo = 0, hi = n;  // last row r with rp[r] <= i
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (rp[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ bool find_entry(const uint64_t *rp, const uint32_t *col, uint64_t r, uint32_t c, uint64_t *at) {
    uint64_t lo = rp[r], hi = rp[r + 1];
    const uint64_t end = hi;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (col[mid] < c) lo = mid + 1; else hi = mid;
    }
    *at = lo;
    return lo < end && col[lo] == c;
}

// thin, pass 1: an entry draws iff r <= c (the `&&` short-circuit of src/graph_csr.rs:235)
__global__ void k_thin_need(const uint64_t *rp, const uint32_t *col, uint64_t n, uint64_t nnz, uint64_t *need) {
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < nnz; i += (uint64_t)gridDim.x * kB)
        need[i] = row_of(rp, n, i) <= col[i] ? 1u : 0u;
}
// pass 2: draw d = dpos[i] -> keep (r,c,v) and the mirror (c,r,get(c,r)) when present and r != c
__global__ void k_thin_keep(const uint64_t *rp, const uint32_t *col, const void *val, int dt, uint64_t n,
                            uint64_t nnz, const uint64_t *need, const uint64_t *dpos, Key8 key, uint64_t w0,
                            double density, uint64_t *emit) {
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < nnz; i += (uint64_t)gridDim.x * kB) {
        uint64_t e = 0;
        if (need[i]) {
            const double x = (double)(chacha12_u64(key.k, w0 + 2 * dpos[i]) >> 12) * (1.0 / 4503599627370496.0);
            if (x < density) {
                e = 1;
                const uint64_t r = row_of(rp, n, i);
                uint64_t at;
                if (r != col[i] && find_entry(rp, col, col[i], (uint32_t)r, &at) && !zero_bits(load_bits(val, at, dt), dt))
                    e = 2;  // `if rev > 0` (stored values are non-zero)
            }
        }
        emit[i] = e;
    }
}
__global__ void k_thin_emit(const uint64_t *rp, const uint32_t *col, const void *val, int dt, uint64_t n,
                            uint64_t nnz, const uint64_t *emit, const uint64_t *epos, uint32_t *trow, uint32_t *tcol,
                            uint64_t *tval) {
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < nnz; i += (uint64_t)gridDim.x * kB) {
        if (!emit[i]) continue;
        const uint64_t r = row_of(rp, n, i), p = epos[i];
        if (p + emit[i] > 2 * nnz) continue;  // the triplet buffers hold 2 per entry
        trow[p] = (uint32_t)r;
        tcol[p] = col[i];
        tval[p] = load_bits(val, i, dt);
        if (emit[i] == 2) {
            uint64_t at;
            (void)find_entry(rp, col, col[i], (uint32_t)r, &at);
            trow[p + 1] = col[i];
            tcol[p + 1] = (uint32_t)r;
            tval[p + 1] = load_bits(val, at, dt);
        }
    }
}

// u64 value bits -> the dtype's array (u32 narrows)
__global__ void k_narrow_u32(const uint64_t *in, uint64_t n, uint32_t *out) {
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kB) out[i] = (uint32_t)in[i];
}

struct Buf {
    slat_ctx *ctx;
    void *p = nullptr;
    hipError_t alloc(size_t bytes) { return slat_dev_alloc(ctx, &p, bytes, ctx->stream); }
    ~Buf() {
        if (p) slat_dev_free(ctx, p, ctx->stream);
    }
};

// the scan of `cnt` u64 flags/counts (n items) into pos[0..n] on the stream, then the total
slat_status scan_total(slat_ctx *ctx, const uint64_t *cnt, uint64_t n, uint64_t *pos, uint64_t *total) {
    slat_status st = slat_launch_scan(ctx, cnt, n, pos, ctx->stream);
    if (st) return st;
    SLAT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *total = ctx->h_out[0];
    return SLAT_OK;
}

// from_coo core over device triplets (rows, cols, value bits `vals` of dtype dt: u32 or u64 words)
slat_status from_coo_dev(slat_ctx *ctx, uint64_t n, uint64_t nt, const uint32_t *rows, const uint32_t *cols,
                         const void *vals, int32_t dt, slat_csr *out, int skip = 0, int keep_zeros = 0) {
    hipStream_t s = ctx->stream;
    std::memset(out, 0, sizeof *out);
    out->n_rows = out->n_cols = n;
    out->dtype = dt;
    out->device = ctx->device;
    const size_t vs = vsize(dt);
    if (nt == 0) {
        SLAT_HIP(ctx, alloc_joint(ctx, out, n, 0, vs, s));
        SLAT_HIP(ctx, hipMemsetAsync(out->row_ptr, 0, (n + 1) * 8, s));
        SLAT_HIP(ctx, hipStreamSynchronize(s));
        return SLAT_OK;
    }
    // scratch: keys 2x u64[nt] | idx 2x u32[nt] | head u64[nt] | upos u64[nt+1] | ukey, uval, keep u64[nt]
    //          | fpos u64[nt+1] | rowcnt u64[n] | sort temp
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    int endbit = 33;
    while (endbit < 64 && ((n + 1) >> (endbit - 32)) != 0) ++endbit;
    // (Round 1 rounded endbit up to whole 8-bit digits after seeing wrong orders above ~3M keys. The
    // cause was the stream-ordered pool's lost writes into a freshly grown block, which the scratch
    // then came from: tools/repro/repro_pool.hip; the sort itself orders partial top digits correctly,
    // tools/repro/repro_radix.cpp.)
    // The sort takes an int item count (hipcub): 2^31 triplets or more would wrap negative.
    if (nt >= 0x7FFFFFFFull) return fail(ctx, SLAT_ENOTSUP, "2^31 or more triplets (the radix sort's int count)");
    size_t sort_b = 0;
    SLAT_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                                     (uint32_t *)nullptr, (uint32_t *)nullptr, (int)nt, 0, endbit, s));
    const size_t o_k2 = up(nt * 8), o_i1 = o_k2 + up(nt * 8), o_i2 = o_i1 + up(nt * 4), o_h = o_i2 + up(nt * 4),
                 o_up = o_h + up(nt * 8), o_uk = o_up + up((nt + 1) * 8), o_uv = o_uk + up(nt * 8),
                 o_kp = o_uv + up(nt * 8), o_fp = o_kp + up(nt * 8), o_rc = o_fp + up((nt + 1) * 8),
                 o_st = o_rc + up(n * 8), total_b = o_st + up(sort_b);
    Buf scratch{ctx};
    if (scratch.alloc(total_b) != hipSuccess) return fail(ctx, SLAT_EOOM, "from_coo scratch");
    uint8_t *w = (uint8_t *)scratch.p;
    uint64_t *k1 = (uint64_t *)w, *k2 = (uint64_t *)(w + o_k2);
    uint32_t *i1 = (uint32_t *)(w + o_i1), *i2 = (uint32_t *)(w + o_i2);
    uint64_t *head = (uint64_t *)(w + o_h), *upos = (uint64_t *)(w + o_up), *ukey = (uint64_t *)(w + o_uk),
             *uval = (uint64_t *)(w + o_uv), *keep = (uint64_t *)(w + o_kp), *fpos = (uint64_t *)(w + o_fp);
    unsigned long long *rowcnt = (unsigned long long *)(w + o_rc);
    ctx->h_out[3] = 0;
    const dim3 g = grid_for(ctx, nt), b(kB);
    hipLaunchKernelGGL(k_coo_keys, g, b, 0, s, rows, cols, nt, n, k1, i1, ctx->h_out_dev + 3, skip);
    SLAT_HIP(ctx, hipGetLastError());
    SLAT_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(w + o_st, sort_b, k1, k2, i1, i2, (int)nt, 0, endbit, s));
    hipLaunchKernelGGL(k_coo_heads, g, b, 0, s, k2, nt, n, head);
    SLAT_HIP(ctx, hipGetLastError());
    uint64_t nu = 0, nnz = 0;
    slat_status st;
    if ((st = scan_total(ctx, head, nt, upos, &nu))) return st;
    if (ctx->h_out[3]) return fail(ctx, SLAT_EINVAL, "from_coo: row or column id >= n");  // the reference panics
    hipLaunchKernelGGL(k_coo_runs, g, b, 0, s, k2, i2, vals, dt, nt, head, upos, ukey, uval, keep, keep_zeros);
    SLAT_HIP(ctx, hipGetLastError());
    if ((st = scan_total(ctx, keep, nu, fpos, &nnz))) return st;
    SLAT_HIP(ctx, alloc_joint(ctx, out, n, nnz, vs, s));
    if (n) SLAT_HIP(ctx, hipMemsetAsync(rowcnt, 0, n * 8, s));
    if (nu) {
        hipLaunchKernelGGL(k_coo_emit, grid_for(ctx, nu), b, 0, s, ukey, uval, keep, fpos, nu, nnz, n, dt,
                           out->col_idx, out->values, rowcnt);
        SLAT_HIP(ctx, hipGetLastError());
    }
    uint64_t tot = 0;
    if ((st = scan_total(ctx, (const uint64_t *)rowcnt, n, out->row_ptr, &tot))) return st;
    out->nnz = nnz;
    out->capacity = std::max<uint64_t>(nnz, 1);
    out->max_row_nnz = ctx->h_out[1];
    return SLAT_OK;
}

}  // namespace

extern "C" slat_status slat_csr_from_coo(slat_ctx *ctx, uint64_t n, uint64_t ntrip, const uint32_t *rows,
                                         const uint32_t *cols, const void *vals, int32_t dtype, int32_t residency,
                                         slat_csr *out) {
    if (!ctx || !out || dtype < SLAT_U32 || dtype > SLAT_F64) return SLAT_EINVAL;
    if (ntrip && (!rows || !cols || !vals)) return fail(ctx, SLAT_EINVAL, "from_coo: null arrays");
    if (n > 0xFFFFFFFFull) return fail(ctx, SLAT_EINVAL, "n exceeds u32 ids");
    if (ntrip >= 0x7FFFFFFFull) return fail(ctx, SLAT_ENOTSUP, "2^31 or more triplets (the radix sort's int count)");
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    if (residency == SLAT_DEVICE) return from_coo_dev(ctx, n, ntrip, rows, cols, vals, dtype, out);
    // host triplets: one staging copy
    Buf stage{ctx};
    const size_t vs = vsize(dtype);
    const size_t bytes = ntrip * (8 + vs) + 64;
    if (stage.alloc(bytes) != hipSuccess) return fail(ctx, SLAT_EOOM, "from_coo staging");
    uint8_t *d = (uint8_t *)stage.p;
    if (ntrip) {
        SLAT_HIP(ctx, hipMemcpyAsync(d, rows, ntrip * 4, hipMemcpyHostToDevice, ctx->stream));
        SLAT_HIP(ctx, hipMemcpyAsync(d + ntrip * 4, cols, ntrip * 4, hipMemcpyHostToDevice, ctx->stream));
        SLAT_HIP(ctx, hipMemcpyAsync(d + ntrip * 8, vals, ntrip * vs, hipMemcpyHostToDevice, ctx->stream));
    }
    return from_coo_dev(ctx, n, ntrip, (const uint32_t *)d, (const uint32_t *)(d + ntrip * 4), d + ntrip * 8, dtype,
                        out);
}

extern "C" slat_status slat_csr_lattice(slat_ctx *ctx, const uint64_t *dims, int ndim, int torus, slat_csr *out) {
    if (!ctx || !out || !dims || ndim < 1 || ndim > 8) return SLAT_EINVAL;
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    LatDims L = {};
    L.ndim = ndim;
    uint64_t total = 1, nnb = 1;
    for (int d = 0; d < ndim; ++d) {
        if (dims[d] == 0) return fail(ctx, SLAT_EINVAL, "lattice: zero dimension");
        L.dims[d] = dims[d];
        total *= dims[d];
        nnb *= 3;
    }
    if (total > 0xFFFFFFFFull) return fail(ctx, SLAT_EINVAL, "lattice: more than 2^32 nodes");
    L.strides[ndim - 1] = 1;
    for (int d = ndim - 2; d >= 0; --d) L.strides[d] = L.strides[d + 1] * dims[d + 1];
    const uint64_t nt = total * nnb;
    Buf trip{ctx};
    if (trip.alloc(nt * 12 + 64) != hipSuccess) return fail(ctx, SLAT_EOOM, "lattice triplets");
    uint32_t *rows = (uint32_t *)trip.p, *cols = rows + nt, *vals = cols + nt;
    hipLaunchKernelGGL(k_lattice, grid_for(ctx, nt), dim3(kB), 0, ctx->stream, L, torus, total, nnb, rows, cols);
    SLAT_HIP(ctx, hipGetLastError());
    SLAT_HIP(ctx, hipMemsetD32Async((hipDeviceptr_t)vals, 1u, nt, ctx->stream));
    // dropped offsets carry row 0xFFFFFFFF: skipped slots, not errors
    return from_coo_dev(ctx, total, nt, rows, cols, vals, SLAT_U32, out, 1);
}

extern "C" slat_status slat_csr_thin(slat_ctx *ctx, const slat_csr_view *m, slat_rng *rng, double density,
                                     slat_csr *out) {
    if (!ctx || !out || !rng) return SLAT_EINVAL;
    slat_status st = slat_check_view(ctx, m, "m");
    if (st) return st;
    if (m->residency != SLAT_DEVICE) return fail(ctx, SLAT_EINVAL, "thin takes a device-resident matrix");
    if (m->n_rows != m->n_cols) return fail(ctx, SLAT_EDIM, "matrix is not square");
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint64_t n = m->n_rows, nnz = m->nnz;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    Buf scratch{ctx};
    const size_t o_dp = up(nnz * 8), o_em = o_dp + up((nnz + 1) * 8), o_ep = o_em + up(nnz * 8),
                 o_tr = o_ep + up((nnz + 1) * 8), o_tc = o_tr + up(2 * nnz * 4), o_tv = o_tc + up(2 * nnz * 4),
                 o_tn = o_tv + up(2 * nnz * 8), total_b = o_tn + up(2 * nnz * 4) + 256;
    if (scratch.alloc(total_b) != hipSuccess) return fail(ctx, SLAT_EOOM, "thin scratch");
    uint8_t *w = (uint8_t *)scratch.p;
    uint64_t *need = (uint64_t *)w, *dpos = (uint64_t *)(w + o_dp), *emit = (uint64_t *)(w + o_em),
             *epos = (uint64_t *)(w + o_ep), *tval = (uint64_t *)(w + o_tv);
    uint32_t *trow = (uint32_t *)(w + o_tr), *tcol = (uint32_t *)(w + o_tc), *tnar = (uint32_t *)(w + o_tn);
    const dim3 g = grid_for(ctx, nnz), b(kB);
    uint64_t draws = 0, ntrip = 0;
    if (nnz) {
        hipLaunchKernelGGL(k_thin_need, g, b, 0, s, m->row_ptr, m->col_idx, n, nnz, need);
        SLAT_HIP(ctx, hipGetLastError());
        if ((st = scan_total(ctx, need, nnz, dpos, &draws))) return st;
        Key8 key;
        uint64_t w0;
        slat_rng_position(rng, key.k, &w0);
        hipLaunchKernelGGL(k_thin_keep, g, b, 0, s, m->row_ptr, m->col_idx, m->values, m->dtype, n, nnz, need, dpos,
                           key, w0, density, emit);
        SLAT_HIP(ctx, hipGetLastError());
        if ((st = scan_total(ctx, emit, nnz, epos, &ntrip))) return st;
        hipLaunchKernelGGL(k_thin_emit, g, b, 0, s, m->row_ptr, m->col_idx, m->values, m->dtype, n, nnz, emit, epos,
                           trow, tcol, tval);
        SLAT_HIP(ctx, hipGetLastError());
        slat_rng_advance(rng, draws);  // the host StdRng is where the reference's would be
    }
    const void *vals = tval;
    if (m->dtype == SLAT_U32 && ntrip) {
        hipLaunchKernelGGL(k_narrow_u32, grid_for(ctx, ntrip), b, 0, s, tval, ntrip, tnar);
        SLAT_HIP(ctx, hipGetLastError());
        vals = tnar;
    }
    return from_coo_dev(ctx, n, ntrip, trow, tcol, vals, m->dtype, out);
}

// ------------------------------------------------------------------------------------------------
// The real-graph path: edge lists to CSR, the RCM order, the symmetric
// permutation and the bandwidth statistics, on the device except the order itself (a sequential
// BFS, computed on the host like the reference's).
// ------------------------------------------------------------------------------------------------
namespace {

__device__ __forceinline__ void flag_bad(unsigned long long *bad) {
    __hip_atomic_store(bad, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// inv[perm[k]] = k; ids >= n flagged
__global__ void k_perm_inverse(const uint32_t *perm, uint64_t n, uint32_t *inv, unsigned long long *bad) {
    for (uint64_t k = (uint64_t)blockIdx.x * kB + threadIdx.x; k < n; k += (uint64_t)gridDim.x * kB) {
        const uint32_t p = perm[k];
        if (p >= n) flag_bad(bad); else inv[p] = (uint32_t)k;
    }
}
// a repeated id leaves inv pointing at only one of its positions
__global__ void k_perm_check(const uint32_t *perm, uint64_t n, const uint32_t *inv, unsigned long long *bad) {
    for (uint64_t k = (uint64_t)blockIdx.x * kB + threadIdx.x; k < n; k += (uint64_t)gridDim.x * kB) {
        const uint32_t p = perm[k];
        if (p < n && inv[p] != (uint32_t)k) flag_bad(bad);
    }
}
// entry i of row r -> (inv[r], inv[col], value bits)
__global__ void k_perm_trip(const uint64_t *rp, const uint32_t *col, const void *val, int dt, uint64_t n,
                            uint64_t nnz, const uint32_t *inv, uint32_t *trow, uint32_t *tcol, uint64_t *tval) {
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < nnz; i += (uint64_t)gridDim.x * kB) {
        trow[i] = inv[row_of(rp, n, i)];
        tcol[i] = inv[col[i]];
        tval[i] = load_bits(val, i, dt);
    }
}
// from_edges / from_edges_undirected (src/graph_csr.rs:132-147): (r, c, 1) then, undirected and
// r != c, (c, r, 1) in the second half (row 0xFFFFFFFF = no triplet); ids >= n flagged
__global__ void k_edges_trip(const uint32_t *src, const uint32_t *dst, uint64_t m, uint64_t n, int undirected,
                             uint32_t *trow, uint32_t *tcol, uint32_t *tval, unsigned long long *bad) {
    for (uint64_t e = (uint64_t)blockIdx.x * kB + threadIdx.x; e < m; e += (uint64_t)gridDim.x * kB) {
        const uint32_t r = src[e], c = dst[e];
        if (r >= n || c >= n) flag_bad(bad);
        trow[e] = r;
        tcol[e] = c;
        tval[e] = 1u;
        if (undirected) {
            trow[m + e] = r != c ? c : 0xFFFFFFFFu;
            tcol[m + e] = r;
            tval[m + e] = 1u;
        }
    }
}
// bandwidth_stats (src/graph_csr.rs:802-818): max and sum of |r - c|
__global__ void k_bandwidth(const uint64_t *rp, const uint32_t *col, uint64_t n, uint64_t nnz,
                            unsigned long long *out) {
    unsigned long long mx = 0, sum = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < nnz; i += (uint64_t)gridDim.x * kB) {
        const uint64_t r = row_of(rp, n, i), c = col[i], d = r > c ? r - c : c - r;
        mx = mx > d ? mx : d;
        sum += d;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long om = __shfl_xor(mx, o), os = __shfl_xor(sum, o);
        mx = mx > om ? mx : om;
        sum += os;
    }
    if ((threadIdx.x & 63) == 0 && (mx || sum)) {
        atomicMax(&out[0], mx);
        atomicAdd(&out[1], sum);
    }
}

// device or host u32 array -> device pointer (staged into `buf` when host)
slat_status device_u32(slat_ctx *ctx, const uint32_t *p, uint64_t count, int32_t residency, Buf &buf,
                       const uint32_t **out) {
    if (residency == SLAT_DEVICE) {
        *out = p;
        return SLAT_OK;
    }
    if (buf.alloc(count * 4 + 64) != hipSuccess) return fail(ctx, SLAT_EOOM, "staging");
    if (count) SLAT_HIP(ctx, hipMemcpyAsync(buf.p, p, count * 4, hipMemcpyHostToDevice, ctx->stream));
    *out = (const uint32_t *)buf.p;
    return SLAT_OK;
}

}  // namespace

extern "C" slat_status slat_csr_permute(slat_ctx *ctx, const slat_csr_view *m, const uint32_t *perm,
                                        int32_t perm_residency, slat_csr *out) {
    if (!ctx || !out || (!perm && m && m->n_rows)) return SLAT_EINVAL;
    slat_status st = slat_check_view(ctx, m, "m");
    if (st) return st;
    if (m->residency != SLAT_DEVICE) return fail(ctx, SLAT_EINVAL, "permute takes a device-resident matrix");
    if (m->n_rows != m->n_cols) return fail(ctx, SLAT_EDIM, "matrix is not square");
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const uint64_t n = m->n_rows, nnz = m->nnz;
    Buf stage{ctx}, scratch{ctx};
    const uint32_t *dperm = nullptr;
    if ((st = device_u32(ctx, perm, n, perm_residency, stage, &dperm))) return st;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_tr = up(std::max<uint64_t>(n, 1) * 4), o_tc = o_tr + up(nnz * 4), o_tv = o_tc + up(nnz * 4),
                 o_tn = o_tv + up(nnz * 8), total_b = o_tn + up(nnz * 4) + 256;
    if (scratch.alloc(total_b) != hipSuccess) return fail(ctx, SLAT_EOOM, "permute scratch");
    uint8_t *w = (uint8_t *)scratch.p;
    uint32_t *inv = (uint32_t *)w, *trow = (uint32_t *)(w + o_tr), *tcol = (uint32_t *)(w + o_tc),
             *tnar = (uint32_t *)(w + o_tn);
    uint64_t *tval = (uint64_t *)(w + o_tv);
    const dim3 b(kB);
    ctx->h_out[3] = 0;
    if (n) {
        hipLaunchKernelGGL(k_perm_inverse, grid_for(ctx, n), b, 0, s, dperm, n, inv, ctx->h_out_dev + 3);
        hipLaunchKernelGGL(k_perm_check, grid_for(ctx, n), b, 0, s, dperm, n, inv, ctx->h_out_dev + 3);
        SLAT_HIP(ctx, hipGetLastError());
        SLAT_HIP(ctx, hipStreamSynchronize(s));
        if (ctx->h_out[3]) return fail(ctx, SLAT_EINVAL, "permute: perm is not a permutation of 0..n");
    }
    const void *vals = tval;
    if (nnz) {
        hipLaunchKernelGGL(k_perm_trip, grid_for(ctx, nnz), b, 0, s, m->row_ptr, m->col_idx, m->values, m->dtype,
                           n, nnz, inv, trow, tcol, tval);
        SLAT_HIP(ctx, hipGetLastError());
        if (m->dtype == SLAT_U32) {
            hipLaunchKernelGGL(k_narrow_u32, grid_for(ctx, nnz), b, 0, s, tval, nnz, tnar);
            SLAT_HIP(ctx, hipGetLastError());
            vals = tnar;
        }
    }
    // a permutation maps distinct entries to distinct entries: from_coo only sorts (zeros kept)
    return from_coo_dev(ctx, n, nnz, trow, tcol, vals, m->dtype, out, 0, 1);
}

extern "C" slat_status slat_csr_from_edges(slat_ctx *ctx, uint64_t n, uint64_t n_edges, const uint32_t *src,
                                           const uint32_t *dst, int32_t undirected, int32_t residency,
                                           slat_csr *out) {
    if (!ctx || !out) return SLAT_EINVAL;
    if (n_edges && (!src || !dst)) return fail(ctx, SLAT_EINVAL, "from_edges: null arrays");
    if (n > 0xFFFFFFFFull) return fail(ctx, SLAT_EINVAL, "n exceeds u32 ids");
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    Buf s_src{ctx}, s_dst{ctx}, scratch{ctx};
    const uint32_t *ds = nullptr, *dd = nullptr;
    slat_status st;
    if ((st = device_u32(ctx, src, n_edges, residency, s_src, &ds))) return st;
    if ((st = device_u32(ctx, dst, n_edges, residency, s_dst, &dd))) return st;
    const uint64_t nt = undirected ? 2 * n_edges : n_edges;
    if (scratch.alloc(nt * 12 + 256) != hipSuccess) return fail(ctx, SLAT_EOOM, "from_edges triplets");
    uint32_t *trow = (uint32_t *)scratch.p, *tcol = trow + nt, *tval = tcol + nt;
    ctx->h_out[3] = 0;
    if (n_edges) {
        hipLaunchKernelGGL(k_edges_trip, grid_for(ctx, n_edges), dim3(kB), 0, s, ds, dd, n_edges, n, undirected,
                           trow, tcol, tval, ctx->h_out_dev + 3);
        SLAT_HIP(ctx, hipGetLastError());
        SLAT_HIP(ctx, hipStreamSynchronize(s));
        if (ctx->h_out[3]) return fail(ctx, SLAT_EINVAL, "from_edges: node id >= n");  // the reference panics
    }
    return from_coo_dev(ctx, n, nt, trow, tcol, tval, SLAT_U32, out, 1);
}

extern "C" slat_status slat_bandwidth_stats(slat_ctx *ctx, const slat_csr_view *m, uint64_t *max_bw,
                                            double *avg_bw) {
    if (!ctx || !max_bw || !avg_bw) return SLAT_EINVAL;
    slat_status st = slat_check_view(ctx, m, "m");
    if (st) return st;
    if (m->residency != SLAT_DEVICE) return fail(ctx, SLAT_EINVAL, "bandwidth_stats takes a device-resident matrix");
    SLAT_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    Buf acc{ctx};
    if (acc.alloc(16) != hipSuccess) return fail(ctx, SLAT_EOOM, "bandwidth accumulators");
    unsigned long long h[2] = {0, 0};
    SLAT_HIP(ctx, hipMemsetAsync(acc.p, 0, 16, s));
    if (m->nnz) {
        hipLaunchKernelGGL(k_bandwidth, grid_for(ctx, m->nnz), dim3(kB), 0, s, m->row_ptr, m->col_idx, m->n_rows,
                           m->nnz, (unsigned long long *)acc.p);
        SLAT_HIP(ctx, hipGetLastError());
    }
    SLAT_HIP(ctx, hipMemcpyAsync(h, acc.p, 16, hipMemcpyDeviceToHost, s));
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    *max_bw = h[0];
    *avg_bw = (double)h[1] / (double)std::max<uint64_t>(m->nnz, 1);
    return SLAT_OK;
}

// CsrMatrix::rcm's order (src/graph_csr.rs:663-722), perm[new] = old: per unvisited seed, a plain
// BFS whose last node starts a BFS that takes unvisited neighbours by ascending degree (ties in
// column order, i.e. a stable sort: the reference's sort_unstable leaves ties unspecified); the
// visit order reversed. The BFS is sequential, so it runs on the host over a host copy.
extern "C" slat_status slat_rcm_order(slat_ctx *ctx, const slat_csr_view *m, uint32_t *perm) {
    if (!ctx || !perm) return SLAT_EINVAL;
    slat_status st = slat_check_view(ctx, m, "m");
    if (st) return st;
    if (m->n_rows != m->n_cols) return fail(ctx, SLAT_EDIM, "matrix is not square");
    const uint64_t n = m->n_rows;
    std::vector<uint64_t> rp_h;
    std::vector<uint32_t> col_h;
    const uint64_t *rp = m->row_ptr;
    const uint32_t *col = m->col_idx;
    if (m->residency == SLAT_DEVICE) {
        SLAT_HIP(ctx, hipSetDevice(ctx->device));
        rp_h.resize(n + 1);
        col_h.resize(std::max<uint64_t>(m->nnz, 1));
        SLAT_HIP(ctx, hipMemcpyAsync(rp_h.data(), m->row_ptr, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
        if (m->nnz)
            SLAT_HIP(ctx, hipMemcpyAsync(col_h.data(), m->col_idx, m->nnz * 4, hipMemcpyDeviceToHost, ctx->stream));
        SLAT_HIP(ctx, hipStreamSynchronize(ctx->stream));
        rp = rp_h.data();
        col = col_h.data();
    }
    if (n == 0) return SLAT_OK;
    auto deg = [&](uint64_t v) { return rp[v + 1] - rp[v]; };
    std::vector<uint8_t> visited(n, 0);
    std::vector<uint64_t> mark(n, 0), queue, order, nbrs;
    queue.reserve(n);
    order.reserve(n);
    for (uint64_t seed = 0; seed < n; ++seed) {
        if (visited[seed]) continue;
        // pseudo-peripheral start: the last node of a BFS from the seed (its own visited marks)
        queue.clear();
        queue.push_back(seed);
        mark[seed] = seed + 1;
        uint64_t last = seed;
        for (size_t h = 0; h < queue.size(); ++h) {
            const uint64_t u = queue[h];
            last = u;
            for (uint64_t i = rp[u]; i < rp[u + 1]; ++i)
                if (mark[col[i]] != seed + 1) {
                    mark[col[i]] = seed + 1;
                    queue.push_back(col[i]);
                }
        }
        queue.clear();
        queue.push_back(last);
        visited[last] = 1;
        for (size_t h = 0; h < queue.size(); ++h) {
            const uint64_t u = queue[h];
            order.push_back(u);
            if (order.size() > n) return fail(ctx, SLAT_EINVAL, "rcm: order is not a permutation");
            nbrs.clear();
            for (uint64_t i = rp[u]; i < rp[u + 1]; ++i)
                if (!visited[col[i]]) nbrs.push_back(col[i]);
            std::stable_sort(nbrs.begin(), nbrs.end(), [&](uint64_t x, uint64_t y) { return deg(x) < deg(y); });
            for (uint64_t v : nbrs)
                if (!visited[v]) {
                    visited[v] = 1;
                    queue.push_back(v);
                }
        }
    }
    // a directed graph can restart a finished component: the reference's permute then panics
    if (order.size() != n) return fail(ctx, SLAT_EINVAL, "rcm: order is not a permutation");
    for (uint64_t i = 0; i < n; ++i) perm[i] = (uint32_t)order[n - 1 - i];
    return SLAT_OK;
}
