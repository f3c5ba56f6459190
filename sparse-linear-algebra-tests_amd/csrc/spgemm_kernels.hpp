// spgemm_kernels.hpp — gfx950 device code for row-wise (Gustavson) SpGEMM C = A·B.
//
// Data layout in HBM (the reference's CSR, src/graph_csr.rs:42-53): row_ptr u64[n+1],
// col_idx u32[nnz] (sorted, unique per row), values u32 | u64 | f64 [nnz].
//
// Pipeline (the reference's matmul_par structure, src/graph_csr.rs:360-476, re-designed):
//   k_symbolic  one wavefront per row: structural nnz via an LDS column bitmap
//   (scan)      hipcub inclusive scan -> C.row_ptr
//   k_numeric   one row GROUP (1 or 4 wavefronts) per row:
//                 1. gather: every scalar product (j, a_ik*b_kj) of the row, loaded with batched
//                    independent loads (Q A-entries x U B-entries per lane in flight), into an LDS
//                    product cache (one global traversal per row);
//                 2. bitmap: the row's column set over an LDS window of 32*ww columns;
//                 3. ranks: word prefix popcounts -> rank(j) = wbase[w] + popc(bits below j),
//                    so the output is emitted already sorted (the reference sorts nz_cols,
//                    src/graph_csr.rs:449);
//                 4. values: accumulate cached products into LDS slots indexed by rank;
//                 5. emit: coalesced stores of (col, value) at C.row_ptr[i] + rank.
//               Rows whose products exceed the cache re-traverse global memory instead; rows with
//               more distinct columns than the LDS slots run several rank chunks; rows wider
//               than a window run several windows (MAGNUS-style fine-level column chunking).
//   k_compact   only when an emitted value is exactly zero (f64 cancellation or explicit zero
//               inputs): drops those entries, rebuilding exact row slices (matmul's `v != 0`).
//
// Semantics kept bit-exact (SURVEY.md §8(a) rules 1-4):
//   u32   : product clamped to u32::MAX, u32 LDS atomic adds, a wrap of the running sum sets a
//           per-slot saturation bit (a wrap happens iff the exact sum >= 2^32) == sadd/smul
//           (src/graph_csr.rs:29-37), valid in any order because all values are non-negative.
//   Sat64 : the same with u64 and __umul64hi overflow detection == Sat64 (src/graph_sprs.rs:29-51).
//   f64   : each wavefront walks A's row entries in order with lanes spread over one B row
//           (distinct columns) and owns a disjoint quarter of the rank range, non-atomic
//           __dmul_rn/__dadd_rn: the left fold from 0.0 in A-row order of linalg/src/csr.rs:325-337.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace slat {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kShards = 64;      // sharded status words (avoid one hot atomic address)
constexpr uint32_t kSent = 0xFFFFFFFFu;  // ELL padding (column ids are < n_cols <= 2^32 - 1)
constexpr int kShardStride = 4;  // [0] total nnz (shard 0), [1] max row nnz, [2] rows with zeros, [3] flops

struct Args {
    const uint64_t *a_rp;
    const uint32_t *a_col;
    const void *a_val;
    const uint64_t *b_rp;
    const uint32_t *b_col;
    const void *b_val;
    uint64_t nrows, ncols;
    uint64_t b_nrows;  // column ids of A index rows of B: anything >= b_nrows is ignored
    uint32_t ww;     // bitmap words per window
    uint32_t cap;    // rank-chunk capacity (value slots per LDS pass)
    uint32_t wide;   // 0 = one window at column 0 covers all columns; 1 = row-span windows
    uint32_t stats;  // count products into shard[3]
    uint32_t ell_wq; // groups of 4 per row in the padded ELL copy of B (0: CSR only)
    uint32_t ablate; // experiments only (SLAT_ABLATE): 1 = symbolic skips its LDS bitmap
    const uint32_t *ell_col;  // [n_B][ell_wq*4] columns, kSent padded
    const void *ell_val;      // [n_B][ell_wq*4] values
    uint64_t *counts;  // symbolic: structural nnz per row; numeric: non-zero nnz per row
    uint64_t *c_rp;    // C.row_ptr (n+1)
    uint32_t *c_col;
    void *c_val;
    unsigned long long *shards;
};

// ------------------------------------------------------------------------------------------------
// value semirings: S storage type, P cached product, V LDS accumulator
// ------------------------------------------------------------------------------------------------
struct SemU32 {
    using S = uint32_t;
    using P = uint32_t;
    using V = unsigned long long;
    static constexpr int kSlots = 1;  // V words per output slot
    static constexpr bool kOrdered = false;
    __device__ static __forceinline__ P prod(S a, S b) {
        const unsigned long long p = (unsigned long long)a * b;
        return p > 0xFFFFFFFFull ? 0xFFFFFFFFu : (P)p;  // Saturating<u32> product
    }
    // exact u64 sum of < 2^32 clamped products, no returned value: the atomics pipeline freely
    __device__ static __forceinline__ void acc(V *vals, uint32_t r, P p) { atomicAdd(&vals[r], (V)p); }
    __device__ static __forceinline__ S finish(const V *vals, uint32_t t) {
        const V v = vals[t];
        return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (S)v;  // the saturating sum
    }
    __device__ static __forceinline__ bool is_zero(S v) { return v == 0; }
};

struct SemSat64 {
    using S = unsigned long long;
    using P = unsigned long long;
    using V = unsigned long long;
    static constexpr int kSlots = 2;  // low / high 32-bit halves of the products, summed apart
    static constexpr bool kOrdered = false;
    __device__ static __forceinline__ P prod(S a, S b) {
        return __umul64hi(a, b) != 0 ? ~0ull : a * b;  // Saturating<u64> product
    }
    __device__ static __forceinline__ void acc(V *vals, uint32_t r, P p) {
        atomicAdd(&vals[2 * r], p & 0xFFFFFFFFull);
        atomicAdd(&vals[2 * r + 1], p >> 32);
    }
    __device__ static __forceinline__ S finish(const V *vals, uint32_t t) {
        const V lo = vals[2 * t], hi = vals[2 * t + 1] + (vals[2 * t] >> 32);
        return hi > 0xFFFFFFFFull ? ~0ull : ((hi << 32) | (lo & 0xFFFFFFFFull));  // exact sum, saturated
    }
    __device__ static __forceinline__ bool is_zero(S v) { return v == 0; }
};

struct SemF64 {
    using S = double;
    using P = double;
    using V = double;
    static constexpr int kSlots = 1;
    static constexpr bool kOrdered = true;
    __device__ static __forceinline__ P prod(S a, S b) { return __dmul_rn(a, b); }
    __device__ static __forceinline__ void acc(V *vals, uint32_t r, P p) {
        vals[r] = __dadd_rn(vals[r], p);  // no FMA contraction: Rust's a*b then +
    }
    __device__ static __forceinline__ S finish(const V *vals, uint32_t t) { return vals[t]; }
    __device__ static __forceinline__ bool is_zero(S v) { return v == 0.0; }
};

// ------------------------------------------------------------------------------------------------
// wave / group helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// LDS written by some lanes and read by others within one wave: DS instructions of a wave execute
// in order; the fences stop the compiler from reordering across the hand-off.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d));
    return v;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, (uint32_t)__shfl_xor(v, d));
    return v;
}
__device__ __forceinline__ uint32_t wave_excl_scan_u32(uint32_t x) {
    const int lane = lane_id();
    uint32_t v = x;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t t = __shfl_up(v, d);
        if (lane >= d) v += t;
    }
    return v - x;
}
__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    return ((uint64_t)readlane_u32((uint32_t)(v >> 32), l) << 32) | readlane_u32((uint32_t)v, l);
}
template <typename S>
__device__ __forceinline__ S readlane_val(S v, int l) {
    if constexpr (sizeof(S) == 4) {
        return (S)readlane_u32((uint32_t)v, l);
    } else {
        return __builtin_bit_cast(S, readlane_u64(__builtin_bit_cast(uint64_t, v), l));
    }
}

// Ordered traversal (f64): A's row entries in order, lanes spread over one B row (distinct
// columns), 64 A entries' row pointers prefetched at a time.
template <typename I, typename S, typename F>
__device__ __forceinline__ void traverse_ordered(const Args &p, I a0, I a1, F &&visit) {
    const int lane = lane_id();
    const S *av_ = (const S *)p.a_val;
    const S *bv_ = (const S *)p.b_val;
    for (I base = a0; base < a1; base += kWave) {
        const I idx = base + (I)lane;
        I bs = 0, be = 0;
        S av = S(0);
        if (idx < a1) {
            const uint32_t k = p.a_col[idx];
            av = av_[idx];
            if (k < p.b_nrows) {
                bs = (I)p.b_rp[k];
                be = (I)p.b_rp[k + 1];
            }
        }
        const int cnt = (int)min<uint64_t>((uint64_t)kWave, (uint64_t)(a1 - base));
        for (int t = 0; t < cnt; ++t) {
            const I s = (I)readlane_u64((uint64_t)bs, t), e = (I)readlane_u64((uint64_t)be, t);
            const S a = readlane_val(av, t);
            for (I jdx = s + (I)lane; jdx < e; jdx += (I)kWave) visit(p.b_col[jdx], a, bv_[jdx]);
        }
    }
}

// Column span [lo, hi] of row i of A·B from B's row ends (B rows are sorted); lo > hi if empty.
template <typename I>
__device__ __forceinline__ void row_span(const Args &p, I a0, I a1, uint64_t &lo, uint64_t &hi) {
    const int lane = lane_id();
    uint32_t l = 0xFFFFFFFFu, h = 0;
    for (I idx = a0 + (I)lane; idx < a1; idx += (I)kWave) {
        const uint32_t k = p.a_col[idx];
        if (k >= p.b_nrows) continue;
        const I bs = (I)p.b_rp[k], be = (I)p.b_rp[k + 1];
        if (be > bs) {
            l = min(l, p.b_col[bs]);
            h = max(h, p.b_col[be - 1]);
        }
    }
    l = wave_min_u32(l);
    h = wave_max_u32(h);
    lo = l;
    hi = h;
    if (l > h) {
        lo = 1;
        hi = 0;
    }
}

// ------------------------------------------------------------------------------------------------
// padded ELL copy of B (rows of B short, e.g. the base adjacency of an A^k chain): row k holds
// ell_wq groups of 4 columns at ell_col[k*ell_wq ..], padded with kSent, and the matching values
// (4 per uint4 for 4-byte values, 4 per 2 uint4 for 8-byte values). One dwordx4 load brings four
// B entries, the B row pointers drop out of the dependent load chain (a_col -> ELL row), and
// rows are 16-byte aligned. Built per call into the context workspace (a few microseconds).
// ------------------------------------------------------------------------------------------------
template <typename S>
__global__ __launch_bounds__(kBlock) void k_build_ell(const uint64_t *rp, const uint32_t *col, const S *val,
                                                       uint32_t n, uint32_t wq, uint32_t *ecol, S *eval) {
    for (uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x; k < n; k += (uint64_t)gridDim.x * kBlock) {
        const uint64_t s0 = rp[k], len = rp[k + 1] - s0;
        for (uint32_t u = 0; u < wq * 4; ++u) {
            const uint64_t o = k * wq * 4 + u;
            ecol[o] = u < len ? col[s0 + u] : kSent;
            eval[o] = u < len ? val[s0 + u] : S(0);
        }
    }
}

template <typename S>
struct Quad {
    S v[4];
};

// the t-th group of 4 values of ELL row k
template <typename S>
__device__ __forceinline__ Quad<S> ell_vals(const Args &p, uint32_t k, uint32_t t) {
    Quad<S> q;
    if constexpr (sizeof(S) == 4) {
        const uint4 x = ((const uint4 *)p.ell_val)[(size_t)k * p.ell_wq + t];
        q.v[0] = __builtin_bit_cast(S, x.x);
        q.v[1] = __builtin_bit_cast(S, x.y);
        q.v[2] = __builtin_bit_cast(S, x.z);
        q.v[3] = __builtin_bit_cast(S, x.w);
    } else {
        const uint4 *b = (const uint4 *)p.ell_val + ((size_t)k * p.ell_wq + t) * 2;
        const uint4 x = b[0], y = b[1];
        q.v[0] = __builtin_bit_cast(S, ((uint64_t)x.y << 32) | x.x);
        q.v[1] = __builtin_bit_cast(S, ((uint64_t)x.w << 32) | x.z);
        q.v[2] = __builtin_bit_cast(S, ((uint64_t)y.y << 32) | y.x);
        q.v[3] = __builtin_bit_cast(S, ((uint64_t)y.w << 32) | y.z);
    }
    return q;
}

__device__ __forceinline__ uint4 ell_cols(const Args &p, uint32_t k, uint32_t t) {
    return ((const uint4 *)p.ell_col)[(size_t)k * p.ell_wq + t];
}

// ------------------------------------------------------------------------------------------------
// group walks: the passes consume B entries four at a time (one ELL group, or a CSR entry padded
// with kSent), branch-free inside a group, so a wave issues every LDS access of a group before
// it waits on any.
// ------------------------------------------------------------------------------------------------
template <typename S>
__device__ __forceinline__ Quad<S> quad1(S v) {
    Quad<S> q{};
    q.v[0] = v;
    return q;
}

// grp(c4, v4, a) for every group of B row k, ELL groups from t0 on (CSR: one entry per group)
template <bool ELL, bool VALS, typename I, typename S, typename G>
__device__ __forceinline__ void walk_brow(const Args &p, uint32_t k, S a, uint32_t t0, G &&grp) {
    if constexpr (ELL) {
        for (uint32_t t = t0; t < p.ell_wq; ++t) {
            const uint4 c = ell_cols(p, k, t);
            Quad<S> v{};
            if constexpr (VALS) v = ell_vals<S>(p, k, t);
            grp(c, v, a);
            if (c.w == kSent) break;
        }
    } else {
        const S *bv_ = (const S *)p.b_val;
        const I bs = (I)p.b_rp[k], be = (I)p.b_rp[k + 1];
        for (I jdx = bs; jdx < be; ++jdx)
            grp(make_uint4(p.b_col[jdx], kSent, kSent, kSent), quad1<S>(VALS ? bv_[jdx] : S(0)), a);
    }
}

// Lane-per-A-entry walk of a row: lane l owns entries base + l and base + 64 + l.
template <bool ELL, bool VALS, typename I, typename S, typename G>
__device__ __forceinline__ void walk_row(const Args &p, I a0, I a1, G &&grp) {
    const int lane = lane_id();
    const S *av_ = (const S *)p.a_val;
    for (I base = a0; base < a1; base += (I)(2 * kWave)) {
        const I i0 = base + (I)lane, i1 = i0 + (I)kWave;
        uint32_t k0 = kSent, k1 = kSent;
        S a0v = S(0), a1v = S(0);
        if (i0 < a1) {
            k0 = p.a_col[i0];
            if constexpr (VALS) a0v = av_[i0];
        }
        if (i1 < a1) {
            k1 = p.a_col[i1];
            if constexpr (VALS) a1v = av_[i1];
        }
        if (k0 < p.b_nrows) walk_brow<ELL, VALS, I, S>(p, k0, a0v, 0, grp);
        if (k1 < p.b_nrows) walk_brow<ELL, VALS, I, S>(p, k1, a1v, 0, grp);
    }
}

// window offset of column c: valid iff c is a real column inside [wlo, wlo + WIN)
__device__ __forceinline__ bool win_off(uint32_t c, uint32_t wlo, uint32_t WIN, uint32_t &off) {
    off = c - wlo;
    return c != kSent && off < WIN;
}

// atomicOr the (up to) four columns of a group into the window bitmap; no returned values
__device__ __forceinline__ void bitmap_or4(uint32_t *L0, uint4 c, uint32_t wlo, uint32_t WIN) {
    const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        uint32_t off;
        if (win_off(cc[e], wlo, WIN, off)) atomicOr(&L0[off >> 5], 1u << (off & 31));
    }
}

// ------------------------------------------------------------------------------------------------
// symbolic: structural nnz per output row, one wavefront per row
// ------------------------------------------------------------------------------------------------
template <typename I, bool ELL>
__global__ __launch_bounds__(kBlock) void k_symbolic(Args p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    constexpr int kWpb = kBlock / kWave;
    const int lane = lane_id();
    const int wv = threadIdx.x / kWave;
    uint32_t *L0 = smem + (size_t)wv * p.ww;
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) p.c_rp[0] = 0;
        if (threadIdx.x < kShards) {  // fields read by k_numeric; [3] (flops) is zeroed by the host
            p.shards[threadIdx.x * kShardStride + 1] = 0;
            p.shards[threadIdx.x * kShardStride + 2] = 0;
        }
    }
    for (uint32_t w = lane; w < p.ww; w += kWave) L0[w] = 0;
    wave_sync();
    const uint32_t WIN = p.ww * 32;
    const uint32_t per = p.ww / kWave;  // odd: lane-contiguous word ownership is conflict-free
    const uint32_t wb0 = lane * per;
    unsigned long long flops = 0;
    const uint64_t stride = (uint64_t)gridDim.x * kWpb;
    for (uint64_t row = (uint64_t)blockIdx.x * kWpb + wv; row < p.nrows; row += stride) {
        const I a0 = (I)p.a_rp[row], a1 = (I)p.a_rp[row + 1];
        uint64_t cnt = 0;
        if (a1 > a0) {
            uint64_t lo = 0, hi = p.ncols - 1;
            if (p.wide) row_span<I>(p, a0, a1, lo, hi);
            bool first = true;
            for (uint64_t wlo = lo & ~31ull; wlo <= hi; wlo += WIN) {
                uint32_t nprod = 0, x = 0;
                walk_row<ELL, false, I, uint32_t>(p, a0, a1, [&](uint4 c, const Quad<uint32_t> &, uint32_t) {
                    if (p.stats) nprod += (c.x != kSent) + (c.y != kSent) + (c.z != kSent) + (c.w != kSent);
                    if (p.ablate & 1u)
                        x ^= c.x ^ c.y ^ c.z ^ c.w;
                    else
                        bitmap_or4(L0, c, (uint32_t)wlo, WIN);
                });
                wave_sync();
                // count = popcount of the window; lane owns words [wb0, wb0 + per) and clears them
                uint32_t lc = 0;
                for (uint32_t q = 0; q < per; ++q) {
                    lc += __popc(L0[wb0 + q]);
                    L0[wb0 + q] = 0;
                }
                if (p.ablate & 1u) lc += x & 1u;
                cnt += wave_sum_u32(lc);
                if (p.stats && first) flops += wave_sum_u32(nprod);
                first = false;
                wave_sync();
            }
        }
        if (lane == 0) p.counts[row] = cnt;
    }
    if (p.stats && lane == 0 && flops)
        atomicAdd(&p.shards[((blockIdx.x * kWpb + wv) % kShards) * kShardStride + 3], flops);
}

// ------------------------------------------------------------------------------------------------
// numeric: one wavefront per row
// ------------------------------------------------------------------------------------------------
struct NumLayout {
    uint32_t off_wb, off_vals, off_cols, bytes;
};

// Per-wave LDS region: L0 ww*4 | wbase ww*2 | vals cap*slot_bytes | cols cap*4
__host__ __device__ inline NumLayout num_layout(uint32_t ww, uint32_t cap, uint32_t slot_bytes) {
    auto up = [](uint32_t x, uint32_t a) { return (x + a - 1) / a * a; };
    NumLayout L;
    L.off_wb = ww * 4;
    L.off_vals = up(L.off_wb + ww * 2, 16);
    L.off_cols = up(L.off_vals + cap * slot_bytes, 16);
    L.bytes = up(L.off_cols + cap * 4, 16);
    return L;
}

constexpr int kRegQ = 4;  // A entries per lane kept in registers across the numeric passes

template <typename Sem, typename I, bool ELL>
__global__ __launch_bounds__(kBlock) void k_numeric(Args p) {
    using S = typename Sem::S;
    using V = typename Sem::V;
    constexpr int kWpb = kBlock / kWave;
    constexpr bool kVals = !Sem::kOrdered;  // f64 accumulates from an ordered CSR walk
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    __shared__ uint32_t red[2][kWpb];

    const int lane = lane_id();
    const int wv = threadIdx.x / kWave;
    const NumLayout lay = num_layout(p.ww, p.cap, sizeof(V) * Sem::kSlots);
    uint8_t *region = smem8 + (size_t)wv * lay.bytes;
    uint32_t *L0 = (uint32_t *)region;
    uint16_t *wbase = (uint16_t *)(region + lay.off_wb);
    V *vals = (V *)(region + lay.off_vals);
    uint32_t *cols = (uint32_t *)(region + lay.off_cols);
    S *cval = (S *)p.c_val;
    const S *av_ = (const S *)p.a_val;

    if (blockIdx.x == 0 && threadIdx.x == 0) p.shards[0] = p.c_rp[p.nrows];
    for (uint32_t w = lane; w < p.ww; w += kWave) L0[w] = 0;
    wave_sync();

    const uint32_t WIN = p.ww * 32;
    const uint32_t per = p.ww / kWave;  // odd: lane-contiguous word ownership is conflict-free
    const uint32_t wb0 = lane * per;
    uint32_t maxrow = 0, zrows = 0;
    const uint64_t stride = (uint64_t)gridDim.x * kWpb;
    for (uint64_t row = (uint64_t)blockIdx.x * kWpb + wv; row < p.nrows; row += stride) {
        const I a0 = (I)p.a_rp[row], a1 = (I)p.a_rp[row + 1];
        const uint64_t out_begin = p.c_rp[row], out_end = p.c_rp[row + 1];
        uint64_t out_pos = out_begin;
        uint32_t zeros = 0;
        if (a1 > a0) {
            // rows of up to 64*kRegQ A entries keep their A entries in registers for both passes
            const bool single = (uint64_t)(a1 - a0) <= (uint64_t)(kWave * kRegQ);
            uint32_t kq[kRegQ];
            S aq[kRegQ];
#pragma unroll
            for (int q = 0; q < kRegQ; ++q) {
                const I idx = a0 + (I)(q * kWave + lane);
                kq[q] = kSent;
                aq[q] = S(0);
                if (single && idx < a1) {
                    kq[q] = p.a_col[idx];
                    if (kq[q] >= p.b_nrows) kq[q] = kSent;  // malformed input: ignore the entry
                    if constexpr (kVals) aq[q] = av_[idx];
                }
            }
            // every group of the row: the first group of every register-resident A entry is
            // loaded for all q before any is consumed, then the tails
            auto each_group = [&](auto &&grp, auto vals_tag) {
                constexpr bool VV = decltype(vals_tag)::value;
                if (single) {
                    if constexpr (ELL) {
                        uint4 cq[kRegQ];
                        Quad<S> vq[kRegQ];
#pragma unroll
                        for (int q = 0; q < kRegQ; ++q) {
                            cq[q] = make_uint4(kSent, kSent, kSent, kSent);
                            vq[q] = Quad<S>{};
                            if (kq[q] != kSent) {
                                cq[q] = ell_cols(p, kq[q], 0);
                                if constexpr (VV) vq[q] = ell_vals<S>(p, kq[q], 0);
                            }
                        }
                        grp.multi(cq, vq, aq);
#pragma unroll
                        for (int q = 0; q < kRegQ; ++q)
                            if (cq[q].w != kSent) walk_brow<true, VV, I, S>(p, kq[q], aq[q], 1, grp);
                    } else {
#pragma unroll
                        for (int q = 0; q < kRegQ; ++q)
                            if (kq[q] != kSent) walk_brow<false, VV, I, S>(p, kq[q], aq[q], 0, grp);
                    }
                } else {
                    walk_row<ELL, VV, I, S>(p, a0, a1, grp);
                }
            };
            uint64_t lo = 0, hi = p.ncols - 1;
            if (p.wide) {
                struct MinMax {
                    uint32_t l = 0xFFFFFFFFu, h = 0;
                    __device__ void operator()(uint4 c, const Quad<S> &, S) {
                        const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (cc[e] != kSent) {
                                l = min(l, cc[e]);
                                h = max(h, cc[e]);
                            }
                    }
                    __device__ void multi(const uint4 *c, const Quad<S> *v, const S *a) {
#pragma unroll
                        for (int q = 0; q < kRegQ; ++q) (*this)(c[q], v[q], a[q]);
                    }
                } mm;
                each_group(mm, std::false_type{});
                const uint32_t l = wave_min_u32(mm.l), h = wave_max_u32(mm.h);
                lo = l;
                hi = h;
                if (l > h) {
                    lo = 1;
                    hi = 0;
                }
            }
            for (uint64_t wlo64 = lo & ~31ull; wlo64 <= hi; wlo64 += WIN) {
                const uint32_t wlo = (uint32_t)wlo64;
                // 1. column bitmap of the window
                struct Or4 {
                    uint32_t *L0;
                    uint32_t wlo, WIN;
                    __device__ void operator()(uint4 c, const Quad<S> &, S) { bitmap_or4(L0, c, wlo, WIN); }
                    __device__ void multi(const uint4 *c, const Quad<S> *, const S *) {
#pragma unroll
                        for (int q = 0; q < kRegQ; ++q) bitmap_or4(L0, c[q], wlo, WIN);
                    }
                } or4{L0, wlo, WIN};
                if (!(p.ablate & 32u)) each_group(or4, std::false_type{});
                wave_sync();
                // 2. word ranks (lane owns words [wb0, wb0 + per))
                uint32_t lc = 0;
                for (uint32_t q = 0; q < per; ++q) lc += __popc(L0[wb0 + q]);
                const uint32_t ex = wave_excl_scan_u32(lc);
                const uint32_t wcnt = readlane_u32(ex + lc, kWave - 1);
                if (wcnt == 0) continue;  // bitmap empty: nothing to clear
                {
                    uint32_t run = ex;
                    for (uint32_t q = 0; q < per; ++q) {
                        wbase[wb0 + q] = (uint16_t)run;
                        run += __popc(L0[wb0 + q]);
                    }
                }
                wave_sync();
                for (uint32_t r0 = 0; r0 < wcnt; r0 += p.cap) {
                    const uint32_t nch = min(p.cap, wcnt - r0);
                    for (uint32_t t = lane; t < nch * Sem::kSlots; t += kWave) vals[t] = V(0);
                    wave_sync();
                    // rank of column c in this chunk, or kSent; the two LDS reads are unconditional
                    auto rank_of = [&](uint32_t c) -> uint32_t {
                        uint32_t off;
                        const bool ok = win_off(c, wlo, WIN, off);
                        const uint32_t w = ok ? (off >> 5) : 0u;
                        const uint32_t r = (uint32_t)wbase[w] + __popc(L0[w] & ((1u << (off & 31)) - 1u)) - r0;
                        return (ok && r < nch) ? r : kSent;
                    };
                    // 3. values + the column of every rank (duplicates store the same column)
                    if constexpr (Sem::kOrdered) {
                        if (!(p.ablate & 8u))
                            traverse_ordered<I, S>(p, a0, a1, [&](uint32_t j, S a, S b) {
                                const uint32_t r = rank_of(j);
                                if (r != kSent) {
                                    Sem::acc(vals, r, Sem::prod(a, b));
                                    cols[r] = j;
                                }
                            });
                    } else if (!(p.ablate & 8u)) {
                        struct Acc4 {
                            decltype(rank_of) &rk;
                            V *vals;
                            uint32_t *cols;
                            __device__ void operator()(uint4 c, const Quad<S> &v, S a) {
                                const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
                                uint32_t r[4];
#pragma unroll
                                for (int e = 0; e < 4; ++e) r[e] = rk(cc[e]);
#pragma unroll
                                for (int e = 0; e < 4; ++e)
                                    if (r[e] != kSent) {
                                        Sem::acc(vals, r[e], Sem::prod(a, v.v[e]));
                                        cols[r[e]] = cc[e];
                                    }
                            }
                            __device__ void multi(const uint4 *c, const Quad<S> *v, const S *a) {
                                uint32_t r[kRegQ][4];
#pragma unroll
                                for (int q = 0; q < kRegQ; ++q) {
                                    const uint32_t cc[4] = {c[q].x, c[q].y, c[q].z, c[q].w};
#pragma unroll
                                    for (int e = 0; e < 4; ++e) r[q][e] = rk(cc[e]);
                                }
#pragma unroll
                                for (int q = 0; q < kRegQ; ++q) {
                                    const uint32_t cc[4] = {c[q].x, c[q].y, c[q].z, c[q].w};
#pragma unroll
                                    for (int e = 0; e < 4; ++e)
                                        if (r[q][e] != kSent) {
                                            Sem::acc(vals, r[q][e], Sem::prod(a[q], v[q].v[e]));
                                            cols[r[q][e]] = cc[e];
                                        }
                                }
                            }
                        } acc4{rank_of, vals, cols};
                        each_group(acc4, std::integral_constant<bool, kVals>{});
                    }
                    wave_sync();
                    // 4. emit at the row's slice, coalesced
                    for (uint32_t t = lane; t < nch; t += kWave) {
                        const S v = Sem::finish(vals, t);
                        zeros += Sem::is_zero(v) ? 1u : 0u;
                        if (out_pos + t < out_end && !(p.ablate & 16u)) {  // never trust blindly
                            p.c_col[out_pos + t] = cols[t];
                            cval[out_pos + t] = v;
                        }
                    }
                    out_pos += nch;
                    wave_sync();
                }
                for (uint32_t q = 0; q < per; ++q) L0[wb0 + q] = 0;
                wave_sync();
            }
        }
        const uint32_t rz = p.ablate ? 0u : wave_sum_u32(zeros);  // ablation runs: no compaction
        const uint64_t got = out_pos - out_begin - rz;
        if (lane == 0) p.counts[row] = got;
        maxrow = max(maxrow, (uint32_t)min<uint64_t>(got, 0xFFFFFFFFull));
        zrows += rz ? 1u : 0u;
    }
    if (lane == 0) {
        red[0][wv] = maxrow;
        red[1][wv] = zrows;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t m = 0, d = 0;
        for (int w = 0; w < kWpb; ++w) {
            m = max(m, red[0][w]);
            d += red[1][w];
        }
        unsigned long long *sh = p.shards + (blockIdx.x % kShards) * kShardStride;
        if (m) atomicMax(&sh[1], (unsigned long long)m);
        if (d) atomicAdd(&sh[2], (unsigned long long)d);
    }
}

// ------------------------------------------------------------------------------------------------
// compaction (rare): drop exact-zero values, moving row slices into exact-size arrays
// ------------------------------------------------------------------------------------------------
template <typename Sem>
__global__ __launch_bounds__(kBlock) void k_compact(const uint64_t *old_rp, const uint64_t *new_rp, uint64_t nrows,
                                                    const uint32_t *old_col, const typename Sem::S *old_val,
                                                    uint32_t *new_col, typename Sem::S *new_val) {
    const int lane = lane_id();
    constexpr int kWpb = kBlock / kWave;
    const uint64_t stride = (uint64_t)gridDim.x * kWpb;
    for (uint64_t row = (uint64_t)blockIdx.x * kWpb + threadIdx.x / kWave; row < nrows; row += stride) {
        const uint64_t s = old_rp[row], e = old_rp[row + 1];
        uint64_t d = new_rp[row];
        for (uint64_t t0 = s; t0 < e; t0 += kWave) {
            const uint64_t t = t0 + lane;
            typename Sem::S v{};
            bool keep = false;
            if (t < e) {
                v = old_val[t];
                keep = !Sem::is_zero(v);
            }
            const unsigned long long m = __ballot(keep);
            const uint32_t off = __popcll(m & ((1ull << lane) - 1ull));
            if (keep) {
                new_col[d + off] = old_col[t];
                new_val[d + off] = v;
            }
            d += __popcll(m);
        }
    }
}

// max over rows of row_ptr[i+1] - row_ptr[i]
__global__ __launch_bounds__(kBlock) void k_max_row(const uint64_t *rp, uint64_t nrows, unsigned long long *shards) {
    __shared__ unsigned long long red[kBlock];
    unsigned long long m = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nrows; i += (uint64_t)gridDim.x * kBlock)
        m = max(m, (unsigned long long)(rp[i + 1] - rp[i]));
    red[threadIdx.x] = m;
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0 && red[0]) atomicMax(&shards[(blockIdx.x % kShards) * kShardStride + 1], red[0]);
}

}  // namespace slat
