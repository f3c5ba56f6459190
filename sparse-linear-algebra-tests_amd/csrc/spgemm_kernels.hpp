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
constexpr int kShardStride = 4;  // [0] total nnz (shard 0), [1] max row nnz, [2] rows with zeros, [3] flops

struct Args {
    const uint64_t *a_rp;
    const uint32_t *a_col;
    const void *a_val;
    const uint64_t *b_rp;
    const uint32_t *b_col;
    const void *b_val;
    uint64_t nrows, ncols;
    uint32_t ww;     // bitmap words per window
    uint32_t cap;    // rank-chunk capacity (value slots per LDS pass)
    uint32_t wide;   // 0 = one window at column 0 covers all columns; 1 = row-span windows
    uint32_t stats;  // count products into shard[3]
    uint32_t sell_w; // B in slot-major ELL: slots per row (= max row nnz of B); 0 = CSR only
    uint32_t sell_n; // rows of B in the slot-major copy
    const uint32_t *sell_col;  // [sell_w][sell_n] column or kSent
    const void *sell_val;      // [sell_w][sell_n] value
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
    using V = uint32_t;
    static constexpr bool kOrdered = false;
    __device__ static __forceinline__ P prod(S a, S b) {
        const unsigned long long p = (unsigned long long)a * b;
        return p > 0xFFFFFFFFull ? 0xFFFFFFFFu : (P)p;  // Saturating<u32> product
    }
    __device__ static __forceinline__ void acc(V *vals, uint32_t *sat, uint32_t r, P p) {
        const V old = atomicAdd(&vals[r], p);
        if (old + p < old) atomicOr(&sat[r >> 5], 1u << (r & 31));  // the running sum wrapped
    }
    __device__ static __forceinline__ S finish(const V *vals, const uint32_t *sat, uint32_t t) {
        return ((sat[t >> 5] >> (t & 31)) & 1u) ? 0xFFFFFFFFu : vals[t];
    }
    __device__ static __forceinline__ bool is_zero(S v) { return v == 0; }
};

struct SemSat64 {
    using S = unsigned long long;
    using P = unsigned long long;
    using V = unsigned long long;
    static constexpr bool kOrdered = false;
    __device__ static __forceinline__ P prod(S a, S b) {
        return __umul64hi(a, b) != 0 ? ~0ull : a * b;  // Saturating<u64> product
    }
    __device__ static __forceinline__ void acc(V *vals, uint32_t *sat, uint32_t r, P p) {
        const V old = atomicAdd(&vals[r], p);
        if (old + p < old) atomicOr(&sat[r >> 5], 1u << (r & 31));
    }
    __device__ static __forceinline__ S finish(const V *vals, const uint32_t *sat, uint32_t t) {
        return ((sat[t >> 5] >> (t & 31)) & 1u) ? ~0ull : vals[t];
    }
    __device__ static __forceinline__ bool is_zero(S v) { return v == 0; }
};

struct SemF64 {
    using S = double;
    using P = double;
    using V = double;
    static constexpr bool kOrdered = true;
    __device__ static __forceinline__ P prod(S a, S b) { return __dmul_rn(a, b); }
    __device__ static __forceinline__ void acc(V *vals, uint32_t *, uint32_t r, P p) {
        vals[r] = __dadd_rn(vals[r], p);  // no FMA contraction: Rust's a*b then +
    }
    __device__ static __forceinline__ S finish(const V *vals, const uint32_t *, uint32_t t) { return vals[t]; }
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

// ------------------------------------------------------------------------------------------------
// register-resident product batch: one wavefront gathers the products of up to 64*Q A entries
// (lane l owns entries base + q*64 + l) with every load of a stage issued before any is
// consumed: a_col/a_val -> b_rp -> U B entries per A entry. Three dependent latencies per batch.
// B rows longer than U leave a tail that is streamed from global memory when visited.
// I = offset type (u32 when every nnz < 2^32, else u64).
// ------------------------------------------------------------------------------------------------
template <typename I, typename S, int Q, int U, bool VALS>
struct Batch {
    I bs[Q], be[Q];
    S av[Q];
    uint32_t jj[Q][U];
    S bv[Q][U];

    __device__ __forceinline__ void load(const Args &p, I base, I a1) {
        const int lane = lane_id();
        const S *av_ = (const S *)p.a_val;
        const S *bv_ = (const S *)p.b_val;
        uint32_t k[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const I idx = base + (I)(q * kWave + lane);
            k[q] = 0;
            av[q] = S(0);
            if (idx < a1) {
                k[q] = p.a_col[idx];
                if constexpr (VALS) av[q] = av_[idx];
            }
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const I idx = base + (I)(q * kWave + lane);
            bs[q] = be[q] = 0;
            if (idx < a1) {
                bs[q] = (I)p.b_rp[k[q]];
                be[q] = (I)p.b_rp[k[q] + 1];
            }
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const I jdx = bs[q] + (I)u;
                jj[q][u] = 0;
                bv[q][u] = S(0);
                if (jdx < be[q]) {
                    jj[q][u] = p.b_col[jdx];
                    if constexpr (VALS) bv[q][u] = bv_[jdx];
                }
            }
        }
    }

    // visit(j, a_ik, b_kj) for every product of the batch (registers first, then tails)
    template <typename F>
    __device__ __forceinline__ void for_each(const Args &p, F &&visit) const {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (bs[q] + (I)u < be[q]) visit(jj[q][u], av[q], bv[q][u]);
        }
        const S *bv_ = (const S *)p.b_val;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            for (I jdx = bs[q] + (I)U; jdx < be[q]; ++jdx) {
                S b = S(0);
                if constexpr (VALS) b = bv_[jdx];
                visit(p.b_col[jdx], av[q], b);
            }
        }
    }

    __device__ __forceinline__ uint32_t count() const {
        uint32_t n = 0;
#pragma unroll
        for (int q = 0; q < Q; ++q) n += (uint32_t)(be[q] - bs[q]);
        return n;
    }
};

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
            bs = (I)p.b_rp[k];
            be = (I)p.b_rp[k + 1];
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

constexpr int kQ = 4, kU = 4;  // batch shape: 4 A entries x 4 B entries per lane
constexpr uint32_t kSent = 0xFFFFFFFFu;  // empty slot (column ids are < n_cols <= 2^32 - 1)

// ------------------------------------------------------------------------------------------------
// slot-major ELL copy of B (for B with short rows, e.g. the base adjacency of an A^k chain):
// slot u of row k lives at [u * n + k]. Lanes that own consecutive A entries read neighbouring
// B rows (sorted columns of a row of A are clustered), so a slot load is coalesced, the B row
// pointers drop out of the dependent load chain (a_col -> slot loads), and the first kU slots
// are fetched for every A entry at once; longer rows stream their tail slots afterwards.
// ------------------------------------------------------------------------------------------------
template <typename S>
__global__ __launch_bounds__(kBlock) void k_build_sell(const uint64_t *rp, const uint32_t *col, const S *val,
                                                        uint32_t n, uint32_t w, uint32_t *scol, S *sval) {
    for (uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x; k < n; k += (uint64_t)gridDim.x * kBlock) {
        const uint64_t s = rp[k], len = rp[k + 1] - s;
        for (uint32_t u = 0; u < w; ++u) {
            const uint64_t o = (uint64_t)u * n + k;
            if (u < len) {
                scol[o] = col[s + u];
                sval[o] = val[s + u];
            } else {
                scol[o] = kSent;
                sval[o] = S(0);
            }
        }
    }
}

template <typename I, typename S, int Q, int U, bool VALS>
struct SellBatch {
    uint32_t kk[Q];
    S av[Q];
    uint32_t jj[Q][U];
    S bv[Q][U];

    __device__ __forceinline__ void load(const Args &p, I base, I a1) {
        const int lane = lane_id();
        const S *av_ = (const S *)p.a_val;
        const S *sv = (const S *)p.sell_val;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const I idx = base + (I)(q * kWave + lane);
            kk[q] = kSent;
            av[q] = S(0);
            if (idx < a1) {
                kk[q] = p.a_col[idx];
                if constexpr (VALS) av[q] = av_[idx];
            }
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                jj[q][u] = kSent;
                bv[q][u] = S(0);
                if (kk[q] != kSent && u < (int)p.sell_w) {
                    const uint32_t o = (uint32_t)u * p.sell_n + kk[q];
                    jj[q][u] = p.sell_col[o];
                    if constexpr (VALS) bv[q][u] = sv[o];
                }
            }
        }
    }

    template <typename F>
    __device__ __forceinline__ void for_each(const Args &p, F &&visit) const {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (jj[q][u] != kSent) visit(jj[q][u], av[q], bv[q][u]);
        }
        const S *sv = (const S *)p.sell_val;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            if (jj[q][U - 1] == kSent) continue;
            for (uint32_t u = U; u < p.sell_w; ++u) {
                const uint32_t o = u * p.sell_n + kk[q];
                const uint32_t j = p.sell_col[o];
                if (j == kSent) break;
                S b = S(0);
                if constexpr (VALS) b = sv[o];
                visit(j, av[q], b);
            }
        }
    }
};

template <bool SELL, typename I, typename S, bool VALS>
using BatchT = std::conditional_t<SELL, SellBatch<I, S, kQ, kU, VALS>, Batch<I, S, kQ, kU, VALS>>;

// ------------------------------------------------------------------------------------------------
// symbolic: structural nnz per output row, one wavefront per row
// ------------------------------------------------------------------------------------------------
template <typename I, bool SELL>
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
    const uint64_t WIN = (uint64_t)p.ww * 32;
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
                uint32_t c = 0, nprod = 0;
                for (I base = a0; base < a1; base += (I)(kWave * kQ)) {
                    BatchT<SELL, I, uint32_t, false> bt;
                    bt.load(p, base, a1);
                    bt.for_each(p, [&](uint32_t j, uint32_t, uint32_t) {
                        if (p.stats) ++nprod;
                        const uint64_t off = (uint64_t)j - wlo;
                        if (off < WIN) {
                            const uint32_t bit = 1u << (off & 31);
                            const uint32_t old = atomicOr(&L0[off >> 5], bit);
                            c += (old & bit) ? 0u : 1u;
                        }
                    });
                }
                const uint32_t wc = wave_sum_u32(c);
                if (p.stats && first) flops += wave_sum_u32(nprod);
                first = false;
                cnt += wc;
                wave_sync();
                if (wc)
                    for (uint32_t w = lane; w < p.ww; w += kWave) L0[w] = 0;
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
    uint32_t off_wb, off_vals, off_cols, off_sat, bytes;
};

// Per-wave LDS region: L0 ww*4 | wbase ww*2 | vals cap*vsz | cols cap*4 | sat cap/8
__host__ __device__ inline NumLayout num_layout(uint32_t ww, uint32_t cap, uint32_t vsz) {
    auto up = [](uint32_t x, uint32_t a) { return (x + a - 1) / a * a; };
    NumLayout L;
    L.off_wb = ww * 4;
    L.off_vals = up(L.off_wb + ww * 2, 16);
    L.off_cols = up(L.off_vals + cap * vsz, 16);
    L.off_sat = up(L.off_cols + cap * 4, 16);
    L.bytes = up(L.off_sat + (cap + 31) / 32 * 4, 16);
    return L;
}

template <typename Sem, typename I, bool SELL>
__global__ __launch_bounds__(kBlock) void k_numeric(Args p) {
    using S = typename Sem::S;
    using V = typename Sem::V;
    constexpr int kWpb = kBlock / kWave;
    constexpr bool kRegVals = !Sem::kOrdered;  // f64 accumulates from an ordered global walk
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    __shared__ uint32_t red[2][kWpb];

    const int lane = lane_id();
    const int wv = threadIdx.x / kWave;
    const NumLayout lay = num_layout(p.ww, p.cap, sizeof(V));
    uint8_t *region = smem8 + (size_t)wv * lay.bytes;
    uint32_t *L0 = (uint32_t *)region;
    uint16_t *wbase = (uint16_t *)(region + lay.off_wb);
    V *vals = (V *)(region + lay.off_vals);
    uint32_t *cols = (uint32_t *)(region + lay.off_cols);
    uint32_t *sat = (uint32_t *)(region + lay.off_sat);
    S *cval = (S *)p.c_val;

    if (blockIdx.x == 0 && threadIdx.x == 0) p.shards[0] = p.c_rp[p.nrows];
    for (uint32_t w = lane; w < p.ww; w += kWave) L0[w] = 0;
    wave_sync();

    const uint64_t WIN = (uint64_t)p.ww * 32;
    const uint32_t per = p.ww / kWave;  // odd: lane-contiguous word ownership is conflict-free
    const uint32_t wb0 = lane * per;
    uint32_t maxrow = 0, zrows = 0;
    const uint64_t stride = (uint64_t)gridDim.x * kWpb;
    for (uint64_t row = (uint64_t)blockIdx.x * kWpb + wv; row < p.nrows; row += stride) {
        const I a0 = (I)p.a_rp[row], a1 = (I)p.a_rp[row + 1];
        const uint64_t out_begin = p.c_rp[row];
        uint64_t out_pos = out_begin;
        uint32_t zeros = 0;
        if (a1 > a0) {
            // the common case keeps the row's whole product set in registers across both passes
            const bool single = (uint64_t)(a1 - a0) <= (uint64_t)(kWave * kQ);
            BatchT<SELL, I, S, kRegVals> bt;
            if (single) bt.load(p, a0, a1);
            auto each_product = [&](auto &&visit) {
                if (single) {
                    bt.for_each(p, visit);
                } else {
                    for (I base = a0; base < a1; base += (I)(kWave * kQ)) {
                        bt.load(p, base, a1);
                        bt.for_each(p, visit);
                    }
                }
            };
            uint64_t lo = 0, hi = p.ncols - 1;
            if (p.wide) {
                if (single) {
                    uint32_t l = 0xFFFFFFFFu, h = 0;
                    bt.for_each(p, [&](uint32_t j, S, S) {
                        l = min(l, j);
                        h = max(h, j);
                    });
                    l = wave_min_u32(l);
                    h = wave_max_u32(h);
                    lo = l;
                    hi = h;
                    if (l > h) {
                        lo = 1;
                        hi = 0;
                    }
                } else {
                    row_span<I>(p, a0, a1, lo, hi);
                }
            }
            for (uint64_t wlo = lo & ~31ull; wlo <= hi; wlo += WIN) {
                // 1. column bitmap of the window
                each_product([&](uint32_t j, S, S) {
                    const uint64_t off = (uint64_t)j - wlo;
                    if (off < WIN) atomicOr(&L0[off >> 5], 1u << (off & 31));
                });
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
                    for (uint32_t t = lane; t < nch; t += kWave) vals[t] = V(0);
                    for (uint32_t t = lane; t < (nch + 31) / 32; t += kWave) sat[t] = 0;
                    wave_sync();
                    // 3. values + the column of every rank (duplicates store the same column)
                    auto rank_of = [&](uint32_t j, uint32_t &r) -> bool {
                        const uint64_t off = (uint64_t)j - wlo;
                        if (off >= WIN) return false;
                        const uint32_t w = (uint32_t)(off >> 5);
                        r = (uint32_t)wbase[w] + __popc(L0[w] & ((1u << (off & 31)) - 1u)) - r0;
                        return r < nch;
                    };
                    if constexpr (Sem::kOrdered) {
                        traverse_ordered<I, S>(p, a0, a1, [&](uint32_t j, S a, S b) {
                            uint32_t r;
                            if (rank_of(j, r)) {
                                Sem::acc(vals, sat, r, Sem::prod(a, b));
                                cols[r] = j;
                            }
                        });
                    } else {
                        each_product([&](uint32_t j, S a, S b) {
                            uint32_t r;
                            if (rank_of(j, r)) {
                                Sem::acc(vals, sat, r, Sem::prod(a, b));
                                cols[r] = j;
                            }
                        });
                    }
                    wave_sync();
                    // 4. emit at the row's slice, coalesced
                    for (uint32_t t = lane; t < nch; t += kWave) {
                        const S v = Sem::finish(vals, sat, t);
                        zeros += Sem::is_zero(v) ? 1u : 0u;
                        p.c_col[out_pos + t] = cols[t];
                        cval[out_pos + t] = v;
                    }
                    out_pos += nch;
                    wave_sync();
                }
                for (uint32_t q = 0; q < per; ++q) L0[wb0 + q] = 0;
                wave_sync();
            }
        }
        const uint32_t rz = wave_sum_u32(zeros);
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
