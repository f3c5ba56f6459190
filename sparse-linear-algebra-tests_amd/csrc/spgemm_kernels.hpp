// spgemm_kernels.hpp — gfx950 device code for row-wise (Gustavson) SpGEMM C = A·B.
//
// One 64-lane wavefront owns one output row at a time (grid-stride over rows). A row's column set
// is built in an LDS *bitmap* over a window of columns (ww words = 32·ww columns); the rank of a
// column among the row's distinct columns is wbase[word] + popcount(bits below it), so the output
// is emitted already sorted by column — the reference's `nz_cols.sort_unstable()`
// (src/graph_csr.rs:331,449) becomes a bitmap prefix scan. Values accumulate in LDS indexed by
// rank (u64 for u32/Sat64, f64 for f64). Rows wider than one window iterate windows; rows with
// more distinct columns than the LDS value capacity iterate rank chunks (the MAGNUS "fine-level"
// split of a long row into cache-sized column chunks, done per LDS window here).
//
// Passes (the reference's matmul_par structure, src/graph_csr.rs:360-476):
//   k_symbolic : structural nnz per row (bitmap popcount of newly set bits)
//   (scan)     : hipcub inclusive scan -> C.row_ptr
//   k_numeric  : bitmap -> ranks -> values -> sorted, zero-free emit into C's row slice
//   k_compact  : only if explicit zeros were dropped (f64 cancellation or zero inputs)
//
// Semantics kept bit-exact (SURVEY.md §8(a) rules 1-4):
//   u32   : product clamped to u32::MAX, summed exactly in u64, clamped at emit
//           == sadd/smul (src/graph_csr.rs:29-37) because all values are non-negative.
//   Sat64 : u64 LDS atomics; a wrap of the running sum sets a per-slot saturation bit
//           (wraps happen iff the exact sum >= 2^64) == Sat64 (src/graph_sprs.rs:29-51).
//   f64   : A's row entries are walked in order, lanes spread over one B row (distinct
//           columns), non-atomic RMW with __dmul_rn/__dadd_rn: the left fold from 0.0 in A-row
//           order of linalg/src/csr.rs:325-337, bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace slat {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kShards = 64;       // sharded status words (avoid one hot atomic address)
constexpr int kShardStride = 4;   // [0] total nnz (shard 0 only), [1] max row nnz, [2] rows with drops, [3] flops

enum : uint32_t { MODE_LANE_PER_A = 0, MODE_WAVE_PER_A = 1 };

struct Args {
    const uint64_t *a_rp;
    const uint32_t *a_col;
    const void *a_val;
    const uint64_t *b_rp;
    const uint32_t *b_col;
    const void *b_val;
    uint64_t nrows, ncols;
    uint32_t ww;    // bitmap words per window (64 * odd)
    uint32_t cap;   // rank-chunk capacity (values per LDS pass)
    uint32_t wide;  // 0: one window at column 0 covers all columns; 1: windows from the row's min col
    uint32_t stats; // count products into shard[3]
    uint64_t *counts;   // symbolic: structural nnz per row; numeric: actual nnz per row
    uint64_t *c_rp;     // C.row_ptr (n+1)
    uint32_t *c_col;
    void *c_val;
    unsigned long long *shards;
};

// ------------------------------------------------------------------------------------------------
// value semirings
// ------------------------------------------------------------------------------------------------
struct SemU32 {
    using S = uint32_t;
    using Acc = unsigned long long;
    static constexpr bool kOrdered = false;
    static constexpr bool kSat = false;
    __device__ static __forceinline__ void acc(Acc *vals, uint32_t *, uint32_t r, S a, S b) {
        unsigned long long p = (unsigned long long)a * (unsigned long long)b;
        p = p > 0xFFFFFFFFull ? 0xFFFFFFFFull : p;  // Saturating<u32> product
        atomicAdd(&vals[r], p);                    // exact: < 2^32 terms of < 2^32
    }
    __device__ static __forceinline__ S finish(const Acc *vals, const uint32_t *, uint32_t t) {
        Acc v = vals[t];
        return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (S)v;
    }
    __device__ static __forceinline__ bool nonzero(S v) { return v != 0; }
};

struct SemSat64 {
    using S = unsigned long long;
    using Acc = unsigned long long;
    static constexpr bool kOrdered = false;
    static constexpr bool kSat = true;
    __device__ static __forceinline__ void acc(Acc *vals, uint32_t *sat, uint32_t r, S a, S b) {
        unsigned long long p = a * b;
        if (__umul64hi(a, b) != 0) p = ~0ull;  // Saturating<u64> product
        unsigned long long old = atomicAdd(&vals[r], p);
        if (old + p < old) atomicOr(&sat[r >> 5], 1u << (r & 31));  // running sum wrapped
    }
    __device__ static __forceinline__ S finish(const Acc *vals, const uint32_t *sat, uint32_t t) {
        return ((sat[t >> 5] >> (t & 31)) & 1u) ? ~0ull : vals[t];
    }
    __device__ static __forceinline__ bool nonzero(S v) { return v != 0; }
};

struct SemF64 {
    using S = double;
    using Acc = double;
    static constexpr bool kOrdered = true;
    static constexpr bool kSat = false;
    __device__ static __forceinline__ void acc(Acc *vals, uint32_t *, uint32_t r, S a, S b) {
        vals[r] = __dadd_rn(vals[r], __dmul_rn(a, b));  // no FMA contraction: Rust's a*b then +
    }
    __device__ static __forceinline__ S finish(const Acc *vals, const uint32_t *, uint32_t t) { return vals[t]; }
    __device__ static __forceinline__ bool nonzero(S v) { return v != 0.0; }
};

// ------------------------------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// LDS written by some lanes and read by others within the same wave: DS instructions of one wave
// execute in order; the fences stop the compiler from reordering across the hand-off.
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
        uint32_t t = __shfl_up(v, d);
        if (lane >= d) v += t;
    }
    return v - x;
}

__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    uint32_t lo = readlane_u32((uint32_t)v, l), hi = readlane_u32((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
template <typename S>
__device__ __forceinline__ S readlane_val(S v, int l) {
    if constexpr (sizeof(S) == 4) {
        return (S)readlane_u32((uint32_t)v, l);
    } else {
        uint64_t u = __builtin_bit_cast(uint64_t, v);
        return __builtin_bit_cast(S, readlane_u64(u, l));
    }
}

// ------------------------------------------------------------------------------------------------
// product traversal of one output row: visit(j, a_ik, b_kj) for every k in A_i, j in B_k
// ------------------------------------------------------------------------------------------------
// MODE_LANE_PER_A: each lane owns one A entry and walks its (short) B row. Any order.
// MODE_WAVE_PER_A: A entries in order; lanes spread over one B row. Ordered per column.
template <uint32_t MODE, bool VALS, typename S, typename F>
__device__ __forceinline__ void traverse(const Args &p, uint64_t a0, uint64_t a1, F &&visit) {
    const int lane = lane_id();
    const S *av_ = (const S *)p.a_val;
    const S *bv_ = (const S *)p.b_val;
    for (uint64_t base = a0; base < a1; base += kWave) {
        const uint64_t idx = base + lane;
        uint64_t bs = 0, be = 0;
        S av = S(0);
        if (idx < a1) {
            const uint32_t k = p.a_col[idx];
            if constexpr (VALS) av = av_[idx];
            bs = p.b_rp[k];
            be = p.b_rp[k + 1];
        }
        if constexpr (MODE == MODE_LANE_PER_A) {
            for (uint64_t jdx = bs; jdx < be; ++jdx) {
                S bv = S(0);
                if constexpr (VALS) bv = bv_[jdx];
                visit(p.b_col[jdx], av, bv);
            }
        } else {
            const int cnt = (int)min<uint64_t>((uint64_t)kWave, a1 - base);
            for (int t = 0; t < cnt; ++t) {
                const uint64_t s = readlane_u64(bs, t), e = readlane_u64(be, t);
                S a = S(0);
                if constexpr (VALS) a = readlane_val(av, t);
                for (uint64_t jdx = s + lane; jdx < e; jdx += kWave) {
                    S bv = S(0);
                    if constexpr (VALS) bv = bv_[jdx];
                    visit(p.b_col[jdx], a, bv);
                }
            }
        }
    }
}

// Column span [lo, hi] of row i of A·B from B's row ends (B rows are sorted). lo > hi if empty.
__device__ __forceinline__ void row_span(const Args &p, uint64_t a0, uint64_t a1, uint64_t &lo, uint64_t &hi) {
    const int lane = lane_id();
    uint32_t l = 0xFFFFFFFFu, h = 0;
    for (uint64_t idx = a0 + lane; idx < a1; idx += kWave) {
        const uint32_t k = p.a_col[idx];
        const uint64_t bs = p.b_rp[k], be = p.b_rp[k + 1];
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
// symbolic: structural nnz per output row
// ------------------------------------------------------------------------------------------------
template <uint32_t MODE>
__global__ __launch_bounds__(kBlock) void k_symbolic(Args p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
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
    const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t row = (uint64_t)blockIdx.x * kWavesPerBlock + wv; row < p.nrows; row += stride) {
        const uint64_t a0 = p.a_rp[row], a1 = p.a_rp[row + 1];
        uint64_t cnt = 0;
        if (a1 > a0) {
            uint64_t lo = 0, hi = p.ncols - 1;
            if (p.wide) row_span(p, a0, a1, lo, hi);
            for (uint64_t wlo = lo & ~31ull; wlo <= hi; wlo += WIN) {
                uint32_t c = 0, nprod = 0;
                traverse<MODE, false, uint32_t>(p, a0, a1, [&](uint32_t j, uint32_t, uint32_t) {
                    const uint64_t off = (uint64_t)j - wlo;
                    ++nprod;
                    if (off < WIN) {
                        const uint32_t bit = 1u << (off & 31);
                        const uint32_t old = atomicOr(&L0[off >> 5], bit);
                        c += (old & bit) ? 0u : 1u;
                    }
                });
                const uint32_t wc = wave_sum_u32(c);
                if (p.stats && wlo == (lo & ~31ull)) flops += wave_sum_u32(nprod);
                cnt += wc;
                wave_sync();
                if (wc) for (uint32_t w = lane; w < p.ww; w += kWave) L0[w] = 0;
                wave_sync();
            }
        }
        if (lane == 0) p.counts[row] = cnt;
    }
    if (p.stats && lane == 0 && flops) atomicAdd(&p.shards[((blockIdx.x * kWavesPerBlock + wv) % kShards) * kShardStride + 3], flops);
}

// ------------------------------------------------------------------------------------------------
// numeric: values + sorted emit
// ------------------------------------------------------------------------------------------------
// Per-wave LDS region (bytes): L0 ww*4 | wbase ww*4 | vals cap*8 | cols cap*4 | sat cap/8 (pad 16)
__host__ __device__ inline size_t numeric_wave_lds(uint32_t ww, uint32_t cap) {
    size_t b = (size_t)ww * 8 + (size_t)cap * 8 + (size_t)cap * 4 + (size_t)((cap + 31) / 32) * 4;
    return (b + 15) & ~(size_t)15;
}

template <typename Sem, uint32_t BUILD_MODE, uint32_t ACC_MODE>
__global__ __launch_bounds__(kBlock) void k_numeric(Args p) {
    using S = typename Sem::S;
    using Acc = typename Sem::Acc;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    __shared__ uint32_t red[2][kWavesPerBlock];
    const int lane = lane_id();
    const int wv = threadIdx.x / kWave;
    uint8_t *region = (uint8_t *)smem + (size_t)wv * numeric_wave_lds(p.ww, p.cap);
    uint32_t *L0 = (uint32_t *)region;
    uint32_t *wbase = L0 + p.ww;
    Acc *vals = (Acc *)(wbase + p.ww);
    uint32_t *cols = (uint32_t *)(vals + p.cap);
    uint32_t *sat = cols + p.cap;
    S *cval = (S *)p.c_val;

    if (blockIdx.x == 0 && threadIdx.x == 0) p.shards[0] = p.c_rp[p.nrows];
    for (uint32_t w = lane; w < p.ww; w += kWave) L0[w] = 0;
    wave_sync();

    const uint64_t WIN = (uint64_t)p.ww * 32;
    const uint32_t per = p.ww / kWave;  // odd: conflict-free lane-contiguous word ownership
    const uint32_t wb = lane * per;
    uint32_t maxrow = 0, drops = 0;
    const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t row = (uint64_t)blockIdx.x * kWavesPerBlock + wv; row < p.nrows; row += stride) {
        const uint64_t a0 = p.a_rp[row], a1 = p.a_rp[row + 1];
        const uint64_t out_begin = p.c_rp[row];
        uint64_t out_pos = out_begin;
        if (a1 > a0) {
            uint64_t lo = 0, hi = p.ncols - 1;
            if (p.wide) row_span(p, a0, a1, lo, hi);
            for (uint64_t wlo = lo & ~31ull; wlo <= hi; wlo += WIN) {
                // 1. column bitmap of this window
                traverse<BUILD_MODE, false, uint32_t>(p, a0, a1, [&](uint32_t j, uint32_t, uint32_t) {
                    const uint64_t off = (uint64_t)j - wlo;
                    if (off < WIN) atomicOr(&L0[off >> 5], 1u << (off & 31));
                });
                wave_sync();
                // 2. word ranks: lane owns words [wb, wb+per)
                uint32_t lc = 0;
                for (uint32_t q = 0; q < per; ++q) lc += __popc(L0[wb + q]);
                const uint32_t ex = wave_excl_scan_u32(lc);
                const uint32_t wcnt = readlane_u32(ex + lc, kWave - 1);
                if (wcnt == 0) continue;  // bitmap is all zero: nothing to clear
                {
                    uint32_t run = ex;
                    for (uint32_t q = 0; q < per; ++q) {
                        wbase[wb + q] = run;
                        run += __popc(L0[wb + q]);
                    }
                }
                wave_sync();
                // 3. values, one rank chunk at a time
                for (uint32_t r0 = 0; r0 < wcnt; r0 += p.cap) {
                    const uint32_t nch = min(p.cap, wcnt - r0);
                    for (uint32_t t = lane; t < nch; t += kWave) vals[t] = Acc(0);
                    if constexpr (Sem::kSat)
                        for (uint32_t t = lane; t < (nch + 31) / 32; t += kWave) sat[t] = 0;
                    wave_sync();
                    traverse<ACC_MODE, true, S>(p, a0, a1, [&](uint32_t j, S a, S b) {
                        const uint64_t off = (uint64_t)j - wlo;
                        if (off < WIN) {
                            const uint32_t w = (uint32_t)(off >> 5);
                            const uint32_t below = L0[w] & ((1u << (off & 31)) - 1u);
                            const uint32_t r = wbase[w] + __popc(below) - r0;
                            if (r < nch) Sem::acc(vals, sat, r, a, b);
                        }
                    });
                    // sorted column list of the chunk
                    {
                        uint32_t run = ex;
                        for (uint32_t q = 0; q < per; ++q) {
                            uint32_t bits = L0[wb + q];
                            const uint32_t pc = __popc(bits);
                            if (run + pc > r0 && run < r0 + nch) {
                                const uint32_t colbase = (uint32_t)(wlo + 32ull * (wb + q));
                                while (bits) {
                                    const uint32_t b = __builtin_ctz(bits);
                                    bits &= bits - 1;
                                    const uint32_t r = run - r0;
                                    if (r < nch) cols[r] = colbase + b;
                                    ++run;
                                }
                            } else {
                                run += pc;
                            }
                        }
                    }
                    wave_sync();
                    // 4. emit, dropping exact zeros (compacted within the row)
                    for (uint32_t t0 = 0; t0 < nch; t0 += kWave) {
                        const uint32_t t = t0 + lane;
                        const bool act = t < nch;
                        S v = S(0);
                        if (act) v = Sem::finish(vals, sat, t);
                        const bool nz = act && Sem::nonzero(v);
                        const unsigned long long m = __ballot(nz);
                        const uint32_t off = __popcll(m & ((1ull << lane) - 1ull));
                        if (nz) {
                            p.c_col[out_pos + off] = cols[t];
                            cval[out_pos + off] = v;
                        }
                        out_pos += __popcll(m);
                    }
                    wave_sync();
                }
                for (uint32_t w = lane; w < p.ww; w += kWave) L0[w] = 0;
                wave_sync();
            }
        }
        const uint64_t got = out_pos - out_begin;
        if (lane == 0) p.counts[row] = got;
        maxrow = max(maxrow, (uint32_t)min<uint64_t>(got, 0xFFFFFFFFull));
        drops += (got != p.c_rp[row + 1] - out_begin) ? 1u : 0u;
    }
    if (lane == 0) {
        red[0][wv] = maxrow;
        red[1][wv] = drops;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t m = 0, d = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) {
            m = max(m, red[0][w]);
            d += red[1][w];
        }
        unsigned long long *sh = p.shards + (blockIdx.x % kShards) * kShardStride;
        if (m) atomicMax(&sh[1], (unsigned long long)m);
        if (d) atomicAdd(&sh[2], (unsigned long long)d);
    }
}

// ------------------------------------------------------------------------------------------------
// compaction (rare): rows lost explicit zeros; move row slices to the exact-size arrays
// ------------------------------------------------------------------------------------------------
template <typename S>
__global__ __launch_bounds__(kBlock) void k_compact(const uint64_t *old_rp, const uint64_t *new_rp, uint64_t nrows,
                                                    const uint32_t *old_col, const S *old_val, uint32_t *new_col,
                                                    S *new_val) {
    const int lane = lane_id();
    const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t row = (uint64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave; row < nrows; row += stride) {
        const uint64_t s = old_rp[row], d = new_rp[row], n = new_rp[row + 1] - d;
        for (uint64_t t = lane; t < n; t += kWave) {
            new_col[d + t] = old_col[s + t];
            new_val[d + t] = old_val[s + t];
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
