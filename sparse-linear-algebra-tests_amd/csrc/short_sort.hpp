// short_sort.hpp — the short-row category of wide launches by in-register sorting (gfx950).
//
// MAGNUS's small-row category (the reference's MagnusMatrix row categorisation, src/graph_sprs.rs;
// SURVEY.md §8 row "wide / power-law inputs") for the rows whose products fit one wave: a batch of
// consecutive rows of a 64-row tile whose B rows contribute <= 64 ELL groups (4 columns each) is
// loaded ONE GROUP PER LANE, i.e. 256 (key, product) pairs in registers, key = (local row << cb) |
// column. A bitonic network over the wave (intra-lane swaps and lane exchanges by DPP / ds_swizzle)
// sorts them; equal keys are then adjacent, so
//   symbolic: a row's nnz = the number of run ends with its local row,
//   numeric : a run's sum is a segmented scan (stopped at the longest run), and the output index of
//             a run is the batch's first C.row_ptr + the number of run ends before it (rows are
//             contiguous in C and the keys sort by (row, column)).
// No LDS hash table, no probe loops, no rank-by-count: the previous batched hash category
// (k_*_short) waits on chains of LDS compare-and-swap round trips per group.
//
// Per row the batch formation needs the row's ELL group count: the symbolic kernel computes it
// from the tile's entries (coalesced a_col loads, a wave prefix of the group counts read at each
// row's ends, as k_symbolic_short's tile_groups) and stores it for the numeric kernel.
#pragma once
#include "spgemm_kernels.hpp"

namespace slat {

constexpr uint32_t kSortG = 64;     // ELL groups per batch: one per lane
constexpr uint32_t kSortEnt = 256;  // A entries per batch: kRegQ per lane

// key of element i + 1 (kSent past the end)
__device__ __forceinline__ void next_keys(const uint32_t (&k)[4], uint32_t (&nk)[4]) {
    uint32_t n0 = (uint32_t)__shfl_down((int)k[0], 1);
    if (lane_id() == kWave - 1) n0 = kSent;
    nk[0] = k[1];
    nk[1] = k[2];
    nk[2] = k[3];
    nk[3] = n0;
}

// the sums the runs of equal keys accumulate in: exact u64 sums of clamped u32 products, saturating
// u64 (every term is non-negative, so min(sum, MAX) in any order), f64 in any order
template <typename Sem>
struct SortAcc;
template <>
struct SortAcc<SemU32> {
    using T = unsigned long long;
    __device__ static __forceinline__ T add(T a, T b) { return a + b; }
    __device__ static __forceinline__ uint32_t fin(T v) { return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)v; }
};
template <>
struct SortAcc<SemSat64> {
    using T = unsigned long long;
    __device__ static __forceinline__ T add(T a, T b) {
        const T s = a + b;
        return s < a ? ~0ull : s;
    }
    __device__ static __forceinline__ T fin(T v) { return v; }
};
template <>
struct SortAcc<SemF64Any> {
    using T = double;
    __device__ static __forceinline__ T add(T a, T b) { return __dadd_rn(a, b); }
    __device__ static __forceinline__ T fin(T v) { return v; }
};

// inclusive sums over runs of equal keys of the sorted wave: Hillis-Steele over distances 1, 2, 4, ...
// (the element D before i has the same key only inside one run), stopped at the first distance no
// key repeats at: every run is then at most that long
template <typename Acc, typename T>
__device__ __forceinline__ void seg_sums(const uint32_t (&k)[4], T (&s)[4]) {
    const uint32_t lane = (uint32_t)lane_id();
    bool go = true;
    sfor<8>([&](auto Dl) {
        constexpr int D = 1 << decltype(Dl)::value;
        if (!go) return;
        uint32_t pk[4];
        T ps[4];
        sfor<4>([&](auto E) {
            constexpr int e = decltype(E)::value;
            if constexpr (D < 4) {
                if constexpr (e >= D) {
                    pk[e] = k[e - D];
                    ps[e] = s[e - D];
                } else {
                    pk[e] = (uint32_t)__shfl_up((int)k[e + 4 - D], 1);
                    ps[e] = __shfl_up(s[e + 4 - D], 1);
                }
            } else {
                pk[e] = (uint32_t)__shfl_up((int)k[e], D / 4);
                ps[e] = __shfl_up(s[e], D / 4);
            }
        });
        bool any = false;
        sfor<4>([&](auto E) {
            constexpr int e = decltype(E)::value;
            const bool m = lane * 4 + e >= (uint32_t)D && k[e] != kSent && pk[e] == k[e];
            s[e] = m ? Acc::add(s[e], ps[e]) : s[e];
            any |= m;
        });
        go = __ballot(any) != 0;
    });
}

// batch of short rows b..e-1 of the tile (wave-uniform): the first short row at or after b, then the
// rows while groups <= kSortG and entries <= kSortEnt (one row per batch without composite keys)
__device__ __forceinline__ uint32_t sort_batch_end(uint32_t b, uint32_t nt, bool shortj, uint32_t gj, uint64_t lj,
                                                   uint32_t cb) {
    const uint32_t lane = (uint32_t)lane_id();
    const bool inb = lane >= b;
    const uint32_t pg = wave_incl_scan(inb ? min(gj, 1u << 20) : 0u, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    const uint32_t pl = wave_incl_scan(inb ? (uint32_t)min<uint64_t>(lj, 1u << 20) : 0u, 0u,
                                       [](uint32_t x, uint32_t y) { return x + y; });
    const unsigned long long stop =
        __ballot(inb && (!shortj || pg > kSortG || pl > kSortEnt || (cb == 0 && lane > b)));
    return stop ? (uint32_t)__builtin_ctzll(stop) : nt;  // > b: row b is short
}

// the batch's A entries: local row (marks: each row's first entry, a running max), column of B
// (kSent when out of range), value, ELL group count; then the (entry, group) pairs staged one per
// slot: tk = B row | group << 24 (B rows < 2^24 with the ELL copy), tl = local row, ta = A value.
// Returns the number of groups (<= kSortG by the batch formation; clamped for safety).
template <bool VALS, typename S>
__device__ __forceinline__ uint32_t sort_stage(const Args &p, uint64_t A0, uint32_t nent, uint32_t b, uint32_t e,
                                               bool inb_row, uint64_t A0j, uint64_t lj, uint32_t *marks, uint32_t *tk,
                                               uint32_t *tl, S *ta) {
    const uint32_t lane = (uint32_t)lane_id();
    if (inb_row && lj > 0) atomicMax(&marks[(uint32_t)(A0j - A0)], lane - b + 1);
    (void)e;
    wave_sync();
    uint32_t kq[kRegQ], lq[kRegQ], ng[kRegQ], pos[kRegQ];
    S aq[kRegQ];
    uint32_t carry = 0;
    sfor<kRegQ>([&](auto Q) {
        const uint32_t i = Q * kWave + lane;
        const uint32_t mk = i < nent ? marks[i] : 0u;
        const uint32_t run = max(wave_incl_scan(mk, 0u, [](uint32_t x, uint32_t y) { return max(x, y); }), carry);
        carry = readlane_u32(run, kWave - 1);
        lq[Q] = run - 1;
        kq[Q] = kSent;
        aq[Q] = S(0);
        if (i < nent) {
            kq[Q] = p.a_col[A0 + i];
            if constexpr (VALS) aq[Q] = ((const S *)p.a_val)[A0 + i];
            marks[i] = 0;
        }
    });
    uint32_t mxg = 0;
    sfor<kRegQ>([&](auto Q) {
        if (kq[Q] >= p.b_nrows) kq[Q] = kSent;
        ng[Q] = kq[Q] != kSent ? p.ell_ng[kq[Q]] : 0u;
        mxg = max(mxg, ng[Q]);
    });
    mxg = wave_max_u32(mxg);
    uint32_t tot = 0;
    sfor<kRegQ>([&](auto Q) {
        const uint32_t incl = wave_incl_scan(ng[Q], 0u, [](uint32_t x, uint32_t y) { return x + y; });
        pos[Q] = tot + incl - ng[Q];
        tot += readlane_u32(incl, kWave - 1);
    });
    for (uint32_t t = 0; t < mxg; ++t)
        sfor<kRegQ>([&](auto Q) {
            const uint32_t g = pos[Q] + t;
            if (t < ng[Q] && g < kSortG) {
                tk[g] = kq[Q] | (t << 24);
                tl[g] = lq[Q];
                if constexpr (VALS) ta[g] = aq[Q];
            }
        });
    wave_sync();
    return min(tot, kSortG);
}

// LDS per wave of k_symbolic_sort: prefix window u32[256] | marks u32[256] | tk u32[64] | tl u32[64]
// | row ends u32[64]
__host__ __device__ constexpr uint32_t sort_sym_bytes() { return (256 + 256 + 3 * kWave) * 4; }

__global__ __launch_bounds__(kBlock) void k_symbolic_sort(Args p) {
    constexpr int kWpb = kBlock / kWave;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t lane = (uint32_t)lane_id();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    uint32_t *pf = smem + (size_t)wv * (sort_sym_bytes() / 4);
    uint32_t *marks = pf + 256, *tk = marks + 256, *tl = tk + kWave, *rend = tl + kWave;
    uint32_t *gout = (uint32_t *)p.rbound;  // written here: the numeric kernel's batch formation
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) p.c_rp[0] = 0;
        if (threadIdx.x < kShards) {
            p.shards[threadIdx.x * kShardStride + 1] = 0;
            p.shards[threadIdx.x * kShardStride + 2] = 0;
        }
    }
    for (uint32_t w = lane; w < 256; w += kWave) marks[w] = 0;
    rend[lane] = 0;
    wave_sync();
    const uint32_t cb = p.cbits;
    unsigned long long flops = 0;
    const uint64_t ntiles = (p.nrows + kWave - 1) / kWave;
    for (uint64_t tile = (uint64_t)blockIdx.x * kWpb + wv; tile < ntiles; tile += (uint64_t)gridDim.x * kWpb) {
        const uint64_t r0 = tile * kWave, r = r0 + lane;
        const uint32_t nt = (uint32_t)min<uint64_t>(kWave, p.nrows - r0);
        uint64_t A0j = 0, A1j = 0;
        if (lane < nt) {
            A0j = p.a_rp[r];
            A1j = p.a_rp[r + 1];
        }
        // ELL groups per row: exclusive prefix of the group counts over the tile's entries (mod 2^32:
        // only rows of <= kSortEnt entries use the difference), read at each row's first and end
        const uint64_t T0 = readlane_u64(A0j, 0), T1 = readlane_u64(A1j, (int)nt - 1);
        uint32_t gs = 0, ge = 0, run = 0;
        for (uint64_t c0 = T0; c0 < T1; c0 += 256) {
            uint32_t kk[4], g[4];
            sfor<4>([&](auto Q) {
                const uint64_t idx = c0 + Q * kWave + lane;
                kk[Q] = idx < T1 ? p.a_col[idx] : kSent;
            });
            sfor<4>([&](auto Q) { g[Q] = kk[Q] < p.b_nrows ? (uint32_t)p.ell_ng[kk[Q]] : 0u; });
            sfor<4>([&](auto Q) {
                const uint32_t incl = wave_incl_scan(g[Q], 0u, [](uint32_t x, uint32_t y) { return x + y; });
                pf[Q * kWave + lane] = run + incl - g[Q];
                run += readlane_u32(incl, kWave - 1);
            });
            wave_sync();
            if (A0j >= c0 && A0j < T1 && A0j - c0 < 256) gs = pf[A0j - c0];
            if (A1j >= c0 && A1j < T1 && A1j - c0 < 256) ge = pf[A1j - c0];
            wave_sync();
        }
        if (A0j >= T1) gs = run;
        if (A1j >= T1) ge = run;
        const uint32_t gj = lane < nt ? ge - gs : 0u;
        if (lane < nt) gout[r] = gj;
        const uint64_t lj = A1j - A0j;
        const bool fatj = lane < nt && fat_row(p, r);
        const bool shortj = lane < nt && gj <= kSortG && lj <= kSortEnt && !fatj;
        list_rows(p, lane < nt && !shortj && !fatj, r);
        const unsigned long long shortm = __ballot(shortj);
        uint32_t b = 0;
        for (;;) {
            const unsigned long long m = b < (uint32_t)kWave ? (shortm >> b) << b : 0ull;
            if (!m) break;
            b = (uint32_t)__builtin_ctzll(m);
            const uint32_t e = sort_batch_end(b, nt, shortj, gj, lj, cb);
            const uint64_t A0 = readlane_u64(A0j, (int)b), A1 = readlane_u64(A1j, (int)(e - 1));
            const bool inb = lane >= b && lane < e;
            const uint32_t G = sort_stage<false, uint32_t>(p, A0, (uint32_t)(A1 - A0), b, e, inb, A0j, lj, marks, tk,
                                                           tl, nullptr);
            uint32_t k[4] = {kSent, kSent, kSent, kSent}, dummy[4];
            if (lane < G) {
                const uint32_t tw = tk[lane];
                const uint4 c = ell_cols(p, tw & 0xFFFFFFu, tw >> 24);
                const uint32_t hi = tl[lane] << cb;
                k[0] = c.x != kSent ? (hi | c.x) : kSent;
                k[1] = c.y != kSent ? (hi | c.y) : kSent;
                k[2] = c.z != kSent ? (hi | c.z) : kSent;
                k[3] = c.w != kSent ? (hi | c.w) : kSent;
            }
            if (p.stats) flops += wave_sum_u32((k[0] != kSent) + (k[1] != kSent) + (k[2] != kSent) + (k[3] != kSent));
            wave_sort256<false, uint32_t>(k, dummy);
            uint32_t nk[4];
            next_keys(k, nk);
            bool tail[4];
            uint32_t tc = 0;
            sfor<4>([&](auto E) {
                tail[E] = k[E] != kSent && nk[E] != k[E];
                tc += tail[E] ? 1u : 0u;
            });
            uint32_t o = wave_excl_scan_u32(tc);
            sfor<4>([&](auto E) {
                if (tail[E]) {
                    ++o;  // inclusive count of run ends
                    const uint32_t lr = cb ? k[E] >> cb : 0u;
                    if (nk[E] == kSent || (cb ? nk[E] >> cb : 0u) != lr) rend[lr] = o;
                }
            });
            wave_sync();
            const uint32_t x = inb ? rend[lane - b] : 0u;
            const uint32_t incl = wave_incl_scan(x, 0u, [](uint32_t u, uint32_t v) { return max(u, v); });
            uint32_t pre = (uint32_t)__shfl_up((int)incl, 1);
            if (lane == 0) pre = 0;
            if (inb) {
                p.counts[r] = x ? x - pre : 0u;
                rend[lane - b] = 0;
            }
            wave_sync();
            b = e;
        }
    }
    if (p.stats && lane == 0 && flops)
        atomicAdd(&p.shards[((blockIdx.x * kWpb + wv) % kShards) * kShardStride + 3], flops);
}

// LDS per wave of k_numeric_sort: marks u32[256] | tk u32[64] | tl u32[64] | zero counts u32[64] |
// A values S[64]
template <typename Sem>
__host__ __device__ constexpr uint32_t sort_num_bytes() {
    return (256 + 3 * kWave) * 4 + kWave * (uint32_t)sizeof(typename Sem::S);
}

template <typename Sem>
__global__ __launch_bounds__(kBlock) void k_numeric_sort(Args p) {
    using S = typename Sem::S;
    using P = typename Sem::P;
    using Acc = SortAcc<Sem>;
    using T = typename Acc::T;
    constexpr int kWpb = kBlock / kWave;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    const uint32_t lane = (uint32_t)lane_id();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    uint32_t *marks = (uint32_t *)(smem8 + (size_t)wv * sort_num_bytes<Sem>());
    uint32_t *tk = marks + 256, *tl = tk + kWave, *zc = tl + kWave;
    S *ta = (S *)(zc + kWave);
    for (uint32_t w = lane; w < 256; w += kWave) marks[w] = 0;
    zc[lane] = 0;
    wave_sync();
    // pattern B (every B value equal): no B-value loads (as k_numeric_short)
    uint32_t bvmax = 0;
    bool buni = false;
    if constexpr (Sem::kNarrowable)
        if (p.b_vmax) {
            const unsigned long long v = ((volatile unsigned long long *)p.b_vmax)[kVMaxWord];
            const unsigned long long vi = ((volatile unsigned long long *)p.b_vmax)[kVMinInvWord];
            if ((uint32_t)(v >> 32) == p.epoch) {
                bvmax = (uint32_t)v;
                buni = (uint32_t)(vi >> 32) == p.epoch && ~(uint32_t)vi == bvmax;
            }
        }
    const S bv0 = (S)bvmax;
    S *cval = (S *)p.c_val;
    uint32_t zrows = 0;
    const uint32_t cb = p.cbits;
    const uint32_t cmask = cb ? (1u << cb) - 1 : 0xFFFFFFFFu;
    const uint64_t ntiles = (p.nrows + kWave - 1) / kWave;
    for (uint64_t tile = (uint64_t)blockIdx.x * kWpb + wv; tile < ntiles; tile += (uint64_t)gridDim.x * kWpb) {
        const uint64_t r0 = tile * kWave, r = r0 + lane;
        const uint32_t nt = (uint32_t)min<uint64_t>(kWave, p.nrows - r0);
        uint64_t A0j = 0, A1j = 0, obj = 0, oej = 0;
        uint32_t gj = 0;
        if (lane < nt) {
            A0j = p.a_rp[r];
            A1j = p.a_rp[r + 1];
            obj = p.c_rp[r];
            oej = p.c_rp[r + 1];
            gj = p.rbound[r];
        }
        const uint64_t lj = A1j - A0j, uj = oej - obj;
        const bool fatj = lane < nt && fat_row(p, r);
        const bool shortj = lane < nt && gj <= kSortG && lj <= kSortEnt && !fatj;
        list_rows(p, lane < nt && !shortj && !fatj, r);  // the window launch's rows
        const unsigned long long shortm = __ballot(shortj);
        uint32_t b = 0;
        for (;;) {
            const unsigned long long m = b < (uint32_t)kWave ? (shortm >> b) << b : 0ull;
            if (!m) break;
            b = (uint32_t)__builtin_ctzll(m);
            const uint32_t e = sort_batch_end(b, nt, shortj, gj, lj, cb);
            const uint64_t A0 = readlane_u64(A0j, (int)b), A1 = readlane_u64(A1j, (int)(e - 1));
            const uint64_t OB = readlane_u64(obj, (int)b);
            const uint64_t lim = readlane_u64(oej, (int)(e - 1)) - OB;  // the batch's outputs
            const bool inb = lane >= b && lane < e;
            const uint32_t G = sort_stage<true, S>(p, A0, (uint32_t)(A1 - A0), b, e, inb, A0j, lj, marks, tk, tl, ta);
            uint32_t k[4] = {kSent, kSent, kSent, kSent};
            P pr[4] = {P(0), P(0), P(0), P(0)};
            if (lane < G) {
                const uint32_t tw = tk[lane], bk = tw & 0xFFFFFFu, t = tw >> 24;
                const uint4 c = ell_cols(p, bk, t);
                const S a = ta[lane];
                Quad<S> q;
                if (buni)
                    q = splat4(Sem::prod(a, bv0));
                else
                    q = prods<Sem>(a, ell_vals<S>(p, bk, t));
                const uint32_t hi = tl[lane] << cb;
                k[0] = c.x != kSent ? (hi | c.x) : kSent;
                k[1] = c.y != kSent ? (hi | c.y) : kSent;
                k[2] = c.z != kSent ? (hi | c.z) : kSent;
                k[3] = c.w != kSent ? (hi | c.w) : kSent;
                sfor<4>([&](auto E) { pr[E] = q.v[E]; });
            }
            wave_sort256<true, P>(k, pr);
            T s[4];
            sfor<4>([&](auto E) { s[E] = (T)pr[E]; });
            seg_sums<Acc>(k, s);
            uint32_t nk[4];
            next_keys(k, nk);
            bool tail[4];
            uint32_t tc = 0;
            sfor<4>([&](auto E) {
                tail[E] = k[E] != kSent && nk[E] != k[E];
                tc += tail[E] ? 1u : 0u;
            });
            uint32_t o = wave_excl_scan_u32(tc);
            sfor<4>([&](auto E) {
                if (tail[E]) {
                    const S v = (S)Acc::fin(s[E]);
                    if (o < lim) {
                        p.c_col[OB + o] = k[E] & cmask;
                        cval[OB + o] = v;
                    }
                    if (Sem::is_zero(v)) atomicAdd(&zc[cb ? k[E] >> cb : 0u], 1u);
                    ++o;
                }
            });
            wave_sync();
            if (inb) {
                const uint32_t z = zc[lane - b];
                if (z) {
                    p.counts[r] = uj - z;
                    ++zrows;
                    zc[lane - b] = 0;
                }
            }
            wave_sync();
            b = e;
        }
    }
    zrows = wave_sum_u32(zrows);
    if (lane == 0 && zrows)
        __hip_atomic_fetch_add(&p.host_out[2], (unsigned long long)zrows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace slat
