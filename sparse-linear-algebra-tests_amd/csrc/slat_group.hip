// slat_group.hip — MAGNUS's dense-accumulation category with a WORKGROUP per output row, for
// single-window launches (every column inside one LDS bitmap window) with B in ELL form.
//
// The wave-per-row kernels (spgemm_kernels.hpp, k_symbolic / k_numeric MODE 0) hold 4 A entries per
// lane and pay a row's chain of dependent loads (row bounds -> A entries -> ELL rows -> stored
// bitmap) with 3 waves per SIMD in numeric: about half of k_numeric's time on the headline (30^3
// A^6 * A) was that chain, paid ~9 times per wave. Here GT threads (a workgroup of GT / 64 waves)
// share ONE row, E A entries per thread, and the rows are software-pipelined one deep: a row's
// bounds (scalar loads) are read when the row before it starts, and its first GT * E A entries and
// (numeric) its stored bitmap words while the row before it emits. So the only latency a row still
// waits on itself is its ELL groups, which depend on its A entries; everything else hides behind the
// row before it. The workgroup's LDS per row (numeric: bitmap with word ranks + narrow rank slots,
// ~19 KB at the 30^3 window) lets one rank chunk hold 2048 outputs.
//
// Symbolic: column bitmap by LDS atomic ORs, then each wave counts and stores its 64-word blocks
// (the stored-bitmap format of k_symbolic, so every numeric instance can read it).
// Numeric: word ranks from the stored bitmap (a wave scan per block, block bases across the waves
// through LDS), then products into rank slots (u32 slots under the narrow bound; the semiring's
// wide slots otherwise), then a coalesced emit of (column, value) at C.row_ptr[row] + rank.
// Semirings: u32, Sat64, f64 in any order (f64 in the reference's fold order keeps the ordered
// wave-per-row walk).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "slat_launch.hpp"
#include "spgemm_kernels.hpp"

namespace slat {

// the row loop of one workgroup: items b, b + G, ... (rows, or the listed rows at those positions),
// fat rows skipped (the fat-row kernels' rows)
struct GroupRows {
    const Args &p;
    bool listed;
    uint64_t nit;
    __device__ __forceinline__ GroupRows(const Args &p_) : p(p_) {
        listed = p.list != nullptr;
        nit = listed ? (uint64_t)__builtin_amdgcn_readfirstlane(*(volatile unsigned int *)p.list_cnt) : p.nrows;
    }
    __device__ __forceinline__ uint32_t row_of(uint64_t it) const {
        return listed ? (uint32_t)__builtin_amdgcn_readfirstlane(p.list[it]) : (uint32_t)it;
    }
    __device__ __forceinline__ uint64_t skip_fat(uint64_t it) const {
        if (p.fr_mark)
            while (it < nit && p.fr_mark[row_of(it)]) it += gridDim.x;  // uniform
        return it;
    }
};

// a row's bounds (uniform: scalar loads)
template <typename I>
struct RowMeta {
    uint32_t row;
    I a0, a1;
    uint64_t o0;
    uint32_t nnz;    // numeric: its output count (C.row_ptr)
    uint32_t bmask;  // numeric: its touched 64-word blocks (stored bitmap)
};

// ---------------------------------------------------------------------------------------------
// symbolic
// ---------------------------------------------------------------------------------------------
template <typename I, int GT, int E>
__global__ __launch_bounds__(GT) void k_grp_symbolic(Args p) {
    constexpr int GW = GT / kWave;
    extern __shared__ __attribute__((aligned(16))) uint32_t bits[];  // p.ww words
    __shared__ uint32_t s_cnt, s_mask;
    const int tid = threadIdx.x, lane = lane_id();
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid / kWave);
    if (blockIdx.x == 0) {
        if (tid == 0) p.c_rp[0] = 0;
        if (tid < kShards) {  // fields read by k_numeric; [3] (flops) is zeroed by the host
            p.shards[tid * kShardStride + 1] = 0;
            p.shards[tid * kShardStride + 2] = 0;
        }
    }
    for (uint32_t w = tid; w < p.ww; w += GT) bits[w] = 0;
    if (tid == 0) s_cnt = s_mask = 0;
    const uint32_t nblk = p.ww / kWave;
    const GroupRows gr(p);
    auto meta = [&](uint64_t it) {
        RowMeta<I> m{};
        if (it < gr.nit) {
            m.row = gr.row_of(it);
            m.a0 = (I)p.a_rp[m.row];
            m.a1 = (I)p.a_rp[m.row + 1];
        }
        return m;
    };
    uint32_t kk[E];  // the row's first GT * E A entries (thread tid: tid, tid + GT, ...)
    auto load_entries = [&](const RowMeta<I> &m, bool live) {
        sfor<E>([&](auto Q) {
            const I j = m.a0 + (I)(tid + Q * GT);
            kk[Q] = kSent;
            if (live && j < m.a1) kk[Q] = p.a_col[j];
        });
    };
    uint32_t mx = 0, nprod = 0;
    uint64_t it = gr.skip_fat(blockIdx.x);
    RowMeta<I> cur = meta(it);
    load_entries(cur, it < gr.nit);
    __syncthreads();
    while (it < gr.nit) {
        const uint64_t it_next = gr.skip_fat(it + gridDim.x);
        const RowMeta<I> nxt = meta(it_next);
        // every product's column into the bitmap: an entry's ELL groups, group 0 with the group count
        auto walk = [&](uint32_t k) {
            if (k >= p.b_nrows) k = kSent;  // malformed input: ignore the entry
            uint4 c = make_uint4(kSent, kSent, kSent, kSent);
            uint32_t ng = 0;
            if (k != kSent) {
                c = ell_cols(p, k, 0);
                ng = p.ell_ng[k];
            }
            auto put = [&](uint4 q) {
                const uint32_t cc[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (cc[e] != kSent) {
                        atomicOr(&bits[cc[e] >> 5], 1u << (cc[e] & 31));
                        if (p.stats) ++nprod;
                    }
            };
            put(c);
            for (uint32_t t = 1; t < p.ell_wq && __ballot(ng > t); ++t)
                if (ng > t) put(ell_cols(p, k, t));
        };
        sfor<E>([&](auto Q) { walk(kk[Q]); });
        for (I j0 = cur.a0 + (I)(GT * E); j0 < cur.a1; j0 += (I)GT) {  // rows longer than GT * E entries
            const I j = j0 + (I)tid;
            walk(j < cur.a1 ? p.a_col[j] : kSent);
        }
        load_entries(nxt, it_next < gr.nit);  // the next row's entries, during this row's count
        __syncthreads();
        // the row's count; its touched 64-word blocks stored for numeric and cleared
        uint32_t lc = 0, wmask = 0;
        uint32_t *keep = p.sbm ? p.sbm + (uint64_t)cur.row * ((uint64_t)nblk * kWave) : nullptr;
        for (uint32_t b = wv; b < nblk; b += GW) {
            const uint32_t w = b * kWave + lane;
            const uint32_t x = bits[w];
            if (__ballot(x != 0)) {
                lc += __popc(x);
                bits[w] = 0;
                if (keep) keep[w] = x;
                wmask |= 1u << b;
            }
        }
        lc = wave_sum_u32(lc);
        if (lane == 0) {
            if (lc) atomicAdd(&s_cnt, lc);
            if (wmask) atomicOr(&s_mask, wmask);
        }
        __syncthreads();
        if (tid == 0) {
            const uint32_t cnt = s_cnt;
            p.counts[cur.row] = cnt;
            if (p.sbm) p.smask[cur.row] = s_mask;
            s_cnt = 0;
            s_mask = 0;
            mx = max(mx, cnt);
        }
        cur = nxt;
        it = it_next;
    }
    if (p.stats) {
        const uint32_t f = wave_sum_u32(nprod);
        if (lane == 0 && f) atomicAdd(&p.shards[((blockIdx.x * GW + wv) % kShards) * kShardStride + 3], (unsigned long long)f);
    }
    if (p.bmax && tid == 0) p.bmax[blockIdx.x] = mx;
}

// ---------------------------------------------------------------------------------------------
// numeric
// ---------------------------------------------------------------------------------------------
// LDS of one workgroup: W [ww + 1] {bits, rank of the word's first column} (W[ww] = the dummy word
// of columns outside the window) | stage [ww]: the next row's stored bitmap, loaded by LDS DMA |
// rank slots: values, then u16 column offsets
__host__ __device__ inline uint32_t grp_stage_off(uint32_t ww) { return ((ww + 1) * 8 + 15) & ~15u; }
__host__ __device__ inline uint32_t grp_slots_off(uint32_t ww) { return grp_stage_off(ww) + ww * 4; }

template <typename Sem, typename I, int GT, int E>
__global__ __launch_bounds__(GT) void k_grp_numeric(Args p) {
    using S = typename Sem::S;
    using V = typename Sem::V;
    constexpr int GW = GT / kWave;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    __shared__ uint32_t s_btot[32];  // popcount of each 64-word block of the row's bitmap
    __shared__ uint32_t s_amax[GW];  // the waves' max A value (narrow bound)
    __shared__ uint32_t s_zero[2];   // zero sums of a row (by row parity)
    const int tid = threadIdx.x, lane = lane_id();
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid / kWave);
    const uint32_t ww = p.ww, nblk = ww / kWave;
    uint2 *W = (uint2 *)smem8;
    uint32_t *stage = (uint32_t *)(smem8 + grp_stage_off(ww));
    uint8_t *slots = smem8 + grp_slots_off(ww);
    uint32_t bvmax = 0xFFFFFFFFu;  // max B value of this call (from the ELL build's partials)
    bool buni = false;             // every B value equals bvmax (a pattern B)
    if constexpr (Sem::kNarrowable)
        if (p.b_vmax) {
            const unsigned long long v = ((volatile unsigned long long *)p.b_vmax)[kVMaxWord];
            const unsigned long long vi = ((volatile unsigned long long *)p.b_vmax)[kVMinInvWord];
            if ((uint32_t)(v >> 32) == p.epoch) {
                bvmax = (uint32_t)v;
                buni = (uint32_t)(vi >> 32) == p.epoch && ~(uint32_t)vi == bvmax && (sizeof(S) == 4 || bvmax != 0xFFFFFFFFu);
            }
        }
    const S bv0 = (S)bvmax;
    for (uint32_t w = tid; w < p.area / 4; w += GT) ((uint32_t *)slots)[w] = 0;  // the emit keeps them zero
    if (tid == 0) {
        W[ww] = make_uint2(0u, 0x80000000u);  // the dummy word: no bits, a rank no chunk holds
        s_zero[0] = s_zero[1] = 0;
    }
    const GroupRows gr(p);
    S *cval = (S *)p.c_val;
    uint32_t zrows = 0;
    uint32_t prev_row = 0, prev_cnt = 0;  // thread 0: the last row's zero sums are settled next row
    bool prev = false;
    uint32_t par = 0;
    auto settle = [&](uint32_t pz) {
        if (tid == 0 && prev) {
            const uint32_t z = s_zero[pz];
            p.counts[prev_row] = prev_cnt - z;
            if (z) {
                ++zrows;
                s_zero[pz] = 0;
            }
        }
    };
    auto meta = [&](uint64_t it) {
        RowMeta<I> m{};
        if (it < gr.nit) {
            m.row = gr.row_of(it);
            m.a0 = (I)p.a_rp[m.row];
            m.a1 = (I)p.a_rp[m.row + 1];
            m.o0 = p.c_rp[m.row];
            m.nnz = (uint32_t)(p.c_rp[m.row + 1] - m.o0);
            m.bmask = __builtin_amdgcn_readfirstlane(p.smask[m.row]);
        }
        return m;
    };
    uint32_t kk[E];  // the row's first GT * E A entries and values
    S av[E];
    // the row's stored bitmap into `stage` (each wave its blocks wv, wv + GW, ...: the touched ones by
    // LDS DMA, no registers held; the rest zero), and its first A entries into registers
    auto load_data = [&](const RowMeta<I> &m, bool live) {
        const uint32_t *src = p.sbm + (uint64_t)m.row * ((uint64_t)nblk * kWave) + lane;
        for (uint32_t b = wv; b < nblk; b += GW) {
            if (live && ((m.bmask >> b) & 1u))
                __builtin_amdgcn_global_load_lds((const void *)(src + b * kWave),
                                                 (__attribute__((address_space(3))) void *)(stage + b * kWave), 4, 0, 0);
            else
                stage[b * kWave + lane] = 0;
        }
        sfor<E>([&](auto Q) {
            const I j = m.a0 + (I)(tid + Q * GT);
            kk[Q] = kSent;
            av[Q] = S(0);
            if (live && j < m.a1) {
                kk[Q] = p.a_col[j];
                av[Q] = ((const S *)p.a_val)[j];
            }
        });
    };
    uint64_t it = gr.skip_fat(blockIdx.x);
    RowMeta<I> cur = meta(it);
    load_data(cur, it < gr.nit);
    __syncthreads();
    while (it < gr.nit) {
        const uint64_t it_next = gr.skip_fat(it + gridDim.x);
        const RowMeta<I> nxt = meta(it_next);
        const I a0 = cur.a0, a1 = cur.a1;
        const uint32_t nnz = cur.nnz;
        // 1. word ranks of the stored bitmap: wave-inclusive scan per block, block totals to LDS;
        //    the row's max A value (narrow bound). The wave's own LDS DMA (its blocks) must have landed
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every load of this wave, the DMA included
        if constexpr (Sem::kNarrowable) {
            uint32_t am = 0;
            sfor<E>([&](auto Q) { am = max(am, sat32(av[Q])); });
            for (I j = a0 + (I)(GT * E + tid); j < a1; j += (I)GT) am = max(am, sat32(((const S *)p.a_val)[j]));
            am = wave_max_u32(am);
            if (lane == 0) s_amax[wv] = am;
        }
        for (uint32_t b = wv; b < nblk; b += GW) {
            const uint32_t incl = wave_incl_scan(__popc(stage[b * kWave + lane]), 0u, [](uint32_t x, uint32_t y) { return x + y; });
            if (lane == kWave - 1) s_btot[b] = incl;
        }
        __syncthreads();  // block totals, A maxima; the previous row's zero sums
        settle(par ^ 1u);
        // block bases: exclusive scan of the block totals (nblk <= 31 < 64 lanes)
        const uint32_t bt = (uint32_t)lane < nblk ? s_btot[lane] : 0u;
        const uint32_t bex = wave_incl_scan(bt, 0u, [](uint32_t x, uint32_t y) { return x + y; }) - bt;
        for (uint32_t b = wv; b < nblk; b += GW) {  // (the scan again: nothing held across the barrier)
            const uint32_t x = stage[b * kWave + lane], c = __popc(x);
            const uint32_t incl = wave_incl_scan(c, 0u, [](uint32_t x_, uint32_t y_) { return x_ + y_; });
            W[b * kWave + lane] = make_uint2(x, readlane_u32(bex, (int)b) + incl - c);
        }
        bool narrow = false;
        if constexpr (Sem::kNarrowable) {
            uint32_t m = 0;
#pragma unroll
            for (int w = 0; w < GW; ++w) m = max(m, s_amax[w]);
            const uint64_t x = (uint64_t)m * bvmax;
            // (a 64-bit value >= 2^32 clamps to 0xFFFFFFFF: its size is unknown, so no narrow slots)
            narrow = bvmax != 0xFFFFFFFFu && (sizeof(S) == 4 || m != 0xFFFFFFFFu) &&
                     (x == 0 || (uint64_t)(a1 - a0) <= 0xFFFFFFFFull / x);
        }
        __syncthreads();  // W complete
        // 2. products into rank slots, one chunk of ranks [r0, r0 + cap) at a time (one chunk unless
        //    the row has more outputs than the slots hold), then the emit of that chunk
        uint32_t zeros = 0;
        // products of the chunk into its slots (NW: u32 slots under the narrow bound; UNI: a pattern
        // B, whose values are never loaded)
        auto acc = [&](auto narrow_tag, auto uni_tag, uint32_t r0, uint32_t nch) {
            constexpr bool NW = decltype(narrow_tag)::value;
            constexpr bool UNI = decltype(uni_tag)::value;
            using VS = std::conditional_t<NW, uint32_t, V>;
            constexpr uint32_t kVW = NW ? 1 : Sem::kSlots;
            using PS = std::conditional_t<NW, SemNarrowT<S>, Sem>;
            const uint32_t cap = p.area / (uint32_t)(kVW * sizeof(VS) + 2);
            VS *vals = (VS *)slots;
            uint16_t *cols = (uint16_t *)(slots + ((cap * kVW * sizeof(VS) + 3) & ~3u));
            // one ELL group: its four rank lookups issued before any is used
            auto group = [&](uint4 c, const Quad<S> &bv, S a) {
                const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
                S pr0 = S(0);
                if constexpr (UNI) pr0 = PS::prod(a, bv0);
                uint2 w[4];
                uint32_t off[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) w[e] = rank_word(W, ww, cc[e], 0u, off[e]);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t r = rank_in(w[e], off[e], r0, nch);
                    if (r != kSent) {
                        const S pr = UNI ? pr0 : PS::prod(a, bv.v[e]);
                        if constexpr (NW)
                            atomicAdd((uint32_t *)vals + r, (uint32_t)pr);
                        else
                            Sem::acc((V *)vals, r, pr);
                        cols[r] = (uint16_t)off[e];
                    }
                }
            };
            // E entries at once: their group 0 and group counts load together; a later group only
            // where some lane of the wave has one (B rows of more than 4 entries)
            auto walk = [&](const uint32_t (&k)[E], const S (&a)[E]) {
                uint4 c[E];
                Quad<S> bv[E];
                uint32_t ng[E];
                sfor<E>([&](auto Q) {
                    c[Q] = make_uint4(kSent, kSent, kSent, kSent);
                    bv[Q] = Quad<S>{};
                    ng[Q] = 0;
                    if (k[Q] != kSent) {
                        c[Q] = ell_cols(p, k[Q], 0);
                        if constexpr (!UNI) bv[Q] = ell_vals<S>(p, k[Q], 0);
                        ng[Q] = p.ell_ng[k[Q]];
                    }
                });
                sfor<E>([&](auto Q) { group(c[Q], bv[Q], a[Q]); });
                sfor<E>([&](auto Q) {
                    for (uint32_t t = 1; t < p.ell_wq && __ballot(ng[Q] > t); ++t) {
                        uint4 ct = make_uint4(kSent, kSent, kSent, kSent);
                        Quad<S> bt{};
                        if (ng[Q] > t) {
                            ct = ell_cols(p, k[Q], t);
                            if constexpr (!UNI) bt = ell_vals<S>(p, k[Q], t);
                        }
                        group(ct, bt, a[Q]);
                    }
                });
            };
            uint32_t k0[E];
            sfor<E>([&](auto Q) { k0[Q] = kk[Q] < p.b_nrows ? kk[Q] : kSent; });
            walk(k0, av);
            for (I j0 = a0 + (I)(GT * E); j0 < a1; j0 += (I)(GT * E)) {  // rows longer than GT * E entries
                uint32_t k1[E];
                S a1v[E];
                sfor<E>([&](auto Q) {
                    const I j = j0 + (I)(tid + Q * GT);
                    k1[Q] = kSent;
                    a1v[Q] = S(0);
                    if (j < a1) {
                        k1[Q] = p.a_col[j];
                        a1v[Q] = ((const S *)p.a_val)[j];
                    }
                });
                sfor<E>([&](auto Q) {
                    if (k1[Q] >= p.b_nrows) k1[Q] = kSent;
                });
                walk(k1, a1v);
            }
        };
        // the chunk's (column, value) pairs at C.row_ptr[row] + rank, coalesced; the slots left zero
        auto emit = [&](auto narrow_tag, uint32_t r0, uint32_t nch) {
            constexpr bool NW = decltype(narrow_tag)::value;
            using VS = std::conditional_t<NW, uint32_t, V>;
            constexpr uint32_t kVW = NW ? 1 : Sem::kSlots;
            const uint32_t cap = p.area / (uint32_t)(kVW * sizeof(VS) + 2);
            VS *vals = (VS *)slots;
            const uint16_t *cols = (const uint16_t *)(slots + ((cap * kVW * sizeof(VS) + 3) & ~3u));
            uint32_t *oc = p.c_col + cur.o0 + r0;
            S *ov = cval + cur.o0 + r0;
            for (uint32_t t = tid; t < nch; t += GT) {
                S v;
                if constexpr (NW)
                    v = (S)vals[t];
                else
                    v = Sem::finish((const V *)vals, t);
                const uint32_t col = cols[t];
#pragma unroll
                for (uint32_t x = 0; x < kVW; ++x) vals[t * kVW + x] = VS(0);
                zeros += Sem::is_zero(v) ? 1u : 0u;
                oc[t] = col;
                ov[t] = v;
            }
        };
        const uint32_t cap = p.area / (narrow ? 6u : (uint32_t)(Sem::kSlots * sizeof(V) + 2));
        const uint32_t nchunks = nnz ? (nnz + cap - 1) / cap : 1u;
        for (uint32_t ci = 0, r0 = 0; ci < nchunks; ++ci, r0 += cap) {
            const uint32_t nch = nnz > r0 ? min(cap, nnz - r0) : 0u;
            if constexpr (Sem::kNarrowable) {
                if (narrow && buni)
                    acc(std::true_type{}, std::true_type{}, r0, nch);
                else if (narrow)
                    acc(std::true_type{}, std::false_type{}, r0, nch);
                else
                    acc(std::false_type{}, std::false_type{}, r0, nch);
            } else {
                acc(std::false_type{}, std::false_type{}, r0, nch);
            }
            __syncthreads();  // the chunk's sums
            // the next row's data loads go out before this row's emit (after the last chunk's walk:
            // the walk reads kk / av)
            if (ci + 1 == nchunks) load_data(nxt, it_next < gr.nit);
            if (Sem::kNarrowable && narrow)
                emit(std::true_type{}, r0, nch);
            else
                emit(std::false_type{}, r0, nch);
            if (ci + 1 < nchunks) __syncthreads();  // the slots clear before the next chunk
        }
        // the row's zero sums (rare: explicit zeros or f64 cancellation), settled next row
        if (zeros) atomicAdd(&s_zero[par], zeros);
        if (tid == 0) {
            prev = true;
            prev_row = cur.row;
            prev_cnt = nnz;
        }
        par ^= 1u;
        cur = nxt;
        it = it_next;
        // (no barrier here: the next row writes W only after its first barrier, which every thread
        // reaches after its emit; the slots are zero again before the next row's second barrier)
    }
    __syncthreads();
    settle(par ^ 1u);
    add_zero_rows(&p.host_out[2], zrows, p.seq != 0);
    signal_done(p);
}

}  // namespace slat

using namespace slat;

// ------------------------------------------------------------------------------------------------
// launchers: GT threads per row (128 or 256), E = 256 / GT entries per thread
// ------------------------------------------------------------------------------------------------
size_t slat_group_numeric_lds(uint32_t ww, uint32_t area) { return grp_slots_off(ww) + area; }

template <int GT, typename F>
static hipError_t sym_instance(bool idx32, F &&f) {
    constexpr int E = 256 / GT;
    return idx32 ? f(k_grp_symbolic<uint32_t, GT, E>) : f(k_grp_symbolic<uint64_t, GT, E>);
}

template <int GT, typename F>
static hipError_t num_instance(int sem, bool idx32, uint32_t, F &&f) {
    constexpr int E = 256 / GT;
    switch (sem) {
    case kSemU32: return idx32 ? f(k_grp_numeric<SemU32, uint32_t, GT, E>) : f(k_grp_numeric<SemU32, uint64_t, GT, E>);
    case kSemSat64: return idx32 ? f(k_grp_numeric<SemSat64, uint32_t, GT, E>) : f(k_grp_numeric<SemSat64, uint64_t, GT, E>);
    case kSemF64Any: return idx32 ? f(k_grp_numeric<SemF64Any, uint32_t, GT, E>) : f(k_grp_numeric<SemF64Any, uint64_t, GT, E>);
    default: return hipErrorInvalidValue;  // f64 in the fold order: the ordered wave-per-row walk
    }
}

hipError_t slat_launch_group_symbolic(int gt, bool idx32, dim3 grid, size_t lds, hipStream_t s, const Args &a) {
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(gt), lds, s, a);
        return hipGetLastError();
    };
    return gt == 128 ? sym_instance<128>(idx32, go) : sym_instance<256>(idx32, go);
}

hipError_t slat_launch_group_numeric(int gt, int sem, bool idx32, dim3 grid, size_t lds, hipStream_t s, const Args &a) {
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(gt), lds, s, a);
        return hipGetLastError();
    };
    return gt == 128 ? num_instance<128>(sem, idx32, a.ww, go) : num_instance<256>(sem, idx32, a.ww, go);
}

int slat_group_blocks_per_cu(int gt, int sem, bool numeric, bool idx32, size_t lds, uint32_t ww) {
    static thread_local int cache_nb[128] = {};
    static thread_local size_t cache_lds[128] = {};
    const int ci = (idx32 ? 1 : 0) | (numeric ? 2 : 0) | ((sem & 3) << 2) | (ww > 16u * kWave ? 16 : 0) | (gt == 128 ? 32 : 0);
    if (cache_lds[ci] == lds && cache_nb[ci] > 0) return cache_nb[ci];
    int nb = 0;
    auto occ = [&](auto kern) { return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, gt, lds); };
    hipError_t e;
    if (!numeric)
        e = gt == 128 ? sym_instance<128>(idx32, occ) : sym_instance<256>(idx32, occ);
    else
        e = gt == 128 ? num_instance<128>(sem, idx32, ww, occ) : num_instance<256>(sem, idx32, ww, occ);
    nb = (e == hipSuccess && nb > 0) ? nb : 1;
    cache_lds[ci] = lds;
    cache_nb[ci] = nb;
    return nb;
}
