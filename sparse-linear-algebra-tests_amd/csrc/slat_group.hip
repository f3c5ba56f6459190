// slat_group.hip — MAGNUS's dense-accumulation category with a WORKGROUP per output row, for
// single-window launches (every column inside one LDS bitmap window) with B in ELL form.
//
// The wave-per-row kernels (spgemm_kernels.hpp, k_symbolic / k_numeric MODE 0) hold 4 A entries per
// lane and pay a row's chain of dependent loads (row bounds -> A entries -> ELL rows -> stored
// bitmap) with 3 waves per SIMD in numeric: about half of k_numeric's time on the headline (30^3
// A^6 * A) was that chain, paid ~9 times per wave. Here the 256 threads of a workgroup share ONE
// row: one A entry per thread, every ELL group of that entry loaded at once (no group counts, no
// lane compaction of the tails), the stored bitmap loaded by all four waves beside the A entries,
// so a row's loads are in flight together and its chain is three loads deep; the row bounds of the
// next row are read while the current one runs. Register use is low enough for 8 waves per SIMD
// (eight rows in flight per CU), and the LDS per row (bitmap with word ranks + narrow rank slots,
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

constexpr int kGT = 256;           // threads per row (the workgroup)
constexpr int kGW = kGT / kWave;   // its waves
constexpr int kGQ = 4;             // ELL groups loaded per step (one entry's up to 16 B columns)

// the row loop of one workgroup: rows b, b + G, ... (or the listed rows at those positions), with
// the next row's bounds read one row ahead
struct GroupRows {
    const Args &p;
    bool listed;
    uint64_t nit;
    __device__ __forceinline__ GroupRows(const Args &p_) : p(p_) {
        listed = p.list != nullptr;
        nit = listed ? (uint64_t)__builtin_amdgcn_readfirstlane(*(volatile unsigned int *)p.list_cnt) : p.nrows;
    }
    __device__ __forceinline__ uint64_t row_of(uint64_t it) const {
        return listed ? (uint64_t)__builtin_amdgcn_readfirstlane(p.list[it]) : it;
    }
};

// ---------------------------------------------------------------------------------------------
// symbolic
// ---------------------------------------------------------------------------------------------
template <typename I>
__global__ __launch_bounds__(kGT) void k_grp_symbolic(Args p) {
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
    for (uint32_t w = tid; w < p.ww; w += kGT) bits[w] = 0;
    if (tid == 0) s_cnt = s_mask = 0;
    __syncthreads();
    const uint32_t nblk = p.ww / kWave;
    const uint32_t wq = p.ell_wq;
    GroupRows gr(p);
    uint32_t mx = 0, nprod = 0;
    for (uint64_t it = blockIdx.x; it < gr.nit; it += gridDim.x) {
        const uint64_t row = gr.row_of(it);
        if (fat_row(p, row)) continue;  // uniform: the fat-row kernels' row
        const I a0 = (I)p.a_rp[row], a1 = (I)p.a_rp[row + 1];
        for (I j0 = a0; j0 < a1; j0 += (I)kGT) {
            const I j = j0 + (I)tid;
            uint32_t k = kSent;
            if (j < a1) k = p.a_col[j];
            if (k >= p.b_nrows) k = kSent;  // malformed input: ignore the entry
            for (uint32_t t0 = 0; t0 < wq; t0 += kGQ) {
                uint4 c[kGQ];
                sfor<kGQ>([&](auto Q) {
                    c[Q] = make_uint4(kSent, kSent, kSent, kSent);
                    if (k != kSent && t0 + Q < wq) c[Q] = ell_cols(p, k, t0 + Q);
                });
                sfor<kGQ>([&](auto Q) {
                    const uint32_t cc[4] = {c[Q].x, c[Q].y, c[Q].z, c[Q].w};
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (cc[e] != kSent) {
                            atomicOr(&bits[cc[e] >> 5], 1u << (cc[e] & 31));
                            if (p.stats) ++nprod;
                        }
                });
            }
        }
        __syncthreads();
        // the row's count; its touched 64-word blocks stored for numeric and cleared
        uint32_t lc = 0, wmask = 0;
        uint32_t *keep = p.sbm ? p.sbm + row * ((uint64_t)nblk * kWave) : nullptr;
        for (uint32_t b = wv; b < nblk; b += kGW) {
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
            p.counts[row] = cnt;
            if (p.sbm) p.smask[row] = s_mask;
            s_cnt = 0;
            s_mask = 0;
            mx = max(mx, cnt);
        }
    }
    if (p.stats) {
        const uint32_t f = wave_sum_u32(nprod);
        if (lane == 0 && f) atomicAdd(&p.shards[((blockIdx.x * kGW + wv) % kShards) * kShardStride + 3], (unsigned long long)f);
    }
    if (p.bmax && tid == 0) p.bmax[blockIdx.x] = mx;
}

// ---------------------------------------------------------------------------------------------
// numeric
// ---------------------------------------------------------------------------------------------
// LDS of one workgroup: W [ww + 1] {bits, rank of the word's first column} (W[ww] = the dummy word
// of columns outside the window) | rank slots: values, then u16 column offsets
__host__ __device__ inline uint32_t grp_slots_off(uint32_t ww) { return ((ww + 1) * 8 + 15) & ~15u; }

template <typename Sem, typename I>
__global__ __launch_bounds__(kGT) void k_grp_numeric(Args p) {
    using S = typename Sem::S;
    using V = typename Sem::V;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    __shared__ uint32_t s_btot[32];   // popcount of each 64-word block of the row's bitmap
    __shared__ uint32_t s_amax[kGW];  // the waves' max A value (narrow bound)
    __shared__ uint32_t s_zero[2];    // zero sums of a row (by row parity)
    const int tid = threadIdx.x, lane = lane_id();
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid / kWave);
    const uint32_t ww = p.ww, nblk = ww / kWave, wq = p.ell_wq;
    uint2 *W = (uint2 *)smem8;
    uint8_t *slots = smem8 + grp_slots_off(ww);
    // rank-chunk capacities: narrow = u32 value + u16 column, wide = V * kSlots + u16 column
    const uint32_t cap_n = p.area / 6, cap_w = p.area / (uint32_t)(sizeof(V) * Sem::kSlots + 2);
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
    for (uint32_t w = tid; w < p.area / 4; w += kGT) ((uint32_t *)slots)[w] = 0;  // the emit keeps them zero
    if (tid == 0) {
        W[ww] = make_uint2(0u, 0x80000000u);  // the dummy word: no bits, a rank no chunk holds
        s_zero[0] = s_zero[1] = 0;
    }
    GroupRows gr(p);
    S *cval = (S *)p.c_val;
    uint32_t zrows = 0;
    uint64_t prev_row = ~0ull, prev_cnt = 0;  // tid 0: the last row's zero sums are settled next row
    uint32_t par = 0;
    // a row's zero sums are known after its emit; thread 0 settles them one barrier later
    auto settle = [&](uint32_t pz) {
        if (tid == 0 && prev_row != ~0ull) {
            const uint32_t z = s_zero[pz];
            p.counts[prev_row] = prev_cnt - z;
            if (z) {
                ++zrows;
                s_zero[pz] = 0;
            }
        }
    };
    __syncthreads();
    for (uint64_t it = blockIdx.x; it < gr.nit; it += gridDim.x) {
        const uint64_t row = gr.row_of(it);
        if (fat_row(p, row)) continue;  // uniform
        const I a0 = (I)p.a_rp[row], a1 = (I)p.a_rp[row + 1];
        const uint64_t o0 = p.c_rp[row], o1 = p.c_rp[row + 1];
        const uint32_t nnz = (uint32_t)(o1 - o0);
        const uint64_t len = (uint64_t)(a1 - a0);
        // 1. the row's stored bitmap (touched blocks; the rest zero) and its first A entries, all
        //    loads issued together
        const uint32_t bmask = __builtin_amdgcn_readfirstlane(p.smask[row]);
        const uint32_t *src = p.sbm + row * ((uint64_t)nblk * kWave) + lane;
        uint32_t xs[8];  // this wave's blocks wv, wv + 4, ... (nblk <= 31)
        sfor<8>([&](auto B) {
            const uint32_t b = wv + kGW * B;
            xs[B] = 0;
            if (b < nblk && ((bmask >> b) & 1u)) xs[B] = src[b * kWave];
        });
        uint32_t k0 = kSent;
        S av0 = S(0);
        {
            const I j = a0 + (I)tid;
            if (j < a1) {
                k0 = p.a_col[j];
                av0 = ((const S *)p.a_val)[j];
            }
        }
        uint32_t am = 0;
        if constexpr (Sem::kNarrowable) {
            am = sat32(av0);
            // a row longer than one pass of the workgroup: every A value for the bound
            for (I j = a0 + (I)(kGT + tid); j < a1; j += (I)kGT) am = max(am, sat32(((const S *)p.a_val)[j]));
            am = wave_max_u32(am);
            if (lane == 0) s_amax[wv] = am;
        }
        // word popcounts: wave-inclusive scan per block, the block totals to LDS
        uint32_t ex[8];
        sfor<8>([&](auto B) {
            const uint32_t b = wv + kGW * B;
            ex[B] = 0;
            if (b < nblk) {
                const uint32_t c = __popc(xs[B]);
                const uint32_t incl = wave_incl_scan(c, 0u, [](uint32_t x, uint32_t y) { return x + y; });
                ex[B] = incl - c;
                if (lane == kWave - 1) s_btot[b] = incl;
            }
        });
        __syncthreads();  // block totals, A maxima; the previous row's zero sums
        settle(par ^ 1u);
        // block bases: exclusive scan of the block totals (nblk <= 31 <= 64 lanes)
        const uint32_t bt = (uint32_t)lane < nblk ? s_btot[lane] : 0u;
        const uint32_t bex = wave_incl_scan(bt, 0u, [](uint32_t x, uint32_t y) { return x + y; }) - bt;
        sfor<8>([&](auto B) {
            const uint32_t b = wv + kGW * B;
            if (b < nblk) W[b * kWave + lane] = make_uint2(xs[B], readlane_u32(bex, (int)b) + ex[B]);
        });
        bool narrow = false;
        if constexpr (Sem::kNarrowable) {
            uint32_t m = 0;
#pragma unroll
            for (int w = 0; w < kGW; ++w) m = max(m, s_amax[w]);
            const uint64_t x = (uint64_t)m * bvmax;
            // (a 64-bit value >= 2^32 clamps to 0xFFFFFFFF: its size is unknown, so no narrow slots)
            narrow = bvmax != 0xFFFFFFFFu && (sizeof(S) == 4 || m != 0xFFFFFFFFu) && (x == 0 || len <= 0xFFFFFFFFull / x);
        }
        __syncthreads();  // W complete
        // 2. products into rank slots, one chunk of ranks [r0, r0 + cap) at a time (one chunk unless
        //    the row has more outputs than the slots hold), then the emit of that chunk
        uint32_t zeros = 0;
        auto run = [&](auto narrow_tag, auto uni_tag) {
            constexpr bool NW = decltype(narrow_tag)::value;
            constexpr bool UNI = decltype(uni_tag)::value;
            using VS = std::conditional_t<NW, uint32_t, V>;
            constexpr uint32_t kVW = NW ? 1 : Sem::kSlots;
            using PS = std::conditional_t<NW, SemNarrowT<S>, Sem>;
            const uint32_t cap = NW ? cap_n : cap_w;
            VS *vals = (VS *)slots;
            uint16_t *cols = (uint16_t *)(slots + ((cap * kVW * sizeof(VS) + 3) & ~3u));
            for (uint32_t r0 = 0; r0 < nnz; r0 += cap) {
                const uint32_t nch = min(cap, nnz - r0);
                for (I j0 = a0; j0 < a1; j0 += (I)kGT) {
                    uint32_t k = k0;
                    S a = av0;
                    if (j0 != a0) {  // later passes of a long row (uniform)
                        const I j = j0 + (I)tid;
                        k = kSent;
                        if (j < a1) {
                            k = p.a_col[j];
                            a = ((const S *)p.a_val)[j];
                        }
                    }
                    if (k >= p.b_nrows) k = kSent;
                    for (uint32_t t0 = 0; t0 < wq; t0 += kGQ) {
                        uint4 c[kGQ];
                        Quad<S> bv[kGQ];
                        sfor<kGQ>([&](auto Q) {
                            c[Q] = make_uint4(kSent, kSent, kSent, kSent);
                            bv[Q] = Quad<S>{};
                            if (k != kSent && t0 + Q < wq) {
                                c[Q] = ell_cols(p, k, t0 + Q);
                                if constexpr (!UNI) bv[Q] = ell_vals<S>(p, k, t0 + Q);
                            }
                        });
                        S pr0 = S(0);
                        if constexpr (UNI) pr0 = PS::prod(a, bv0);
                        // a group's four rank lookups issued before any is used (few registers
                        // live: the kernel runs at 8 waves per SIMD)
                        sfor<kGQ>([&](auto Q) {
                            const uint32_t cc[4] = {c[Q].x, c[Q].y, c[Q].z, c[Q].w};
                            uint2 w[4];
                            uint32_t off[4];
#pragma unroll
                            for (int e = 0; e < 4; ++e) w[e] = rank_word(W, ww, cc[e], 0u, off[e]);
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const uint32_t r = rank_in(w[e], off[e], r0, nch);
                                if (r != kSent) {
                                    const S pr = UNI ? pr0 : PS::prod(a, bv[Q].v[e]);
                                    if constexpr (NW)
                                        atomicAdd((uint32_t *)vals + r, (uint32_t)pr);
                                    else
                                        Sem::acc((V *)vals, r, pr);
                                    cols[r] = (uint16_t)off[e];
                                }
                            }
                        });
                    }
                }
                __syncthreads();  // the chunk's sums
                uint32_t *oc = p.c_col + o0 + r0;
                S *ov = cval + o0 + r0;
                for (uint32_t t = tid; t < nch; t += kGT) {
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
                if (r0 + cap < nnz) __syncthreads();  // the slots clear before the next chunk
            }
        };
        if constexpr (Sem::kNarrowable) {
            if (narrow && buni)
                run(std::true_type{}, std::true_type{});
            else if (narrow)
                run(std::true_type{}, std::false_type{});
            else
                run(std::false_type{}, std::false_type{});
        } else {
            run(std::false_type{}, std::false_type{});
        }
        // the row's zero sums (rare: explicit zeros or f64 cancellation), settled next row
        if (zeros) atomicAdd(&s_zero[par], zeros);
        if (tid == 0) {
            prev_row = row;
            prev_cnt = nnz;
        }
        par ^= 1u;
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
// launchers
// ------------------------------------------------------------------------------------------------
size_t slat_group_numeric_lds(uint32_t ww, uint32_t area) { return grp_slots_off(ww) + area; }

hipError_t slat_launch_group_symbolic(bool idx32, dim3 grid, size_t lds, hipStream_t s, const Args &a) {
    if (idx32)
        hipLaunchKernelGGL(k_grp_symbolic<uint32_t>, grid, dim3(kGT), lds, s, a);
    else
        hipLaunchKernelGGL(k_grp_symbolic<uint64_t>, grid, dim3(kGT), lds, s, a);
    return hipGetLastError();
}

template <typename F>
static hipError_t grp_instance(int sem, bool idx32, F &&f) {
    switch (sem) {
    case kSemU32: return idx32 ? f(k_grp_numeric<SemU32, uint32_t>) : f(k_grp_numeric<SemU32, uint64_t>);
    case kSemSat64: return idx32 ? f(k_grp_numeric<SemSat64, uint32_t>) : f(k_grp_numeric<SemSat64, uint64_t>);
    case kSemF64Any: return idx32 ? f(k_grp_numeric<SemF64Any, uint32_t>) : f(k_grp_numeric<SemF64Any, uint64_t>);
    default: return hipErrorInvalidValue;  // f64 in the fold order: the ordered wave-per-row walk
    }
}

hipError_t slat_launch_group_numeric(int sem, bool idx32, dim3 grid, size_t lds, hipStream_t s, const Args &a) {
    return grp_instance(sem, idx32, [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(kGT), lds, s, a);
        return hipGetLastError();
    });
}

int slat_group_blocks_per_cu(int sem, bool numeric, bool idx32, size_t lds) {
    static thread_local int cache_nb[32] = {};
    static thread_local size_t cache_lds[32] = {};
    const int ci = (idx32 ? 1 : 0) | (numeric ? 2 : 0) | ((sem & 3) << 2);
    if (cache_lds[ci] == lds && cache_nb[ci] > 0) return cache_nb[ci];
    int nb = 0;
    hipError_t e;
    if (!numeric)
        e = idx32 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_grp_symbolic<uint32_t>, kGT, lds)
                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_grp_symbolic<uint64_t>, kGT, lds);
    else
        e = grp_instance(sem, idx32, [&](auto kern) { return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, kGT, lds); });
    nb = (e == hipSuccess && nb > 0) ? nb : 1;
    cache_lds[ci] = lds;
    cache_nb[ci] = nb;
    return nb;
}
