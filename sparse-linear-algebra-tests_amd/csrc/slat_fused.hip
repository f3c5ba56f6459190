// slat_fused.hip — the single-kernel SpGEMM for launches whose columns fit one LDS window and whose
// B has short rows (the ELL copy): the reference's matmul_par (src/graph_csr.rs:350-484) runs its
// symbolic pass, a serial prefix sum and its numeric pass over the whole matrix; here ONE wavefront
// takes an output row through all three:
//
//   1. walk:   A's row segment in registers (kRegQ entries per lane), the ELL groups of the B rows
//              it references loaded once and KEPT in registers (cols, and B values unless B is a
//              pattern) for rows of one segment — the second pass replays them without a load;
//   2. bitmap: ds_or of every product's column into the row's LDS window bitmap;
//   3. ranks:  popcount prefix over the touched 64-word blocks -> the row's structural count;
//              published at once as the row's aggregate in an epoch-tagged status word;
//   4. values: products into LDS rank slots (replayed from registers);
//   5. offset: decoupled look-back over the preceding rows' status words (64 per round, one lane
//              each) -> the row's exclusive prefix = C.row_ptr[row]; publish the inclusive prefix;
//   6. emit:   (col, value) at C.row_ptr[row] + rank, already sorted, slots cleared on the way.
//
// Rows go to waves in order (row = wave + k * waves; the grid is resident), and a row publishes its
// count before it waits on anything, so the wave on the lowest unfinished row always proceeds. The
// look-back is two-level (the row's group of 64, then group aggregates back to a group inclusive
// prefix: two loads per lane), and runs after the values pass, by which time the rows of the groups
// before are counted. A look-back that spins past a time limit (a grid that was not all resident)
// abandons the kernel and the host reruns the call on the three-kernel path. No symbolic kernel, no
// scan kernel, no stored bitmaps: A is read once and C written once.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "slat.h"
#include "slat_internal.hpp"
#include "spgemm_kernels.hpp"

#ifndef SLAT_FUSED_NOLB
#define SLAT_FUSED_NOLB 0  // experiments: no look-back (every row at offset 0: timing only)
#endif
#ifndef SLAT_FUSED_WPS
#define SLAT_FUSED_WPS 3  // waves per SIMD the register budget is sized for (LDS allows 3 at the 30^3 window)
#endif

namespace slat {

// status word: epoch (bits 44..63) | flag (bits 42..43) | value (bits 0..41)
constexpr unsigned long long kLbAgg = 1ull << 42, kLbInc = 2ull << 42, kLbVal = (1ull << 42) - 1;
constexpr int kLbEpochShift = 44;

struct FusedArgs {
    Args a;
    unsigned long long *status;  // [n] per-row aggregates (the row's count), epoch-tagged
    unsigned long long *gstat;   // [n/64] per-group aggregate / inclusive prefix, epoch-tagged
    unsigned long long *gacc;    // [n/64] per-group arrivals (low 8 bits) and count sum; zero between calls
    unsigned long long *done;    // finished waves (monotonic across calls)
    unsigned long long done_base;
    unsigned long long *maxw;    // (epoch << 32) | max row count
    unsigned int *abort;         // a look-back that waited too long (grid not resident): give up
    uint32_t epoch;              // look-back epoch (20 bits)
    uint32_t nwaves;
};

// u64 sum over the wave of values < 2^42 (24-bit low / 18-bit high halves summed apart)
__device__ __forceinline__ uint64_t wave_sum_u42(uint64_t v) {
    const uint32_t lo = wave_sum_u32((uint32_t)(v & 0xFFFFFFu));
    const uint32_t hi = wave_sum_u32((uint32_t)(v >> 24));
    return (uint64_t)lo + ((uint64_t)hi << 24);
}

// A spin longer than this (s_memrealtime, 100 MHz ticks: 0.2 s) means a row's owner is not running:
// the grid was not resident. The kernel then gives up (every wave leaves) and the host reruns the
// call on the three-kernel path.
constexpr uint64_t kSpinTicks = 20000000ull;

__device__ __forceinline__ bool aborted(const FusedArgs &f) {
    return __hip_atomic_load(f.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// Exclusive prefix of `row`, two-level: the counts of the rows before it in its group of 64 (one
// lane each) plus the prefix of the groups before: group aggregates (complete once all 64 rows have
// arrived) summed back to the nearest group inclusive prefix, 64 groups per round. Returns false
// when it gave up (abort).
__device__ __forceinline__ bool look_back(const FusedArgs &f, uint64_t row, uint64_t &excl) {
    const int lane = lane_id();
    const unsigned long long tag = (unsigned long long)f.epoch;
    const uint64_t g = row >> 6, k = row & 63;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    auto ready = [&](unsigned long long x) { return (x >> kLbEpochShift) == tag && (x & (kLbAgg | kLbInc)) != 0; };
    // rows 64g .. row-1 (lane l: row 64g + l)
    unsigned long long rx = 0;
    bool rok = (uint64_t)lane >= k;
    uint64_t sum = 0;
    // groups g-1, g-2, ... (lane l: group gj - 1 - l)
    uint64_t gj = g;
    for (;;) {
        const bool greal = (uint64_t)lane < gj;
        const uint64_t gidx = greal ? gj - 1 - (uint64_t)lane : 0;
        unsigned long long gx = greal ? 0ull : kLbInc;
        bool gok = !greal;
        for (;;) {
            if (!rok) {
                rx = __hip_atomic_load(&f.status[(g << 6) + (uint64_t)lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                rok = ready(rx);
            }
            if (!gok) {
                gx = __hip_atomic_load(&f.gstat[gidx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                gok = ready(gx);
            }
            const unsigned long long gready = __ballot(gok), ginc = __ballot(gok && (gx & kLbInc));
            const uint32_t first_nr = ~gready ? (uint32_t)__builtin_ctzll(~gready) : 64u;
            const uint32_t first_inc = ginc ? (uint32_t)__builtin_ctzll(ginc) : 64u;
            const bool rows_done = __ballot(!rok) == 0;
            if (rows_done && (first_inc < first_nr || first_nr == 64u)) {
                if (first_inc < first_nr) {
                    sum += wave_sum_u42((uint32_t)lane <= first_inc ? (gx & kLbVal) : 0ull);
                    gj = 0;
                } else {
                    sum += wave_sum_u42(gx & kLbVal);
                    gj = gj > 64 ? gj - 64 : 0;
                }
                break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks || aborted(f)) {
                if (lane == 0) {
                    __hip_atomic_store(f.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&f.a.host_out[3], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (gj == 0) break;
        rok = true;  // the row part is summed once (below), from the first round's loads
    }
    excl = sum + wave_sum_u42((uint64_t)lane < k ? (rx & kLbVal) : 0ull);
    return true;
}

// a row's count is in: its status word, and its group's arrival counter; the row completing the
// group publishes the group aggregate and clears the counter for the next call
__device__ __forceinline__ void arrive(const FusedArgs &f, uint64_t row, uint32_t cnt) {
    const unsigned long long tag = (unsigned long long)f.epoch << kLbEpochShift;
    __hip_atomic_store(&f.status[row], tag | kLbAgg | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t g = row >> 6;
    const uint64_t members = min<uint64_t>(64, f.a.nrows - (g << 6));
    const unsigned long long old = atomicAdd(&f.gacc[g], ((unsigned long long)cnt << 8) | 1ull);
    if ((old & 0xFFull) + 1 == members) {
        f.gacc[g] = 0;
        // max: an inclusive prefix the group's last row may have published first stays (its flag
        // is the larger one), and a stale epoch always loses
        atomicMax(&f.gstat[g], tag | kLbAgg | ((old >> 8) + cnt));
    }
}

// the row's exclusive prefix is known: row_ptr[row + 1], and the group's inclusive prefix when the
// row is the group's last
__device__ __forceinline__ void settle(const FusedArgs &f, uint64_t row, uint64_t excl, uint32_t cnt) {
    if (lane_id() != 0) return;
    const unsigned long long tag = (unsigned long long)f.epoch << kLbEpochShift;
    f.a.c_rp[row + 1] = excl + cnt;
    if (row == 0) f.a.c_rp[0] = 0;
    if ((row & 63) == 63) atomicMax(&f.gstat[row >> 6], tag | kLbInc | (excl + cnt));
}

// The row's groups segment by segment (RowWalker: kRegQ A entries per lane, the compacted ELL tail
// batches), with the ELL column groups of the segment held in registers: the bitmap pass walks the
// segments in order and leaves the last one in registers, the values pass starts with it and
// reloads only the others (one-segment rows: no reload at all). B values, unless B is a pattern, are
// loaded by the values pass (L2 hits). A segment whose tails overflow the register batches (rare)
// walks its B rows entry by entry.
template <typename Sem, typename I, bool UNI>
struct SegRow : RowWalker<Sem, I, true, true> {
    using Base = RowWalker<Sem, I, true, true>;
    using S = typename Sem::S;
    uint4 cq[kRegQ], ct0, ct1;
    uint32_t cur = 0;  // the segment in registers

    __device__ __forceinline__ SegRow(const Args &p, I a0, I a1) : Base(p, a0, a1) {
        if (!this->single) this->load_seg(a0);
        load_cols();
    }
    __device__ __forceinline__ void load_cols() {
        const Args &p = this->p;
        ct0 = ct1 = make_uint4(kSent, kSent, kSent, kSent);
        sfor<kRegQ>([&](auto Q) { cq[Q] = make_uint4(kSent, kSent, kSent, kSent); });
        if (this->nb == Base::kOvf) return;
        sfor<kRegQ>([&](auto Q) {
            if (this->kq[Q] != kSent) cq[Q] = ell_cols(p, this->kq[Q], 0);
        });
        if (this->bk0 != kSent) ct0 = ell_cols(p, this->bk0, this->bt0);
        if (this->bk1 != kSent) ct1 = ell_cols(p, this->bk1, this->bt1);
    }
    __device__ __forceinline__ void go(uint32_t sg) {
        if (sg == cur) return;
        this->load_seg(this->a0 + (I)((uint64_t)sg * Base::kSeg));
        load_cols();
        cur = sg;
    }
    // the groups of the segment in registers; VV: with products a * b under PSem
    template <bool VV, typename PSem, typename G>
    __device__ __forceinline__ void seg(G &grp, S v0) {
        const Args &p = this->p;
        if (this->nb == Base::kOvf) {
            sfor<kRegQ>([&](auto Q) {
                if (this->kq[Q] != kSent) walk_brow<Sem, true, VV, I>(p, this->kq[Q], this->aq[Q], 0, grp);
            });
            return;
        }
        Quad<S> pq[kRegQ], pt0 = {}, pt1 = {};
        sfor<kRegQ>([&](auto Q) { pq[Q] = Quad<S>{}; });
        if constexpr (VV && UNI) {
            sfor<kRegQ>([&](auto Q) { pq[Q] = splat4(PSem::prod(this->aq[Q], v0)); });
            pt0 = splat4(PSem::prod(this->ba0, v0));
            pt1 = splat4(PSem::prod(this->ba1, v0));
        } else if constexpr (VV) {
            sfor<kRegQ>([&](auto Q) {
                if (this->kq[Q] != kSent) pq[Q] = ell_vals<S>(p, this->kq[Q], 0);
            });
            if (this->bk0 != kSent) pt0 = ell_vals<S>(p, this->bk0, this->bt0);
            if (this->bk1 != kSent) pt1 = ell_vals<S>(p, this->bk1, this->bt1);
            sfor<kRegQ>([&](auto Q) { pq[Q] = slat::prods<PSem>(this->aq[Q], pq[Q]); });
            pt0 = slat::prods<PSem>(this->ba0, pt0);
            pt1 = slat::prods<PSem>(this->ba1, pt1);
        }
        grp.multi(cq, pq);
        if (this->nb > 0) grp(ct0, pt0);
        if (this->nb > 1) grp(ct1, pt1);
    }
    // the bitmap pass: every segment in order (the last stays in registers)
    template <typename G>
    __device__ __forceinline__ void cols(G &grp) {
        for (uint32_t sg = 0; sg < this->nseg; ++sg) {
            go(sg);
            seg<false, Sem>(grp, S(0));
        }
    }
    // the values pass: the segment in registers first, then the others
    template <typename PSem, typename G>
    __device__ __forceinline__ void prods(G &grp, S v0) {
        const uint32_t first = cur;
        seg<true, PSem>(grp, v0);
        for (uint32_t sg = 0; sg < this->nseg; ++sg) {
            if (sg == first) continue;
            go(sg);
            seg<true, PSem>(grp, v0);
        }
    }
};

// the row loop of one wave; UNI: every B value equals bvmax (a pattern B: no B-value loads)
template <typename Sem, typename I, bool UNI>
__device__ __forceinline__ void fused_rows(const FusedArgs &f, uint8_t *region, uint32_t bvmax, uint32_t &zrows,
                                           uint32_t &rowmax) {
    using S = typename Sem::S;
    using V = typename Sem::V;
    const Args &p = f.a;
    const int lane = lane_id();
    const NumLayout lay = num_layout(p.ww, p.area);
    uint2 *W = (uint2 *)region;
    uint32_t *L0 = (uint32_t *)region;
    uint8_t *slots = region + lay.off_slots;
    const uint32_t cap_n = p.area / 6, cap_w = p.area / (uint32_t)(sizeof(V) * Sem::kSlots + 2);
    const S bv0 = (S)bvmax;
    S *cval = (S *)p.c_val;
    const uint32_t WIN = p.ww * 32;
    const unsigned long long tag = (unsigned long long)f.epoch << kLbEpochShift;
    // rows by wave: row = wave + k * nwaves, in order (every wave of the grid is resident, so the
    // owner of any row a look-back waits on is running; the spin limit covers the case it is not)
    const uint64_t wid = (uint64_t)blockIdx.x * (kBlock / kWave) + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    for (uint64_t row = wid; row < p.nrows; row += f.nwaves) {
        const I a0 = (I)p.a_rp[row], a1 = (I)p.a_rp[row + 1];
        uint32_t wcnt = 0, zeros = 0;
        if (a1 > a0) {
            SegRow<Sem, I, UNI> rw(p, a0, a1);
            // 2. the row's column bitmap
            BitmapPass<S, 2, true> bm{L0, 0u, WIN};
            rw.cols(bm);
            wave_sync();
            // 3. word ranks over the touched 64-word blocks
            const uint32_t bmask = wave_or_u32(bm.blk);
            for (uint32_t m = bmask; m; m &= m - 1) {
                const uint32_t w = (uint32_t)__builtin_ctz(m) * kWave + lane;
                const uint32_t c = __popc(W[w].x);
                const uint32_t incl = wave_incl_scan(c, 0u, [](uint32_t x, uint32_t y) { return x + y; });
                W[w].y = wcnt + incl - c;
                wcnt += readlane_u32(incl, kWave - 1);
            }
            if (lane == 0) arrive(f, row, wcnt);
            // narrow u32 slots when no partial sum can reach 2^32
            bool narrow = false;
            if constexpr (Sem::kNarrowable) {
                if (bvmax != 0xFFFFFFFFu) {
                    const uint64_t x = (uint64_t)wave_max_u32(rw.amax) * bvmax;
                    narrow = x == 0 || rw.len <= 0xFFFFFFFFull / x;
                }
            }
            uint64_t out_pos = 0;
            bool located = false, gave_up = false;
            auto locate = [&]() {
                if (located) return;
                located = true;
                if (!SLAT_FUSED_NOLB && !look_back(f, row, out_pos)) {
                    gave_up = true;
                    return;
                }
                settle(f, row, out_pos, wcnt);
            };
            // one rank chunk [r0, r0 + nch): values from the cached groups, then the emit
            auto chunk = [&](auto narrow_tag, uint32_t r0, uint32_t cap) {
                constexpr bool NW = decltype(narrow_tag)::value;
                using VS = std::conditional_t<NW, uint32_t, V>;
                constexpr uint32_t kVW = NW ? 1 : Sem::kSlots;
                VS *vals = (VS *)slots;
                uint16_t *cols = (uint16_t *)(slots + ((cap * kVW * sizeof(VS) + 3) & ~3u));
                const uint32_t nch = min(cap, wcnt - r0);
                if (r0 == 0 && nch == wcnt) {
                    AccPass<Sem, NW, true, true, UNI> acc{W, vals, cols, p.ww, 0u, 0u, nch, nullptr};
                    if constexpr (NW) rw.template prods<SemU32Narrow>(acc, bv0);
                    else rw.template prods<Sem>(acc, bv0);
                } else {
                    AccPass<Sem, NW, true, false, UNI> acc{W, vals, cols, p.ww, 0u, r0, nch, nullptr};
                    if constexpr (NW) rw.template prods<SemU32Narrow>(acc, bv0);
                    else rw.template prods<Sem>(acc, bv0);
                }
                wave_sync();
                locate();
                if (gave_up) {  // leave the slots clean; nothing is emitted
                    for (uint32_t q = lane; q < nch; q += kWave) {
#pragma unroll
                        for (uint32_t w = 0; w < kVW; ++w) vals[q * kVW + w] = VS(0);
                        cols[q] = 0;
                    }
                    wave_sync();
                    return;
                }
                uint32_t *oc = p.c_col + out_pos + r0;
                S *ov = cval + out_pos + r0;
                for (uint32_t q = lane; q < nch; q += kWave) {
                    S v;
                    if constexpr (NW) v = (S)vals[q];
                    else v = Sem::finish((const V *)vals, q);
                    const uint32_t col = cols[q];
#pragma unroll
                    for (uint32_t w = 0; w < kVW; ++w) vals[q * kVW + w] = VS(0);
                    cols[q] = 0;
                    zeros += Sem::is_zero(v) ? 1u : 0u;
                    oc[q] = col;
                    ov[q] = v;
                }
                wave_sync();
            };
            if constexpr (Sem::kNarrowable) {
                if (narrow) {
                    for (uint32_t r0 = 0; r0 < wcnt; r0 += cap_n) chunk(std::true_type{}, r0, cap_n);
                } else {
                    for (uint32_t r0 = 0; r0 < wcnt; r0 += cap_w) chunk(std::false_type{}, r0, cap_w);
                }
            } else {
                for (uint32_t r0 = 0; r0 < wcnt; r0 += cap_w) chunk(std::false_type{}, r0, cap_w);
            }
            locate();  // a row whose products touch no column
            for (uint32_t m = bmask; m; m &= m - 1) W[(uint32_t)__builtin_ctz(m) * kWave + lane].x = 0;
            wave_sync();
            if (gave_up) return;
        } else {
            if (lane == 0) arrive(f, row, 0);
            uint64_t out_pos = 0;
            if (!SLAT_FUSED_NOLB && !look_back(f, row, out_pos)) return;
            settle(f, row, out_pos, 0);
        }
        const uint32_t rz = wave_sum_u32(zeros);
        if (lane == 0) p.counts[row] = wcnt - rz;
        zrows += rz ? 1u : 0u;
        rowmax = max(rowmax, wcnt);
    }
}

template <typename Sem, typename I>
__global__ __launch_bounds__(kBlock, SLAT_FUSED_WPS) void k_fused(FusedArgs f) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    const Args &p = f.a;
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const NumLayout lay = num_layout(p.ww, p.area);
    uint8_t *region = smem8 + (size_t)wv * lay.bytes;
    uint2 *W = (uint2 *)region;
    uint8_t *slots = region + lay.off_slots;
    for (uint32_t w = lane; w < p.ww; w += kWave) W[w] = make_uint2(0u, 0u);
    if (lane == 0) W[p.ww] = make_uint2(0u, 0x80000000u);  // dummy word: out-of-window columns
    for (uint32_t w = lane; w < p.area / 4; w += kWave) ((uint32_t *)slots)[w] = 0;
    wave_sync();
    // max(B) and whether B is a pattern (max == min), from k_build_ell's epoch-tagged words
    uint32_t bvmax = 0xFFFFFFFFu;
    bool buni = false;
    if constexpr (Sem::kNarrowable) {
        if (p.b_vmax) {
            const unsigned long long v = ((volatile unsigned long long *)p.b_vmax)[kVMaxWord];
            const unsigned long long vi = ((volatile unsigned long long *)p.b_vmax)[kVMinInvWord];
            if ((uint32_t)(v >> 32) == p.epoch) {
                bvmax = (uint32_t)v;
                buni = (uint32_t)(vi >> 32) == p.epoch && ~(uint32_t)vi == bvmax;
            }
        }
    }
    uint32_t zrows = 0, rowmax = 0;
    if (buni)
        fused_rows<Sem, I, true>(f, region, bvmax, zrows, rowmax);
    else
        fused_rows<Sem, I, false>(f, region, bvmax, zrows, rowmax);
    // the call's totals: max row count into the epoch-tagged word; the last wave to finish writes
    // nnz (row_ptr[n]) and the max into mapped host memory
    if (lane == 0) {
        if (zrows)
            __hip_atomic_fetch_add(&p.host_out[2], (unsigned long long)zrows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        atomicMax(f.maxw, ((unsigned long long)f.epoch << 32) | rowmax);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned long long d = atomicAdd(f.done, 1ull) - f.done_base;
        if (d == (unsigned long long)f.nwaves - 1) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            const unsigned long long nnz =
                __hip_atomic_load((unsigned long long *)&p.c_rp[p.nrows], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long mw = __hip_atomic_load(f.maxw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&p.host_out[0], nnz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&p.host_out[1], (uint32_t)(mw >> 32) == f.epoch ? (mw & 0xFFFFFFFFull) : 0ull,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <typename Sem, typename I>
static hipError_t launch_fused_t(dim3 grid, size_t lds, hipStream_t s, const FusedArgs &f) {
    hipLaunchKernelGGL((k_fused<Sem, I>), grid, dim3(kBlock), lds, s, f);
    return hipGetLastError();
}

template <typename Sem, typename I>
static int fused_blocks_per_cu(size_t lds) {
    int nb = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_fused<Sem, I>, kBlock, lds);
    return (e == hipSuccess && nb > 0) ? nb : 1;
}

}  // namespace slat

using namespace slat;

// One fused launch (see the file comment). `a` is the numeric pass's argument block (ELL copy of B
// built, C allocated by the bound, counts workspace set); the look-back words live in the context.
// *gave_up: the kernel abandoned the call (its grid was not resident); the caller reruns the product
// on the three-kernel path.
slat_status slat_launch_fused(slat_ctx *ctx, const Args &a, int32_t dtype, bool idx32, size_t lds) {
    const hipStream_t s = ctx->stream;
    const uint64_t n = a.nrows;
    const uint64_t groups = (n + 63) / 64;
    if (n > ctx->lb_cap) {
        if (ctx->lb_status) slat_dev_free(ctx, ctx->lb_status, s);
        ctx->lb_status = nullptr;
        const uint64_t cap = std::max<uint64_t>((n + 63) & ~63ull, 4096);
        // [cap] row words | [cap / 64] group words | [cap / 64] group arrival counters
        const size_t bytes = (cap + 2 * (cap / 64)) * 8;
        SLAT_HIP(ctx, slat_dev_alloc(ctx, (void **)&ctx->lb_status, bytes, s));
        SLAT_HIP(ctx, hipMemsetAsync(ctx->lb_status, 0, bytes, s));
        ctx->lb_cap = cap;
    }
    if (++ctx->lb_epoch >= (1u << 20)) {  // tag wrap: clear every tagged word once
        SLAT_HIP(ctx, hipMemsetAsync(ctx->lb_status, 0, (ctx->lb_cap + ctx->lb_cap / 64) * 8, s));
        SLAT_HIP(ctx, hipMemsetAsync(ctx->d_words + 5, 0, 8, s));
        ctx->lb_epoch = 1;
    }
    // a resident grid: rows are assigned by wave, so every wave must run at once
    static thread_local int cache_nb[8] = {};
    static thread_local size_t cache_lds[8] = {};
    const int ci = (dtype == SLAT_SAT64 ? 4 : 0) | (idx32 ? 2 : 0);
    if (cache_lds[ci] != lds || cache_nb[ci] == 0) {
        cache_lds[ci] = lds;
        cache_nb[ci] = dtype == SLAT_SAT64 ? (idx32 ? fused_blocks_per_cu<SemSat64, uint32_t>(lds)
                                                    : fused_blocks_per_cu<SemSat64, uint64_t>(lds))
                                           : (idx32 ? fused_blocks_per_cu<SemU32, uint32_t>(lds)
                                                    : fused_blocks_per_cu<SemU32, uint64_t>(lds));
    }
    const uint64_t wpb = kBlock / kWave;
    const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((n + wpb - 1) / wpb, (uint64_t)ctx->cu_count * cache_nb[ci]));
    FusedArgs f;
    f.a = a;
    f.status = ctx->lb_status;
    f.gstat = ctx->lb_status + ctx->lb_cap;
    f.gacc = ctx->lb_status + ctx->lb_cap + ctx->lb_cap / 64;
    f.done = ctx->d_words + 6;
    f.done_base = ctx->lb_done;
    f.maxw = ctx->d_words + 5;
    f.abort = (unsigned int *)(ctx->d_words + 7);
    f.epoch = ctx->lb_epoch;
    f.nwaves = (uint32_t)(blocks * wpb);
    (void)groups;
    hipError_t e;
    if (dtype == SLAT_SAT64)
        e = idx32 ? launch_fused_t<SemSat64, uint32_t>(dim3((unsigned)blocks), lds, s, f)
                  : launch_fused_t<SemSat64, uint64_t>(dim3((unsigned)blocks), lds, s, f);
    else
        e = idx32 ? launch_fused_t<SemU32, uint32_t>(dim3((unsigned)blocks), lds, s, f)
                  : launch_fused_t<SemU32, uint64_t>(dim3((unsigned)blocks), lds, s, f);
    SLAT_HIP(ctx, e);
    ctx->lb_done += f.nwaves;
    return SLAT_OK;
}

// after a fused launch gave up: clear its abort word and the group counters it left behind
slat_status slat_fused_reset(slat_ctx *ctx) {
    const hipStream_t s = ctx->stream;
    SLAT_HIP(ctx, hipMemsetAsync(ctx->d_words + 7, 0, 8, s));
    SLAT_HIP(ctx, hipMemsetAsync(ctx->lb_status + ctx->lb_cap + ctx->lb_cap / 64, 0, ctx->lb_cap / 64 * 8, s));
    ctx->h_out[3] = 0;
    return SLAT_OK;
}
