// slat_tiny.hip — the whole SpGEMM of a small product in ONE regular kernel launch (SURVEY.md §8(d)
// config C3's small cells: 5^3 .. 15^3 tori, 125 .. 3375 rows). There the regular pipeline's four
// launches (ELL build, symbolic, scan, numeric) cost more host time (~4.5 us each on this runtime)
// than the work itself.
//
// k_tiny: one wavefront per row, every row in flight at once (grid = rows / 4 blocks, all resident):
//   1. the row's column bitmap and word ranks in LDS (numeric's steps 1-2: B walked in CSR form, no
//      ELL image to build); the rank total IS the row's structural count;
//   2. the block's counts summed in LDS, then the block's offset by a decoupled look-back over the
//      earlier blocks' epoch-tagged status words (lookback_prefix_wave: the first wave reads 256
//      predecessors per round) — no grid
//      barrier, no cooperative launch: a block only ever waits on lower-numbered blocks, which the
//      hardware dispatched before it;
//   3. row_ptr[row + 1] stored, then the row's values accumulated in rank slots and emitted sorted
//      from the bitmap it still holds (no second traversal for the structure, nothing stored between
//      passes); the last block stores the call's completion word (signal_done).
// A round-3 predecessor used a cooperative grid with a grid barrier, every block re-scanning all
// counts and a second full traversal; it measured slower than the pipeline (34-80 vs 28-45 us per
// call, profiles/r03_small_cells_tiny_vs_regular.csv) and was removed.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "slat_launch.hpp"
#include "spgemm_kernels.hpp"

using namespace slat;

namespace {

template <typename Sem>
__global__ __launch_bounds__(kBlock) void k_tiny(Args p, unsigned long long *status, uint32_t epoch,
                                                 unsigned long long *maxw) {
    using I = uint32_t;
    using S = typename Sem::S;
    using V = typename Sem::V;
    constexpr int kWpb = kBlock / kWave;
    constexpr bool kVals = !Sem::kOrdered;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    __shared__ uint32_t s_cnt[kWpb];
    __shared__ unsigned long long s_pre;
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t row = (uint64_t)blockIdx.x * kWpb + wv;
    const bool has = row < p.nrows;
    const NumLayout lay = num_layout(p.ww, p.area);
    uint8_t *region = smem8 + (size_t)wv * lay.bytes;
    uint2 *W = (uint2 *)region;
    uint32_t *L0 = (uint32_t *)region;  // L0[2w] aliases W[w].x
    uint8_t *slots = region + lay.off_slots;
    for (uint32_t w = lane; w < p.ww; w += kWave) W[w] = make_uint2(0u, 0u);
    if (lane == 0) W[p.ww] = make_uint2(0u, 0x80000000u);  // dummy word of out-of-window columns
    for (uint32_t w = lane; w < p.area / 4; w += kWave) ((uint32_t *)slots)[w] = 0;
    wave_sync();

    // 1. bitmap and word ranks of the row
    I a0 = 0, a1 = 0;
    if (has) {
        a0 = (I)p.a_rp[row];
        a1 = (I)p.a_rp[row + 1];
    }
    RowWalker<Sem, I, false, kVals> rw(p, a0, a1);
    uint32_t wcnt = 0;
    if (a1 > a0) {
        BitmapPass<S, 2, true> bm{L0, 0u, p.ww * 32};
        rw.template each_group<false>(bm);
        wave_sync();
        for (uint32_t m = wave_or_u32(bm.blk); m; m &= m - 1) {
            const uint32_t w = (uint32_t)__builtin_ctz(m) * kWave + lane;
            const uint32_t c = __popc(W[w].x);
            const uint32_t incl = wave_incl_scan(c, 0u, [](uint32_t x, uint32_t y) { return x + y; });
            W[w].y = wcnt + incl - c;
            wcnt += readlane_u32(incl, kWave - 1);
        }
        wave_sync();
    }

    // 2. the block's offset: its aggregate published, the earlier blocks' looked back over
    if (lane == 0) s_cnt[wv] = wcnt;
    __syncthreads();
    if (threadIdx.x < kWave) {  // the first wave: the look-back reads 64 predecessors per round
        unsigned long long agg = 0;
        uint32_t mx = 0;
#pragma unroll
        for (int k = 0; k < kWpb; ++k) {
            agg += s_cnt[k];
            mx = max(mx, s_cnt[k]);
        }
        // the max row first (its result waited for): it is in place once a later block sees this
        // block's status, so the last block reads the final max after its look-back
        if (threadIdx.x == 0) maxw_raise(maxw, epoch, mx);
        const unsigned long long excl = lookback_prefix_wave(status, blockIdx.x, epoch, agg);
        if (threadIdx.x == 0) s_pre = excl;
        const bool last = blockIdx.x == gridDim.x - 1;
        const unsigned long long mxr = last ? maxw_read(maxw, epoch) : 0u;
        if (threadIdx.x == 0 && last) {
            // returned values: both words have landed before this block reports done (signal_done)
            const unsigned long long o0 =
                __hip_atomic_exchange(&p.host_out[0], excl + agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const unsigned long long o1 = __hip_atomic_exchange(&p.host_out[1], mxr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            asm volatile("" ::"v"(o0), "v"(o1));
        }
    }
    __syncthreads();
    uint64_t out = s_pre;
    for (int k = 0; k < wv; ++k) out += s_cnt[k];
    if (has && lane == 0) {
        p.c_rp[row + 1] = out + wcnt;
        if (row == 0) p.c_rp[0] = 0;
    }

    // 3. values per rank chunk, emitted sorted at the row's slice
    uint32_t zeros = 0;
    if (wcnt) {
        const uint32_t cap = p.area / (uint32_t)(sizeof(V) * Sem::kSlots + 2);
        V *vals = (V *)slots;
        uint16_t *cols = (uint16_t *)(slots + ((cap * Sem::kSlots * sizeof(V) + 3) & ~3u));
        PhaseClock pc{};
        for (uint32_t r0 = 0; r0 < wcnt; r0 += cap) {
            const uint32_t nch = min(cap, wcnt - r0);
            if constexpr (Sem::kOrdered) {
                // the reference's left fold: lanes over one B row at a time, A entries in order
                traverse_ordered<I, S>(p, a0, a1, [&](uint32_t j, S a, S b) {
                    uint32_t off;
                    const uint2 w = rank_word(W, p.ww, j, 0u, off);
                    const uint32_t r = rank_in(w, off, r0, nch);
                    if (r != kSent) {
                        Sem::acc(vals, r, Sem::prod(a, b));
                        cols[r] = (uint16_t)off;
                    }
                });
            } else {
                AccPass<Sem, false, false, false, false> acc{W, vals, cols, p.ww, 0u, r0, nch, &pc};
                rw.template each_group<true>(acc);
            }
            wave_sync();
            uint32_t *oc = p.c_col + out + r0;
            S *ov = (S *)p.c_val + out + r0;
            for (uint32_t t = lane; t < nch; t += kWave) {
                const S v = Sem::finish(vals, t);
                oc[t] = cols[t];
                ov[t] = v;
                zeros += Sem::is_zero(v) ? 1u : 0u;
#pragma unroll
                for (int k = 0; k < Sem::kSlots; ++k) vals[t * Sem::kSlots + k] = V(0);
                cols[t] = 0;
            }
            wave_sync();
        }
    }
    const uint32_t rz = wave_sum_u32(zeros);
    if (has && lane == 0) p.counts[row] = wcnt - rz;  // non-zero count (compaction input)
    add_zero_rows(&p.host_out[2], rz ? 1u : 0u, true);
    signal_done(p);
}

template <typename Sem>
hipError_t launch(dim3 grid, size_t lds, hipStream_t s, const Args &a, unsigned long long *status, uint32_t epoch,
                  unsigned long long *maxw) {
    hipLaunchKernelGGL(k_tiny<Sem>, grid, dim3(kBlock), lds, s, a, status, epoch, maxw);
    return hipGetLastError();
}

}  // namespace

hipError_t slat_launch_tiny(int sem, dim3 grid, size_t lds, hipStream_t s, const Args &a, unsigned long long *status,
                            uint32_t epoch, unsigned long long *maxw) {
    switch (sem) {
    case kSemU32: return launch<SemU32>(grid, lds, s, a, status, epoch, maxw);
    case kSemSat64: return launch<SemSat64>(grid, lds, s, a, status, epoch, maxw);
    case kSemF64: return launch<SemF64>(grid, lds, s, a, status, epoch, maxw);
    default: return launch<SemF64Any>(grid, lds, s, a, status, epoch, maxw);
    }
}
