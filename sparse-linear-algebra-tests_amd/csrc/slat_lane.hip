// slat_lane.hip — products whose rows are all short (at most kLaneCap products each: the 30^3 chain's
// C1 = A * A, 27 000 rows of ~12 products) in ONE kernel, a row per LANE (SURVEY.md §8(d) config C1;
// the fixed per-row cost of the single-window path).
//
// The pipeline gives such a call four launches and a wave per row, so each wave walks ~9 rows of ~12
// products one after another, every row a chain of dependent loads (bounds, A entries, B rows, stored
// bitmap) that nothing hides: C1 took 88 us, 46 of them in k_numeric. Here a wave owns 64 rows:
//
//   1. the rows' A entries (contiguous in A) are walked 256 at a time, four per lane; each entry
//      learns its row (a marker at the row's first entry, a running max), its B row's length, and its
//      products' offset in the wave's flattened product space (a wave prefix);
//   2. the products are walked flattened, 256 per pass, every lane on one (an entry by markers, as
//      the fat rows' fr_flat) and written into their row's lane of an LDS slot table (slot s of row l
//      at s * rows + l) as (column << 6 | slot, product): the slot is the product's position in the
//      row, A order then B order, so the key is unique and keeps the reference's order for equal
//      columns;
//   3. every lane sorts its row's keys in registers (a bitonic network of 16, 32 or 64 keys, the
//      wave's longest row decides; the values stay in LDS, found by the slot in the key) and counts
//      its distinct columns;
//   4. the wave's offset by a decoupled look-back over the earlier waves' status words (one wave per
//      block; lookback_walk reads 256 predecessors per round), then row_ptr, and the rows'
//      sums in key order — the f64 left fold from 0.0 in A order, the saturating integer sums — are
//      stored; zero sums (explicit zero inputs, f64 cancellation) are counted for the host's
//      compaction, as after k_numeric. The last block stores
//      nnz, the max row and the completion word.
//
// A row of more than kLaneCap products sets the mapped overflow word: the host then runs the call
// through the pipeline (the host only tries this kernel when max row(A) x max row(B) <= 4 kLaneCap).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "slat_launch.hpp"
#include "spgemm_kernels.hpp"

using namespace slat;

namespace {

constexpr uint32_t kLaneCap = 64;   // products per row (sort slots per lane)
constexpr uint32_t kLaneRows = 64;  // rows per one-wave block (a row per lane)
constexpr uint32_t kLaneSeg = 256;  // A entries / products per pass (four per lane)
#ifndef SLAT_LANE_PG
#define SLAT_LANE_PG 4
#endif
constexpr uint32_t kLanePG = SLAT_LANE_PG;  // product passes whose loads are issued together (variant builds: 1)

template <typename S>
__host__ __device__ constexpr size_t lane_lds() {
    // slot keys u32[64 * rows] | slot values S[64 * rows] | entry bases u32[256] | entry A values S[256] |
    // entry rows u8[256] | entry markers u8[256] | product markers u16[256] | row bases u32[64] |
    // row counts u32[64]
    // (+ u32 values: an output-value staging area u32[64 * rows], so the wave's outputs are stored
    // coalesced; the columns stage in the slot keys' area, free once the keys are in registers)
    return (size_t)kLaneCap * kLaneRows * (4 + sizeof(S)) + kLaneSeg * (4 + sizeof(S) + 1 + 1 + 2 * kLanePG) + kWave * 8 +
           (sizeof(S) == 4 ? (size_t)kLaneCap * kLaneRows * 4 : 0);
}

// the semiring's running sum of one output
template <typename Sem>
struct LaneSum {
    using S = typename Sem::S;
    using T = std::conditional_t<std::is_same_v<Sem, SemU32>, unsigned long long, S>;
    __device__ static __forceinline__ T first(S p) {
        if constexpr (std::is_same_v<S, double>)
            return __dadd_rn(0.0, p);  // the reference's fold starts from 0.0 (0.0 + -0.0 = +0.0)
        else
            return (T)p;
    }
    __device__ static __forceinline__ T add(T s, S p) {
        if constexpr (std::is_same_v<S, double>)
            return __dadd_rn(s, p);  // no FMA contraction: a*b then +
        else if constexpr (std::is_same_v<Sem, SemU32>)
            return s + p;  // < 64 products of < 2^32: exact in u64, clamped at the end
        else
            return s + p < s ? ~0ull : s + p;  // Saturating<u64>
    }
    __device__ static __forceinline__ S done(T s) {
        if constexpr (std::is_same_v<Sem, SemU32>)
            return s > 0xFFFFFFFFull ? 0xFFFFFFFFu : (S)s;
        else
            return s;
    }
};

// ascending bitonic sort of the lane's N keys (compile-time indices only). The keys are unique
// (column << 6 | slot) and carry their slot, so no payload moves: each compare-exchange is one min
// and one max
template <int N>
__device__ __forceinline__ void lane_sort(uint32_t (&k)[kLaneCap]) {
#pragma unroll
    for (int size = 2; size <= N; size <<= 1)
#pragma unroll
        for (int stride = size / 2; stride > 0; stride >>= 1)
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const int j = i ^ stride;
                if (j > i) {
                    const uint32_t lo = min(k[i], k[j]), hi = max(k[i], k[j]);
                    const bool asc = (i & size) == 0;
                    k[i] = asc ? lo : hi;
                    k[j] = asc ? hi : lo;
                }
            }
}

// the lane's sorted keys: distinct columns (the row's structural count; no values read)
template <int N>
__device__ __forceinline__ uint32_t lane_count(const uint32_t (&k)[kLaneCap]) {
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < N; ++i)
        nz += (k[i] != kSent && (i == 0 || (k[i] >> 6) != (k[i - 1] >> 6))) ? 1u : 0u;
    return nz;
}

// the lane's sorted keys: emit(col, value, index) for each column's sum in column order (values by
// slot from the lane's column of the slot table); returns the number of zero sums among them
template <typename Sem, int N, typename F>
__device__ __forceinline__ uint32_t lane_combine(const uint32_t (&k)[kLaneCap], const typename Sem::S *sv, F &&emit) {
    using L = LaneSum<Sem>;
    typename L::T s{};
    uint32_t prev = kSent, j = 0, zeros = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint32_t c = k[i] == kSent ? kSent : k[i] >> 6;
        const typename Sem::S v = c == kSent ? typename Sem::S(0) : sv[(k[i] & 63u) * kLaneRows];
        if (c != prev) {
            if (prev != kSent) {
                const auto out = L::done(s);
                zeros += Sem::is_zero(out) ? 1u : 0u;
                emit(prev, out, j++);
            }
            if (c != kSent) s = L::first(v);
            prev = c;
        } else if (c != kSent) {
            s = L::add(s, v);
        }
    }
    if (prev != kSent) {
        const auto out = L::done(s);
        zeros += Sem::is_zero(out) ? 1u : 0u;
        emit(prev, out, j++);
    }
    return zeros;
}

template <typename Sem>
__global__ __launch_bounds__(kWave) void k_lane(Args p, unsigned long long *status, uint32_t epoch,
                                                unsigned long long *maxw) {
    using S = typename Sem::S;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t *skey = (uint32_t *)smem;
    S *sval = (S *)(smem + kLaneCap * kLaneRows * 4);
    uint8_t *q = smem + kLaneCap * kLaneRows * (4 + sizeof(S));
    uint32_t *eb = (uint32_t *)q;
    S *ea = (S *)(q + kLaneSeg * 4);
    uint8_t *erl = q + kLaneSeg * (4 + sizeof(S));
    uint8_t *amk = erl + kLaneSeg;
    uint16_t *pmk = (uint16_t *)(amk + kLaneSeg);
    uint32_t *rbase = (uint32_t *)(pmk + kLaneSeg * kLanePG), *rcnt = rbase + kWave;
    S *stg = (S *)(rcnt + kWave);  // (u32 values) the outputs' value staging
    const uint32_t lane = (uint32_t)lane_id();
    const S *av = (const S *)p.a_val;
    const S *bv = (const S *)p.b_val;
    const auto plus = [](uint32_t x, uint32_t y) { return x + y; };
    const auto mx = [](uint32_t x, uint32_t y) { return max(x, y); };

    PhaseClock pc{};  // diagnostic builds (SLAT_PHASES): where a wave's time goes
    if constexpr (SLAT_PHASES) pc.t = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = (uint64_t)blockIdx.x * kLaneRows, r = r0 + lane;
    const uint32_t nt = (uint32_t)min<uint64_t>(kLaneRows, p.nrows - r0);
    uint32_t A0j = 0, A1j = 0;
    if (lane < nt) {
        A0j = (uint32_t)p.a_rp[r];
        A1j = (uint32_t)p.a_rp[r + 1];
    }
    const uint32_t A0 = readlane_u32(A0j, 0), A1 = readlane_u32(A1j, (int)nt - 1);
    for (uint32_t w = lane; w < kLaneSeg / 4; w += kWave) ((uint32_t *)amk)[w] = 0;
    for (uint32_t w = lane; w < kLaneSeg * kLanePG / 2; w += kWave) ((uint32_t *)pmk)[w] = 0;
    rcnt[lane] = 0;
    rbase[lane] = 0;
    wave_sync();

    pc.mark(0);  // row bounds, LDS init
    // 1-2. entries 256 at a time, then their products flattened
    uint32_t rcarry = 0, fcarry = 0;  // row lane (+1) running into the segment, flat products so far
    for (uint32_t sb = A0; sb < A1; sb += kLaneSeg) {
        // each row's first entry in this segment marks its lane (a later non-empty row wins a tie
        // with empty rows before it)
        if (lane < nt && A1j > A0j && A0j >= sb && A0j - sb < kLaneSeg) amk[A0j - sb] = (uint8_t)(lane + 1);
        wave_sync();
        uint32_t rl[4], kq[4], bl[4], off[4], first[4];
        S aq[4];
        sfor<4>([&](auto Q) {
            const uint32_t i = sb + Q * kWave + lane;
            const uint32_t m = amk[Q * kWave + lane];
            first[Q] = m;
            const uint32_t run = max(wave_incl_scan(m, 0u, mx), rcarry);
            rcarry = readlane_u32(run, kWave - 1);
            rl[Q] = run - 1;
            kq[Q] = kSent;
            aq[Q] = S(0);
            if (i < A1) {
                kq[Q] = p.a_col[i];
                aq[Q] = av[i];
            }
        });
        sfor<4>([&](auto Q) { amk[Q * kWave + lane] = 0; });
        uint32_t bs[4];
        sfor<4>([&](auto Q) {
            bs[Q] = 0;
            bl[Q] = 0;
            if (kq[Q] < p.b_nrows) {
                const uint64_t b0 = p.b_rp[kq[Q]], b1 = p.b_rp[kq[Q] + 1];
                bs[Q] = (uint32_t)b0;
                bl[Q] = (uint32_t)min<uint64_t>(b1 - b0, kLaneCap + 1);  // (a longer row overflows)
            }
        });
        uint32_t stot = 0;
        sfor<4>([&](auto Q) {
            const uint32_t incl = wave_incl_scan(bl[Q], 0u, plus);
            off[Q] = fcarry + stot + incl - bl[Q];
            stot += readlane_u32(incl, kWave - 1);
        });
        sfor<4>([&](auto Q) {
            const uint32_t e = Q * kWave + lane;
            if (first[Q] && sb + e < A1) rbase[rl[Q]] = off[Q];  // the row's first entry
            if (sb + e < A1 && bl[Q]) atomicAdd(&rcnt[rl[Q]], bl[Q]);
            eb[e] = bs[Q] - off[Q];  // product t of the entry: B index eb + t
            ea[e] = aq[Q];
            erl[e] = (uint8_t)rl[Q];
        });
        wave_sync();
        pc.mark(1);  // entries: rows, B row bounds, offsets
        // the segment's products, 256 per pass, kLanePG passes at a time (their loads in flight
        // together): entry by markers, slot = t - the row's base
        constexpr uint32_t kSpan = kLaneSeg * kLanePG, kQ = 4 * kLanePG;
        for (uint32_t p0 = 0; p0 < stot; p0 += kSpan) {
            const uint32_t t0 = fcarry + p0;
            sfor<4>([&](auto Q) {
                if (bl[Q] && off[Q] < t0 + kSpan && off[Q] + bl[Q] > t0)
                    pmk[max(off[Q], t0) - t0] = (uint16_t)(Q * kWave + lane + 1);
            });
            wave_sync();
            uint32_t L[kQ], carry = 0;
            sfor<kQ>([&](auto Q) {
                const uint32_t m = pmk[Q * kWave + lane];
                L[Q] = max(wave_incl_scan(m, 0u, mx), carry);
                carry = readlane_u32(L[Q], kWave - 1);
            });
            for (uint32_t w = lane; w < kSpan / 2; w += kWave) ((uint32_t *)pmk)[w] = 0;
            uint32_t c[kQ], row[kQ], slot[kQ];
            S v[kQ], a[kQ];
            sfor<kQ>([&](auto Q) {
                const uint32_t t = t0 + Q * kWave + lane;
                c[Q] = kSent;
                v[Q] = a[Q] = S(0);
                row[Q] = slot[Q] = 0;
                if (t < fcarry + stot) {
                    const uint32_t e = L[Q] - 1;  // position 0 is always marked: L >= 1
                    const uint32_t bi = eb[e] + t;
                    row[Q] = erl[e];
                    slot[Q] = t - rbase[row[Q]];
                    a[Q] = ea[e];
                    c[Q] = p.b_col[bi];
                    v[Q] = bv[bi];
                }
            });
            sfor<kQ>([&](auto Q) {
                if (c[Q] != kSent && slot[Q] < kLaneCap) {
                    skey[slot[Q] * kLaneRows + row[Q]] = (c[Q] << 6) | slot[Q];
                    sval[slot[Q] * kLaneRows + row[Q]] = Sem::prod(a[Q], v[Q]);
                }
            });
            wave_sync();
        }
        fcarry += stot;
        pc.mark(2);  // products into the slot table
    }

    // 3. the lane's row: its slots sorted in registers, equal columns summed
    const uint32_t cnt = lane < nt ? rcnt[lane] : 0u;
    if (cnt > kLaneCap)  // the host runs the call through the pipeline instead
        __hip_atomic_store(&p.host_out[3], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t cn = cnt > kLaneCap ? 0u : cnt;
    const uint32_t wmax = wave_max_u32(cn);
    // sorted once (network size by the wave's longest row); the non-zero count first, then the
    // wave's offset, then the outputs from the same registers
    auto body = [&](auto ntag) {
        constexpr int N = decltype(ntag)::value;
        uint32_t k[kLaneCap];
#pragma unroll
        for (int s = 0; s < N; ++s) k[s] = (uint32_t)s < cn ? skey[s * kLaneRows + lane] : kSent;
        pc.mark(3);
        lane_sort<N>(k);
        pc.mark(4);  // the sort
        const S *sv = sval + lane;  // slot s of this lane's row at sv[s * kLaneRows]
        const uint32_t nz = lane_count<N>(k);  // structural: zero sums are dropped afterwards
        pc.mark(5);  // the count pass
        // 4. the wave's offset (look-back over the earlier blocks), row_ptr, the rows' outputs
        const uint32_t incl = wave_incl_scan(nz, 0u, plus);
        const uint32_t agg = readlane_u32(incl, kWave - 1);
        const uint32_t rmax = wave_max_u32(nz);
        // (the max row first, its result waited for: it is in place once a later block sees this
        // block's status, so the last block reads the final max after its look-back)
        if (lane == 0) pin_u64(atomicMax(maxw, ((unsigned long long)epoch << 32) | rmax));
        // the aggregate published first; u32 rows then stage their outputs in LDS at the wave-local
        // offset while the earlier blocks finish, and only the coalesced store waits for the offset
        lookback_publish(status, blockIdx.x, epoch, agg);
        uint32_t zeros = 0;
        if constexpr (sizeof(S) == 4) {
            const uint32_t o0 = incl - nz;
            if (nz)
                zeros = lane_combine<Sem, N>(k, sv, [&](uint32_t col, S val, uint32_t j) {
                    skey[o0 + j] = col;
                    stg[o0 + j] = val;
                });
            wave_sync();
        }
        pc.mark(7);  // (u32) the outputs staged
        const unsigned long long excl = lookback_walk(status, blockIdx.x, epoch, agg);
        if (lane == 0) {
            if (blockIdx.x == gridDim.x - 1) {
                const unsigned long long mw = __hip_atomic_load(maxw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long mxr = (uint32_t)(mw >> 32) == epoch ? (mw & 0xFFFFFFFFull) : 0ull;
                const unsigned long long o0 =
                    __hip_atomic_exchange(&p.host_out[0], excl + agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                const unsigned long long o1 =
                    __hip_atomic_exchange(&p.host_out[1], mxr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                asm volatile("" ::"v"(o0), "v"(o1));
            }
        }
        pc.mark(6);  // look-back
        const uint64_t base = excl + (incl - nz);
        if (lane < nt) {
            p.c_rp[r + 1] = base + nz;
            if (r == 0) p.c_rp[0] = 0;
        }
        if constexpr (sizeof(S) == 4) {
            // the wave's rows are contiguous in C: the staged outputs stored coalesced (scattered
            // per-lane stores cost one instruction per output)
            uint32_t *oc = p.c_col + excl;
            S *ov = (S *)p.c_val + excl;
            for (uint32_t u = lane; u < agg; u += kWave) {
                oc[u] = skey[u];
                ov[u] = stg[u];
            }
        } else if (nz) {
            uint32_t *oc = p.c_col + base;
            S *ov = (S *)p.c_val + base;
            zeros = lane_combine<Sem, N>(k, sv, [&](uint32_t col, S val, uint32_t j) {
                oc[j] = col;
                ov[j] = val;
            });
        }
        // zero sums (explicit zero inputs, f64 cancellation) stay in C for now: the row's non-zero
        // count goes to p.counts and the rows with zeros to host_out[2], and the host compacts
        // (as after k_numeric)
        if (lane < nt) p.counts[r] = nz - zeros;
        add_zero_rows(&p.host_out[2], wave_sum_u32(zeros ? 1u : 0u), true);
        pc.mark(8);  // row_ptr, the emit
    };
    if (wmax <= 16)
        body(std::integral_constant<int, 16>{});
    else if (wmax <= 32)
        body(std::integral_constant<int, 32>{});
    else
        body(std::integral_constant<int, 64>{});
    if constexpr (SLAT_PHASES) {
        pc.ph[kPhaseSlots - 1] = 1;  // waves
        if (lane == 0) {
            unsigned long long *dst = p.shards + 512 + (blockIdx.x % 64) * kPhaseSlots;
            for (int i = 0; i < kPhaseSlots; ++i) atomicAdd(&dst[i], (unsigned long long)pc.ph[i]);
        }
    }
    signal_done(p);
}

template <typename Sem>
hipError_t launch(dim3 grid, hipStream_t s, const Args &a, unsigned long long *status, uint32_t epoch,
                  unsigned long long *maxw) {
    constexpr size_t lds = lane_lds<typename Sem::S>();
    static bool attr = false;  // > 64 KB of dynamic LDS is not needed (<= 53 KB); set once anyway
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)k_lane<Sem>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    hipLaunchKernelGGL(k_lane<Sem>, grid, dim3(kWave), lds, s, a, status, epoch, maxw);
    return hipGetLastError();
}

}  // namespace

uint32_t slat_lane_cap() { return kLaneCap; }
uint32_t slat_lane_rows() { return kLaneRows; }

hipError_t slat_launch_lane(int sem, dim3 grid, hipStream_t s, const Args &a, unsigned long long *status,
                            uint32_t epoch, unsigned long long *maxw) {
    switch (sem) {
    case kSemU32: return launch<SemU32>(grid, s, a, status, epoch, maxw);
    case kSemSat64: return launch<SemSat64>(grid, s, a, status, epoch, maxw);
    case kSemF64: return launch<SemF64>(grid, s, a, status, epoch, maxw);
    default: return launch<SemF64Any>(grid, s, a, status, epoch, maxw);
    }
}
