// slat_lane.hip — products whose rows are all short (at most kLaneCap products each: the 30^3 chain's
// C1 = A * A, 27 000 rows of ~12 products) in ONE kernel (VERDICT round 3
// item 3, round 4 item 4).
//
// The pipeline gives such a call four launches and a wave per row, so each wave walks ~9 rows of ~12
// products one after another, every row a chain of dependent loads (bounds, A entries, B rows, stored
// bitmap) that nothing hides: C1 took 88 us, 46 of them in k_numeric. Here a block of four waves
// owns 64 consecutive rows, 16 per wave:
//
//   1. a wave's rows' A entries (contiguous in A) are walked 64 at a time, one per lane; each entry
//      learns its row (a marker at the row's first entry, a running max), its B row's length, and its
//      products' offset in the wave's flattened product space (a wave prefix);
//   2. the products are walked flattened, 64 per round, every lane on one (an entry by markers, as
//      the fat rows' fr_flat) and written into their row's column of an LDS slot table (slot s of row
//      r at s * 16 + r) as (column << 6 | slot, product): the slot is the product's position in the
//      row, A order then B order, so the key is unique and keeps the reference's order for equal
//      columns;
//   3. each row's keys are sorted by its QUAD of lanes (a bitonic network of 16, 32 or 64 keys, the
//      wave's longest row decides, 4 / 8 / 16 per lane, DPP quad permutes across the quad) and
//      written back row-major; the quad's first lane then holds the row's sorted keys and counts its
//      distinct columns;
//   4. the block's offset by a decoupled look-back over the earlier blocks' status words (the block
//      aggregate published first, lookback_walk reads 256 predecessors per round); meanwhile u32
//      rows sum equal columns in key order — the saturating integer sums, the f64 left fold from 0.0
//      in A order — into an LDS staging area at their block-local offsets, which the block stores
//      coalesced once its offset is known (8-byte values are summed and stored after the
//      look-back); zero sums (explicit zero inputs, f64 cancellation) are counted for the host's
//      compaction, as after k_numeric. The last block stores nnz, the max row and the completion
//      word.
//
// Round 4's version gave each row one LANE (a 64-key network per lane, 64 rows per one-wave block):
// 422 waves for C1 on 1 024 SIMDs, each a long chain; here four times the waves share it.
// A row of more than kLaneCap products sets the mapped overflow word: the host then runs the call
// through the pipeline (the host only tries this kernel when max row(A) x max row(B) <= 4 kLaneCap).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "slat_launch.hpp"
#include "spgemm_kernels.hpp"

using namespace slat;

namespace {

constexpr uint32_t kLaneCap = 64;                     // products per row (sort slots per row)
constexpr uint32_t kQR = 16;                          // rows per wave (a quad of lanes per row)
constexpr uint32_t kLaneWaves = 4;                    // waves per block
constexpr uint32_t kLaneRows = kQR * kLaneWaves;      // rows per block
constexpr uint32_t kLaneSeg = kWave;                  // A entries per pass (one per lane)
#ifndef SLAT_LANE_PG
#define SLAT_LANE_PG 4
#endif
constexpr uint32_t kLanePG = SLAT_LANE_PG;  // product passes of 64 whose loads are issued together

// LDS of one wave: slot keys u32[64 * 16] (slot-major, then the sorted keys row-major) | slot values
// S[64 * 16] | entry bases u32[64] | entry A values S[64] | entry rows u8[64] | entry markers u8[64] |
// product markers u16[64 * PG] | row bases u32[16] | row counts u32[16]
template <typename S>
__host__ __device__ constexpr size_t lane_wave_lds() {
    return ((size_t)kLaneCap * kQR * (4 + sizeof(S)) + kLaneSeg * (4 + sizeof(S) + 1 + 1) + kLaneSeg * kLanePG * 2 +
            kQR * 8 + 15) & ~(size_t)15;
}
// the block: four wave regions | (u32 values) the block's outputs staged, columns u32[64 * 64] and
// values u32[64 * 64], so they are stored coalesced once the block's offset is known | wave sums
// u32[4] | the block's max row u32 | the broadcast offset u64
template <typename S>
__host__ __device__ constexpr size_t lane_lds() {
    return lane_wave_lds<S>() * kLaneWaves + (sizeof(S) == 4 ? (size_t)kLaneCap * kLaneRows * 8 : 0) + 32;
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

// Ascending bitonic sort of a row's N keys held by its quad of lanes, NL = N / 4 per lane (element
// e = q * NL + j of lane q's register j). The keys are unique (column << 6 | slot) and carry their
// slot, so no payload moves: a compare-exchange is a min and a max. Strides below NL stay in a lane;
// NL and 2 NL exchange with lane q ^ 1 / q ^ 2 of the quad (DPP quad permutes). Against one lane
// per row (a 64-key network per lane, 672 compare-exchanges on C1) the row's sort is ~2.5x shorter
// and a wave holds 16 rows, not 64, so four times the waves share the work.
template <int NL>
__device__ __forceinline__ void quad_sort(uint32_t (&k)[kLaneCap / 4], uint32_t q) {
    constexpr int N = 4 * NL;
#pragma unroll
    for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
        for (int stride = size / 2; stride > 0; stride >>= 1) {
            if (stride < NL) {
#pragma unroll
                for (int j = 0; j < NL; ++j) {
                    const int pj = j ^ stride;
                    if (pj > j) {
                        // ascending iff element e = q * NL + j has bit `size` clear
                        const bool asc = size >= N ? true : size < NL ? (j & size) == 0 : ((q * NL) & size) == 0;
                        const uint32_t lo = min(k[j], k[pj]), hi = max(k[j], k[pj]);
                        k[j] = asc ? lo : hi;
                        k[pj] = asc ? hi : lo;
                    }
                }
            } else {
                const uint32_t m = (uint32_t)(stride / NL);  // 1 or 2: the partner lane q ^ m
                const bool lower = (q & m) == 0;
                const bool asc = size >= N ? true : ((q * NL) & size) == 0;
                const bool keep_min = lower == asc;
#pragma unroll
                for (int j = 0; j < NL; ++j) {
                    const uint32_t o = m == 1 ? lane_xor<1>(k[j]) : lane_xor<2>(k[j]);
                    k[j] = keep_min ? min(k[j], o) : max(k[j], o);
                }
            }
        }
    }
}

// the row's sorted keys (all N in one lane): emit(col, value, index) for each column's sum in column
// order (values by slot: the row's column of the slot table, stride kQR); returns the zero sums
template <typename Sem, int N, typename F>
__device__ __forceinline__ uint32_t lane_combine(const uint32_t (&k)[kLaneCap], const typename Sem::S *sv, F &&emit) {
    using L = LaneSum<Sem>;
    typename L::T s{};
    uint32_t prev = kSent, j = 0, zeros = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint32_t c = k[i] == kSent ? kSent : k[i] >> 6;
        const typename Sem::S v = c == kSent ? typename Sem::S(0) : sv[(k[i] & 63u) * kQR];
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

// quad helpers (DPP quad permutes): lane q's value from quad lane CTRL picks
template <int CTRL>
__device__ __forceinline__ uint32_t quad_perm(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, true);
}
template <int CTRL>
__device__ __forceinline__ unsigned long long quad_perm64(unsigned long long x) {
    return ((unsigned long long)quad_perm<CTRL>((uint32_t)(x >> 32)) << 32) | quad_perm<CTRL>((uint32_t)x);
}
constexpr int kQPrev = 0x90, kQNext = 0xF9, kQFirst = 0x00, kQLast = 0xFF;  // [0,0,1,2] [1,2,3,3] [0,0,0,0] [3,3,3,3]

// Integer semirings: the row's sorted keys stay where the sort left them, NL per quad lane, and the
// quad counts and sums the row's columns together (a quarter of the serial work of one lane walking
// all N keys). A key starts a column when its column differs from the key before it in row order
// (the previous lane's last key for j = 0); the quad's prefix of the starts numbers the outputs. Each
// lane sums its keys' values run by run: elements before its first start belong to a run from an
// earlier lane (its head), and its last run may continue into later lanes, which is the sum of their
// heads up to the first lane with a start of its own. Sums are exact in any order (u32: u64 sums;
// Sat64: saturating), so the split changes nothing. f64 keeps one lane per row (the left fold).
template <int NL>
__device__ __forceinline__ void quad_count(const uint32_t (&kk)[kLaneCap / 4], uint32_t q, uint32_t &starts,
                                           uint32_t &first, uint32_t &total) {
    uint32_t prev = quad_perm<kQPrev>(kk[NL - 1]);
    if (q == 0) prev = kSent;
    starts = 0;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        const uint32_t pk = j == 0 ? prev : kk[j - 1];
        const bool st = kk[j] != kSent && (pk == kSent || (pk >> 6) != (kk[j] >> 6));
        starts |= (st ? 1u : 0u) << j;
    }
    const uint32_t n = __popc(starts);
    uint32_t v = n;
    const uint32_t v1 = quad_perm<kQPrev>(v);
    v += q >= 1 ? v1 : 0u;
    const uint32_t v2 = quad_perm<0x40>(v);  // [0,0,0,1]: lane q - 2
    v += q >= 2 ? v2 : 0u;
    first = v - n;
    total = quad_perm<kQLast>(v);
}

template <typename Sem>
__device__ __forceinline__ typename LaneSum<Sem>::T quad_comb(typename LaneSum<Sem>::T a, typename LaneSum<Sem>::T b) {
    if constexpr (std::is_same_v<Sem, SemU32>)
        return a + b;  // < 2^38
    else
        return a + b < a ? ~0ull : a + b;  // Saturating<u64>
}

// emit(col, value, row output index) for the lane's outputs; returns the lane's zero sums
template <typename Sem, int NL, typename F>
__device__ __forceinline__ uint32_t quad_combine(const uint32_t (&kk)[kLaneCap / 4], uint32_t starts, uint32_t first,
                                                 const typename Sem::S *sv, uint32_t q, F &&emit) {
    using S = typename Sem::S;
    using L = LaneSum<Sem>;
    using T = typename L::T;
    S v[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) v[j] = kk[j] == kSent ? S(0) : sv[(kk[j] & 63u) * kQR];
    T head = 0, cur = 0;
    uint32_t ccol = 0, idx = first, zeros = 0;
    bool seen = false;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        if (kk[j] == kSent) continue;
        if ((starts >> j) & 1u) {
            if (seen) {
                const S out = L::done(cur);
                zeros += Sem::is_zero(out) ? 1u : 0u;
                emit(ccol, out, idx++);
            }
            cur = (T)v[j];
            ccol = kk[j] >> 6;
            seen = true;
        } else if (seen) {
            cur = quad_comb<Sem>(cur, (T)v[j]);
        } else {
            head = quad_comb<Sem>(head, (T)v[j]);
        }
    }
    // X_q = head_q + (a start in lane q ? 0 : X_{q+1}): what lane q adds to a run from before it
    T x = head;
#pragma unroll
    for (int it = 0; it < 3; ++it) {
        const T xn = quad_perm64<kQNext>(x);
        x = (q < 3 && !seen) ? quad_comb<Sem>(head, xn) : head;
    }
    const T xn = quad_perm64<kQNext>(x);
    if (seen) {
        const S out = L::done(quad_comb<Sem>(cur, q < 3 ? xn : T(0)));
        zeros += Sem::is_zero(out) ? 1u : 0u;
        emit(ccol, out, idx);
    }
    return zeros;
}

template <typename Sem>
__global__ __launch_bounds__(kLaneWaves * kWave) void k_lane(Args p, unsigned long long *status, uint32_t epoch,
                                                               unsigned long long *maxw) {
    using S = typename Sem::S;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    uint8_t *wr = smem + (size_t)wv * lane_wave_lds<S>();
    uint32_t *skey = (uint32_t *)wr;
    S *sval = (S *)(wr + kLaneCap * kQR * 4);
    uint8_t *q8 = wr + kLaneCap * kQR * (4 + sizeof(S));
    uint32_t *eb = (uint32_t *)q8;
    S *ea = (S *)(q8 + kLaneSeg * 4);
    uint8_t *erl = q8 + kLaneSeg * (4 + sizeof(S));
    uint8_t *amk = erl + kLaneSeg;
    uint16_t *pmk = (uint16_t *)(amk + kLaneSeg);
    uint32_t *rbase = (uint32_t *)(pmk + kLaneSeg * kLanePG), *rcnt = rbase + kQR;
    uint8_t *blk = smem + lane_wave_lds<S>() * kLaneWaves;
    uint32_t *stc = (uint32_t *)blk;                          // (u32 values) staged columns
    S *stv = (S *)(blk + (size_t)kLaneCap * kLaneRows * 4);   // (u32 values) staged values
    uint32_t *s_wsum = (uint32_t *)(blk + (sizeof(S) == 4 ? (size_t)kLaneCap * kLaneRows * 8 : 0));
    // the 32-byte tail of lane_lds(): wave sums at bytes 0-15, the max row at 16, the offset at 24-31
    static_assert(kLaneWaves * 4 <= 16, "wave sums fit the tail's first 16 bytes");
    uint32_t *s_max = s_wsum + 4;
    unsigned long long *s_off = (unsigned long long *)(s_wsum + 6);
    const S *av = (const S *)p.a_val;
    const S *bv = (const S *)p.b_val;
    const auto plus = [](uint32_t x, uint32_t y) { return x + y; };
    const auto mx = [](uint32_t x, uint32_t y) { return max(x, y); };
    // diagnostic builds (-DSLAT_PHASES=1): s_memtime cycles per phase, summed over waves
    PhaseClock pc{};
    if constexpr (SLAT_PHASES) {
        pc.t = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int i = 0; i < kPhaseSlots; ++i) pc.ph[i] = 0;
        pc.ph[kPhaseSlots - 1] = 1;
    }

    // this wave's rows [r0, r0 + nt): lanes < nt hold their bounds
    const uint64_t r0 = (uint64_t)blockIdx.x * kLaneRows + (uint64_t)wv * kQR;
    const uint32_t nt = r0 < p.nrows ? (uint32_t)min<uint64_t>(kQR, p.nrows - r0) : 0u;
    uint32_t A0j = 0, A1j = 0;
    if (lane < nt) {
        A0j = (uint32_t)p.a_rp[r0 + lane];
        A1j = (uint32_t)p.a_rp[r0 + lane + 1];
    }
    const uint32_t A0 = nt ? readlane_u32(A0j, 0) : 0u, A1 = nt ? readlane_u32(A1j, (int)nt - 1) : 0u;
    amk[lane] = 0;
    for (uint32_t w = lane; w < kLaneSeg * kLanePG / 2; w += kWave) ((uint32_t *)pmk)[w] = 0;
    if (lane < kQR) {
        rcnt[lane] = 0;
        rbase[lane] = 0;
    }
    if (threadIdx.x == 0) *s_max = 0;
    __syncthreads();  // (the block's max row word is clear before any wave adds to it)
    pc.mark(0);  // row bounds

    // 1-2. the rows' entries 64 at a time, then their products flattened into the slot table
    uint32_t rcarry = 0, fcarry = 0;  // row (+1) running into the pass, flat products so far
    for (uint32_t sb = A0; sb < A1; sb += kLaneSeg) {
        // each row's first entry in this pass marks its row (a later non-empty row wins a tie with
        // empty rows before it)
        if (lane < nt && A1j > A0j && A0j >= sb && A0j - sb < kLaneSeg) amk[A0j - sb] = (uint8_t)(lane + 1);
        wave_sync();
        const uint32_t i = sb + lane;
        const uint32_t first = amk[lane];
        const uint32_t run = max(wave_incl_scan(first, 0u, mx), rcarry);
        rcarry = readlane_u32(run, kWave - 1);
        const uint32_t rl = run - 1;
        uint32_t kq = kSent;
        S aq = S(0);
        if (i < A1) {
            kq = p.a_col[i];
            aq = av[i];
        }
        amk[lane] = 0;
        uint32_t bs = 0, bl = 0;
        if (kq < p.b_nrows) {
            const uint64_t b0 = p.b_rp[kq], b1 = p.b_rp[kq + 1];
            bs = (uint32_t)b0;
            bl = (uint32_t)min<uint64_t>(b1 - b0, kLaneCap + 1);  // (a longer row overflows)
        }
        const uint32_t incl = wave_incl_scan(bl, 0u, plus);
        const uint32_t off = fcarry + incl - bl, stot = readlane_u32(incl, kWave - 1);
        pc.mark(1);  // A entries, B row bounds
        if (first && i < A1) rbase[rl] = off;  // the row's first entry
        if (i < A1 && bl) atomicAdd(&rcnt[rl], bl);
        eb[lane] = bs - off;  // product t of the entry: B index eb + t
        ea[lane] = aq;
        erl[lane] = (uint8_t)rl;
        wave_sync();
        // the pass's products, 64 per round, kLanePG rounds at a time (their loads in flight
        // together): entry by markers, slot = t - the row's base
        constexpr uint32_t kSpan = kLaneSeg * kLanePG;
        for (uint32_t p0 = 0; p0 < stot; p0 += kSpan) {
            const uint32_t t0 = fcarry + p0;
            if (bl && off < t0 + kSpan && off + bl > t0) pmk[max(off, t0) - t0] = (uint16_t)(lane + 1);
            wave_sync();
            uint32_t L[kLanePG], carry = 0;
            sfor<kLanePG>([&](auto Q) {
                const uint32_t m = pmk[Q * kWave + lane];
                L[Q] = max(wave_incl_scan(m, 0u, mx), carry);
                carry = readlane_u32(L[Q], kWave - 1);
            });
            for (uint32_t w = lane; w < kSpan / 2; w += kWave) ((uint32_t *)pmk)[w] = 0;
            uint32_t c[kLanePG], row[kLanePG], slot[kLanePG];
            S v[kLanePG], a[kLanePG];
            sfor<kLanePG>([&](auto Q) {
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
            sfor<kLanePG>([&](auto Q) {
                if (c[Q] != kSent && slot[Q] < kLaneCap) {
                    skey[slot[Q] * kQR + row[Q]] = (c[Q] << 6) | slot[Q];
                    sval[slot[Q] * kQR + row[Q]] = Sem::prod(a[Q], v[Q]);
                }
            });
            wave_sync();
        }
        fcarry += stot;
        pc.mark(2);  // products into the slot table
    }

    // 3. each row's keys sorted by its quad (lane 4r + q: row r, elements q * NL ..); integer rows
    //    are counted and summed by the quad from there (quad_count / quad_combine), f64 rows are
    //    written back row-major and lane q = 0 of the quad reads its row's N sorted keys (the fold)
    constexpr bool kQuad = !std::is_same_v<S, double>;
    const uint32_t r = lane >> 2, q = lane & 3u;
    const uint32_t cnt = r < nt ? rcnt[r] : 0u;
    if (cnt > kLaneCap)  // the host runs the call through the pipeline instead
        __hip_atomic_store(&p.host_out[3], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t cn = cnt > kLaneCap ? 0u : cnt;
    const uint32_t wmax = wave_max_u32(cn);
    uint32_t nz = 0, zeros = 0, roff = 0;  // (q = 0 lanes) distinct columns, zero sums, offset in the wave
    uint32_t k[kLaneCap];
    uint32_t kq[kLaneCap / 4], qst = 0, qfirst = 0;  // (integer rows) the lane's sorted keys, starts, first output
    auto sort_and_count = [&](auto ntag) {
        constexpr int N = decltype(ntag)::value, NL = N / 4;
        uint32_t kk[kLaneCap / 4];
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const uint32_t e = q * NL + (uint32_t)j;
            kk[j] = e < cn ? skey[e * kQR + r] : kSent;
        }
        quad_sort<NL>(kk, q);
        if constexpr (kQuad) {
            uint32_t tot = 0;
            quad_count<NL>(kk, q, qst, qfirst, tot);
#pragma unroll
            for (int j = 0; j < (int)kLaneCap / 4; ++j) kq[j] = j < NL ? kk[j] : kSent;
            nz = q == 0 ? tot : 0u;
            return;
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < NL; ++j) skey[r * kLaneCap + q * NL + (uint32_t)j] = kk[j];
        wave_sync();
        if (q == 0) {
#pragma unroll
            for (int e = 0; e < N; ++e) k[e] = skey[r * kLaneCap + (uint32_t)e];
#pragma unroll
            for (int e = N; e < (int)kLaneCap; ++e) k[e] = kSent;
            // distinct columns (structural: zero sums are dropped afterwards)
#pragma unroll
            for (int e = 0; e < N; ++e) nz += (k[e] != kSent && (e == 0 || (k[e] >> 6) != (k[e - 1] >> 6))) ? 1u : 0u;
        }
    };
    if (wmax <= 16)
        sort_and_count(std::integral_constant<int, 16>{});
    else if (wmax <= 32)
        sort_and_count(std::integral_constant<int, 32>{});
    else
        sort_and_count(std::integral_constant<int, 64>{});
    const uint32_t wincl = wave_incl_scan(nz, 0u, plus);
    roff = wincl - nz;
    const uint32_t wsum = readlane_u32(wincl, kWave - 1);
    if (lane == 0) s_wsum[wv] = wsum;
    const uint32_t rmax = wave_max_u32(nz);
    if (lane == 0 && rmax) atomicMax(s_max, rmax);
    pc.mark(3);  // sort, count
    __syncthreads();
    pc.mark(4);  // block barrier
    // 4. the block's aggregate published first; u32 rows then stage their outputs in LDS at the
    //    block-local offset while the earlier blocks finish, and only the coalesced store waits for
    //    the offset (decoupled look-back over the earlier blocks' status words)
    uint32_t wbase = 0, agg = 0;
#pragma unroll
    for (uint32_t w = 0; w < kLaneWaves; ++w) {
        const uint32_t x = s_wsum[w];
        wbase += w < wv ? x : 0u;
        agg += x;
    }
    if (threadIdx.x == 0) {
        // the max row first, its result waited for: it is in place once a later block sees this
        // block's status, so the last block reads the final max after its look-back
        maxw_raise(maxw, epoch, *s_max);
        lookback_publish(status, blockIdx.x, epoch, agg);
    }
    const S *sv = sval + r;  // slot e of this lane's row at sv[e * kQR]
    // (integer rows) the quad's outputs by every lane of it, at the row's offset q = 0 holds
    const uint32_t roffq = kQuad ? quad_perm<kQFirst>(roff) : roff;
    auto quad_all = [&](auto &&emit) {
        if (wmax <= 16)
            return quad_combine<Sem, 4>(kq, qst, qfirst, sv, q, emit);
        else if (wmax <= 32)
            return quad_combine<Sem, 8>(kq, qst, qfirst, sv, q, emit);
        else
            return quad_combine<Sem, 16>(kq, qst, qfirst, sv, q, emit);
    };
    if constexpr (sizeof(S) == 4) {
        const uint32_t o0 = wbase + roffq;
        zeros = quad_all([&](uint32_t col, S val, uint32_t j) {
            stc[o0 + j] = col;
            stv[o0 + j] = val;
        });
    }
    pc.mark(5);  // publish, combine into staging
    __syncthreads();
    pc.mark(6);  // block barrier
    if (wv == 0) {
        const unsigned long long excl = lookback_walk(status, blockIdx.x, epoch, agg);
        const bool last = blockIdx.x == gridDim.x - 1;
        const unsigned long long mxr = last ? maxw_read(maxw, epoch) : 0u;
        if (lane == 0) {
            *s_off = excl;
            if (last) {
                const unsigned long long o0 =
                    __hip_atomic_exchange(&p.host_out[0], excl + agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                const unsigned long long o1 =
                    __hip_atomic_exchange(&p.host_out[1], mxr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                asm volatile("" ::"v"(o0), "v"(o1));
            }
        }
    }
    __syncthreads();
    pc.mark(7);  // look-back (wave 0), barrier
    const unsigned long long excl = *s_off;
    const uint64_t base = excl + wbase + roff;  // (q = 0 lanes) the row's first output
    if (q == 0 && r < nt) {
        p.c_rp[r0 + r + 1] = base + nz;
        if (r0 + r == 0) p.c_rp[0] = 0;
    }
    if constexpr (sizeof(S) == 4) {
        // the block's rows are contiguous in C: the staged outputs stored coalesced
        uint32_t *oc = p.c_col + excl;
        S *ov = (S *)p.c_val + excl;
        for (uint32_t u = threadIdx.x; u < agg; u += kLaneWaves * kWave) {
            oc[u] = stc[u];
            ov[u] = stv[u];
        }
    } else if constexpr (kQuad) {
        const uint64_t bq = excl + wbase + roffq;
        uint32_t *oc = p.c_col + bq;
        S *ov = (S *)p.c_val + bq;
        zeros = quad_all([&](uint32_t col, S val, uint32_t j) {
            oc[j] = col;
            ov[j] = val;
        });
    } else if (q == 0 && nz) {
        uint32_t *oc = p.c_col + base;
        S *ov = (S *)p.c_val + base;
        auto emit = [&](uint32_t col, S val, uint32_t j) {
            oc[j] = col;
            ov[j] = val;
        };
        if (wmax <= 16)
            zeros = lane_combine<Sem, 16>(k, sv, emit);
        else if (wmax <= 32)
            zeros = lane_combine<Sem, 32>(k, sv, emit);
        else
            zeros = lane_combine<Sem, 64>(k, sv, emit);
    }
    // zero sums (explicit zero inputs, f64 cancellation) stay in C for now: the row's non-zero count
    // goes to p.counts and the rows with zeros to host_out[2], and the host compacts (as after
    // k_numeric)
    if constexpr (kQuad) {  // the row's zero sums from its quad's lanes, kept in lane q = 0
        zeros += quad_perm<0xB1>(zeros);  // [1,0,3,2]
        zeros += quad_perm<0x4E>(zeros);  // [2,3,0,1]
        if (q != 0) zeros = 0;
    }
    if (q == 0 && r < nt) p.counts[r0 + r] = nz - zeros;
    add_zero_rows(&p.host_out[2], wave_sum_u32(zeros ? 1u : 0u), true);
    pc.mark(8);  // stores
    if constexpr (SLAT_PHASES) {
        if (lane == 0) {
            unsigned long long *dst = p.shards + 512 + ((blockIdx.x * kLaneWaves + wv) % 64) * kPhaseSlots;
            for (int i = 0; i < kPhaseSlots; ++i) atomicAdd(&dst[i], (unsigned long long)pc.ph[i]);
        }
    }
    signal_done(p);
}

template <typename Sem>
hipError_t launch(dim3 grid, hipStream_t s, const Args &a, unsigned long long *status, uint32_t epoch,
                  unsigned long long *maxw) {
    constexpr size_t lds = lane_lds<typename Sem::S>();
    static bool attr = false;  // over 64 KB of dynamic LDS (u32: ~70 KB, two blocks per CU)
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)k_lane<Sem>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    hipLaunchKernelGGL(k_lane<Sem>, grid, dim3(kLaneWaves * kWave), lds, s, a, status, epoch, maxw);
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
