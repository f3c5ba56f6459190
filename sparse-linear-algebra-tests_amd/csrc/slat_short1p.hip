// slat_short1p.hip — wide products whose rows are all short (config C4: the 100^3 torus' A^3 * A, 1 M
// columns, ~91 products and ~57 outputs a row) in ONE kernel ("next round" item 1).
//
// The pipeline gives such a call three passes over the products: k_symbolic_short counts each row's
// distinct columns in an LDS hash table, k_scan_rows turns the counts into row offsets, and
// k_numeric_short inserts every product into a hash table again, with its value, then sorts the
// table's keys and writes the row. The second hash pass is the numeric pass's own work; the first is
// there only to learn the offsets (0.40 of C4's 1.22 ms), and the scan and the empty listed-row
// launches of a wide call are fixed costs that do not shrink with a row block (the multi-GPU split).
//
// Here a wave owns a tile of kT1 consecutive rows and learns the offsets as it goes:
//
//   1. the tile's exact products per row (the A entries' B row lengths, from the ELL image's length
//      byte), then batches of consecutive rows of at most kHashT / 2 products, so a batch's distinct
//      columns always fit one 256-key sort;
//   2. per batch, numeric's accumulation into the per-wave LDS hash table (composite (row, column)
//      keys, u32 slots with wrap bits), then the table's keys packed with their slot (key << 9 | slot)
//      and sorted across the wave (128 or 256 keys by the batch's count), values read and the table
//      cleared; the sorted outputs stay in registers (at most one batch per row of the tile);
//   3. the tile's aggregate (its distinct outputs) published, a decoupled look-back over the earlier
//      tiles' status words for its offset, then row_ptr and the outputs stored.
//
// Tiles are taken in dispatch order (a wave's tile is blockIdx * waves + its index), so every earlier
// tile belongs to a wave that is running or done. The aggregate is published once the tile's batches
// are accumulated and sorted, so a tile waits only for earlier tiles to get that far, never for their
// stores. A row the tables cannot take (more than 256 A entries, more than kHashT products, or more
// than 256 distinct columns) sets the mapped overflow word and the host runs the call through the
// pipeline instead (slat_api.hip remembers the operands).
#include <hip/hip_runtime.h>

#include "slat_launch.hpp"
#include "spgemm_kernels.hpp"

using namespace slat;

namespace {

constexpr uint32_t kT1 = 4;              // rows per tile (a wave)
constexpr uint32_t kS1W = 4;             // waves per block: the block is the look-back's tile
constexpr uint32_t kCapP1 = kHashT / 2;  // exact products per batch
constexpr uint32_t kEmpty1 = 0xFFFFFFFFu;

// LDS of one wave: the k_numeric_short<SemU32> layout (hash table | scratch | zero counts | staged
// rows) plus the tile rows' output ends u32[kT1]
__host__ __device__ constexpr uint32_t s1p_wave_bytes() { return (short_bytes<SemU32>() + kT1 * 4 + 15) & ~15u; }

// exact length of B row k (the ELL image's length byte: groups | padding << 4)
__device__ __forceinline__ uint32_t ell_len(const Args &p, uint32_t k) {
    const uint32_t g = p.ell_ng[k];
    return 4u * (g & 15u) - (g >> 4);
}

// Ascending bitonic sort of 64 * NPL distinct u32 keys, element i = lane * NPL + e in k[e] (kSent
// last). A compare-exchange is a min and a max: distinct keys need no payload or tie rule.
template <int NPL, int K, int J>
__device__ __forceinline__ void pk_step(uint32_t (&k)[4], uint32_t lane) {
    if constexpr (J >= NPL) {
        constexpr int M = J / NPL;  // the partner lane is lane ^ M
        const bool asc = ((lane * NPL) & (uint32_t)K) == 0;
        const bool tmin = ((lane & (uint32_t)M) == 0) == asc;
        sfor<NPL>([&](auto E) {
            const uint32_t o = lane_xor<M>(k[E]);
            k[E] = tmin ? min(k[E], o) : max(k[E], o);
        });
    } else {
        sfor<NPL>([&](auto E) {
            constexpr int e = decltype(E)::value;
            if constexpr ((e & J) == 0) {
                constexpr int f = e | J;
                const bool asc = (((lane * NPL) | (uint32_t)e) & (uint32_t)K) == 0;
                const uint32_t lo = min(k[e], k[f]), hi = max(k[e], k[f]);
                k[e] = asc ? lo : hi;
                k[f] = asc ? hi : lo;
            }
        });
    }
}
template <int NPL, int K, int J>
__device__ __forceinline__ void pk_merge(uint32_t (&k)[4], uint32_t lane) {
    pk_step<NPL, K, J>(k, lane);
    if constexpr (J > 1) pk_merge<NPL, K, J / 2>(k, lane);
}
template <int NPL, int K = 2>
__device__ __forceinline__ void pk_sort(uint32_t (&k)[4], uint32_t lane) {
    pk_merge<NPL, K, K / 2>(k, lane);
    if constexpr (K < 64 * NPL) pk_sort<NPL, K * 2>(k, lane);
}

// The batch in the hash table -> its outputs sorted, in registers: ck[e] = composite key (local row
// << cb | column) of element lane * npl + e (kSent past nk), cv[e] its saturated sum. The table and
// its wrap bits are left clean. Returns nk, the batch's distinct keys (> kHashT / 2: not sorted).
__device__ __forceinline__ uint32_t batch_regs(uint32_t *hkeys, uint32_t *hvals, uint32_t *hstage, uint32_t *hslot,
                                               uint32_t (&ck)[4], uint32_t (&cv)[4], uint32_t &npl) {
    using Sem = SemU32W;
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t hk[kHashHeld], nh = 0;
    sfor<kHashHeld>([&](auto I_) {
        hk[I_] = hkeys[I_ * kWave + lane];
        nh += hk[I_] != kSent ? 1u : 0u;
    });
    const uint32_t incl = wave_incl_scan(nh, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    const uint32_t nk = readlane_u32(incl, kWave - 1);
    uint32_t at = incl - nh;
    sfor<kHashHeld>([&](auto I_) {
        if (hk[I_] != kSent) {
            if (at < kHashT / 2) {
                hstage[at] = hk[I_];
                hslot[at] = I_ * kWave + lane;
            }
            ++at;
            hkeys[I_ * kWave + lane] = kSent;
        }
    });
    wave_sync();
    uint32_t k[4] = {kSent, kSent, kSent, kSent};
    if (nk <= kHashT / 4) {
        npl = 2;
        sfor<2>([&](auto E) {
            const uint32_t i = lane * 2 + E;
            if (i < nk) k[E] = (hstage[i] << 9) | hslot[i];
        });
        pk_sort<2>(k, lane);
    } else {
        npl = 4;
        const uint4 k4 = ((const uint4 *)hstage)[lane], s4 = ((const uint4 *)hslot)[lane];
        const uint32_t kk[4] = {k4.x, k4.y, k4.z, k4.w}, ss[4] = {s4.x, s4.y, s4.z, s4.w};
        sfor<4>([&](auto E) {
            if (lane * 4 + E < min(nk, kHashT / 2)) k[E] = (kk[E] << 9) | ss[E];
        });
        pk_sort<4>(k, lane);
    }
    sfor<4>([&](auto E) {
        ck[E] = kSent;
        cv[E] = 0;
        if (k[E] != kSent) {
            const uint32_t sl = k[E] & (kHashT - 1);
            ck[E] = k[E] >> 9;
            cv[E] = Sem::finish(hvals, sl);
            hvals[sl] = 0;
        }
    });
    if (nk > kHashT / 2)  // (overflowed: the keys past the sort still hold their values)
        for (uint32_t w = lane; w < kHashT; w += kWave) hvals[w] = 0;
    if (lane < ExtraWords<Sem>::value) hvals[kHashT + lane] = 0;
    wave_sync();
    return nk;
}

// The look-back walk of a block (one wave): lookback_walk's rounds of kWave * R predecessors, but a
// wait re-reads only the statuses still unpublished, with a growing sleep. With ~1 300 blocks in
// flight many walks wait at once, and re-reading every status of the round on each poll (device-scope
// loads past the XCD's L2) flooded the fabric: C4's eighth took 0.65 ms, 56 us of each block's time
// in its walk.
template <int R>
__device__ __forceinline__ unsigned long long walk1p(unsigned long long *status, uint64_t tile, uint32_t epoch,
                                                     unsigned long long agg) {
    auto ld = [](unsigned long long *x) { return __hip_atomic_load(x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    const uint32_t lane = (uint32_t)lane_id();
    const unsigned long long tag = (unsigned long long)epoch << 42;
    if (tile == 0) return 0;
    unsigned long long excl = 0;
    for (int64_t j0 = (int64_t)tile - 1;; j0 -= kWave * R) {
        unsigned long long x[R];
        uint32_t valid = 0;
        sfor<R>([&](auto I) {
            const int64_t j = j0 - (int64_t)(lane * R + I);
            x[I] = j >= 0 ? ld(&status[j]) : 0ull;
        });
        int first = R, last = kWave;
        unsigned long long inc = 0;
        for (uint32_t nap = 1;; nap = min(nap * 2, 16u)) {
            // valid: published this epoch (or before status 0); the lane's nearest inclusive prefix,
            // the wave's nearest by ballot; only the statuses up to it are needed
            valid = 0;
            first = R;
            sfor<R>([&](auto I) {
                const int64_t j = j0 - (int64_t)(lane * R + I);
                const bool v = j < 0 || ((x[I] >> 42) == epoch && (x[I] & (kStAgg | kStInc)) != 0);
                valid |= (v ? 1u : 0u) << I;
                if (first == R && j >= 0 && v && (x[I] & kStInc)) first = I;
            });
            inc = __ballot(first < R);
            last = inc ? (int)__builtin_ctzll(inc) : kWave;
            const uint32_t need = (int)lane < last ? (1u << R) - 1 : (int)lane == last ? (1u << first) - 1 : 0u;
            if (__ballot((valid & need) != need) == 0) break;
            __builtin_amdgcn_s_sleep(2);
            if (nap > 1) __builtin_amdgcn_s_sleep(8);
            if (nap > 4) __builtin_amdgcn_s_sleep(16);
            sfor<R>([&](auto I) {
                const int64_t j = j0 - (int64_t)(lane * R + I);
                if (((need & ~valid) >> I) & 1u) x[I] = ld(&status[j]);
            });
        }
        unsigned long long v = 0;
        sfor<R>([&](auto I) {
            const int64_t j = j0 - (int64_t)(lane * R + I);
            if (j >= 0 && ((int)lane < last || ((int)lane == last && (int)I <= first))) v += x[I] & kStVal;
        });
        v = wave_incl_scan_u64(v);
        excl += readlane_u64(v, kWave - 1);
        if (inc || j0 - (int64_t)(kWave * R) < 0) break;
    }
    if (lane == 0) __hip_atomic_store(&status[tile], tag | kStInc | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

__global__ __launch_bounds__(kWave * kS1W) __attribute__((amdgpu_waves_per_eu(5))) void k_short1p(
    Args p, unsigned long long *status, uint32_t epoch, unsigned long long *maxw) {
    using Sem = SemU32W;
    using S = uint32_t;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t tile = (uint64_t)blockIdx.x * kS1W + wv;  // the wave's rows
    const uint64_t ntiles = (p.nrows + kT1 - 1) / kT1;
    const bool spare = tile >= ntiles;  // (the last block's waves past the rows: they join the barriers)
    __shared__ uint32_t s_agg[kS1W], s_max;
    __shared__ unsigned long long s_off;
    if (threadIdx.x == 0) s_max = 0;
    constexpr uint32_t kMx = short_mx<SemU32>();
    uint8_t *region = smem8 + (size_t)wv * s1p_wave_bytes();
    uint32_t *hkeys = (uint32_t *)region;
    uint32_t *hvals = (uint32_t *)(region + kHashT * 4);
    uint32_t *hstage = (uint32_t *)(region + kHashT * 8 + ExtraWords<Sem>::value * 4);
    uint32_t *marks = (uint32_t *)(region + hash_bytes<Sem>());
    uint32_t *hslot = marks;  // the emit's slots
    S *ga = (S *)marks;       // the accumulation's A values
    uint32_t *zc = marks + kMx / 4;
    uint32_t *gk = hstage;
    uint8_t *gl = (uint8_t *)(zc + kWave);
    uint32_t *rend = (uint32_t *)(gl + kStageG);
    for (uint32_t w = lane; w < kHashT; w += kWave) hkeys[w] = kSent;
    for (uint32_t w = lane; w < kHashT + ExtraWords<Sem>::value; w += kWave) hvals[w] = 0;
    for (uint32_t w = lane; w < kMx / 16; w += kWave) ((uint4 *)marks)[w] = make_uint4(0, 0, 0, 0);
    zc[lane] = 0;
    if (lane < kT1) rend[lane] = kEmpty1;
    // pattern B (every B value equal): no B-value loads; the B-value maximum for narrow batches
    uint32_t bvmax = 0;
    bool buni = false;
    if (p.b_vmax) {
        const unsigned long long v = ((volatile unsigned long long *)p.b_vmax)[kVMaxWord];
        const unsigned long long vi = ((volatile unsigned long long *)p.b_vmax)[kVMinInvWord];
        if ((uint32_t)(v >> 32) == p.epoch) {
            bvmax = (uint32_t)v;
            buni = SLAT_NUM_UNI && (uint32_t)(vi >> 32) == p.epoch && ~(uint32_t)vi == bvmax && bvmax != 0xFFFFFFFFu;
        }
    }
    const S bv0 = (S)bvmax;
    const S *av_ = (const S *)p.a_val;
    const uint32_t cb = p.cbits;
    PhaseClock pc{};  // diagnostic builds (-DSLAT_PHASES=1): s_memtime cycles per phase
    if constexpr (SLAT_PHASES) {
        pc.t = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int i = 0; i < kPhaseSlots; ++i) pc.ph[i] = 0;
        pc.ph[kPhaseSlots - 1] = 1;
    }

    // the tile's rows: lanes < nt hold their bounds
    const uint64_t r0 = tile * kT1;
    const uint32_t nt = spare ? 0u : (uint32_t)min<uint64_t>(kT1, p.nrows - r0);
    uint64_t A0j = 0, A1j = 0;
    if (lane < nt) {
        A0j = p.a_rp[r0 + lane];
        A1j = p.a_rp[r0 + lane + 1];
    }
    const uint64_t lj = A1j - A0j;
    // 1. exact products per row, the tile's entries 64 at a time (each entry finds its row among the
    //    tile's <= kT1 bounds)
    uint64_t rb[kT1 + 1];
    const int last = nt ? (int)nt - 1 : 0;
    sfor<kT1>([&](auto J) { rb[J] = J < nt ? readlane_u64(A0j, J) : readlane_u64(A1j, last); });
    rb[kT1] = readlane_u64(A1j, last);
    uint32_t pj = 0;
    for (uint64_t c0 = rb[0]; c0 < rb[kT1]; c0 += kWave) {
        const uint64_t idx = c0 + lane;
        uint32_t len = 0;
        if (idx < rb[kT1]) {
            const uint32_t k = p.a_col[idx];
            len = k < p.b_nrows ? ell_len(p, k) : 0u;
        }
        sfor<kT1>([&](auto J) {
            const uint32_t s = wave_sum_u32(idx >= rb[J] && idx < rb[J + 1] ? len : 0u);
            if (lane == (uint32_t)J) pj += s;
        });
    }
    bool ov = __ballot(lane < nt && (lj > 256 || pj > kHashT)) != 0;
    pc.mark(0);  // row bounds, exact products

    // 2. batches of consecutive rows, each a hash accumulation and a sort; outputs held in registers
    uint32_t ck[kT1][4], cv[kT1][4], nkb[kT1], nplb[kT1], bbase[kT1];
    uint32_t agg = 0, b = 0;
    sfor<kT1>([&](auto Bi) {
        nkb[Bi] = 0;
        nplb[Bi] = 4;
        bbase[Bi] = agg;
        sfor<4>([&](auto E) {
            ck[Bi][E] = kSent;
            cv[Bi][E] = 0;
        });
        if (b >= nt || ov) return;
        const bool inb = lane >= b && lane < nt;
        const uint32_t pu = wave_incl_scan(inb ? pj : 0u, 0u, [](uint32_t x, uint32_t y) { return x + y; });
        const uint32_t pl = wave_incl_scan(inb ? (uint32_t)lj : 0u, 0u, [](uint32_t x, uint32_t y) { return x + y; });
        const unsigned long long stop = __ballot(inb && lane > b && (pu > kCapP1 || pl > 256));
        const uint32_t e = stop ? (uint32_t)__builtin_ctzll(stop) : nt;
        const uint64_t A0 = readlane_u64(A0j, (int)b), A1 = readlane_u64(A1j, (int)(e - 1));
        const uint32_t nent = (uint32_t)(A1 - A0);
        // entry -> local row: each row's first entry marked (a later non-empty row wins a tie with
        // empty rows before it), then a running max
        if (inb && lane < e && lj > 0) atomicMax(&marks[(uint32_t)(A0j - A0)], lane - b + 1);
        wave_sync();
        uint32_t kq[kRegQ], lq[kRegQ], ng[kRegQ];
        S aq[kRegQ];
        uint32_t carry = 0, mxg = 0;
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
                aq[Q] = av_[A0 + i];
                marks[i] = 0;
            }
        });
        sfor<kRegQ>([&](auto Q) {
            ng[Q] = short_brow<false>(p, kq[Q]);
            mxg = max(mxg, ng[Q]);
        });
        mxg = wave_max_u32(mxg);
        uint32_t pos[kRegQ];
        const uint32_t G = group_positions(ng, pos);
        bool narrow = false;  // no sum of this batch can wrap (each key takes <= G products)
        if (bvmax) {
            uint32_t am = 0;
            sfor<kRegQ>([&](auto Q) { am = max(am, (uint32_t)aq[Q]); });
            const unsigned long long ab = (unsigned long long)wave_max_u32(am) * bvmax;
            narrow = ab < (1ull << 32) && ab * G < (1ull << 32);
        }
        for (uint32_t base = 0; base < G; base += kStageG) {
            stage_groups<true, false, S>(base, mxg, kq, lq, ng, pos, aq, gk, gl, ga);
            const uint32_t n = min(G - base, kStageG);
            for (uint32_t g0 = 0; g0 < n; g0 += kWave) {
                const uint32_t g = g0 + lane;
                uint4 cc = make_uint4(kSent, kSent, kSent, kSent);
                Quad<S> pr{};
                if (g < n) {
                    const uint32_t w = gk[g], glb = gl[g];
                    const uint4 c = staged_cols<false>(p, w, glb);
                    const S a = ga[g];
                    pr = buni ? splat4(Sem::prod(a, bv0)) : prods<Sem>(a, staged_vals<false, S>(p, w, glb));
                    const uint32_t hi = (glb & 63u) << cb;
                    cc.x = c.x != kSent ? (hi | c.x) : kSent;
                    cc.y = c.y != kSent ? (hi | c.y) : kSent;
                    cc.z = c.z != kSent ? (hi | c.z) : kSent;
                    cc.w = c.w != kSent ? (hi | c.w) : kSent;
                }
                if (narrow)
                    HashAcc<SemU32WN>{hkeys, hvals}(cc, pr);
                else
                    HashAcc<Sem>{hkeys, hvals}(cc, pr);
            }
            wave_sync();
        }
        wave_sync();
        pc.mark(1);  // accumulation
        uint32_t npl = 4;
        const uint32_t nk = batch_regs(hkeys, hvals, hstage, hslot, ck[Bi], cv[Bi], npl);
        if (nk > kHashT / 2) ov = true;
        // each row's end in the tile's outputs: the last element of its run (sorted by local row)
        uint32_t nxt0 = __shfl_down(ck[Bi][0], 1);
        if (lane == kWave - 1) nxt0 = kSent;
        sfor<4>([&](auto E) {
            const uint32_t c = ck[Bi][E];
            if (E < npl && c != kSent) {
                const uint32_t nx = E + 1 < npl ? ck[Bi][(E + 1) & 3] : nxt0;
                const uint32_t lr = c >> cb;
                if (nx == kSent || (nx >> cb) != lr) rend[b + lr] = agg + lane * npl + E + 1;
                if (cv[Bi][E] == 0) atomicAdd(&zc[b + lr], 1u);
            }
        });
        nkb[Bi] = nk;
        nplb[Bi] = npl;
        agg += nk;
        b = e;
        for (uint32_t w = lane; w < kMx / 16; w += kWave) ((uint4 *)marks)[w] = make_uint4(0, 0, 0, 0);
        wave_sync();
        pc.mark(2);  // sort, row ends
    });
    if (ov) {
        // a row the tables cannot take: the host reruns the call through the pipeline. The block still
        // publishes (this wave adding 0) so no later block's walk waits on it
        agg = 0;
        if (lane == 0) __hip_atomic_store(&p.host_out[3], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // row ends: a row without outputs ends where the row before it does
    uint32_t re = lane < nt ? rend[lane] : 0u;
    if (re == kEmpty1) re = 0;
    re = wave_incl_scan(re, 0u, [](uint32_t x, uint32_t y) { return max(x, y); });
    uint32_t prev = __shfl_up(re, 1);
    if (lane == 0) prev = 0;
    const uint32_t cnt = lane < nt ? re - prev : 0u;
    const uint32_t mx = wave_max_u32(cnt);
    // 3. the block's aggregate and max row from its waves, then one look-back per block (the max row
    //    raised only past this epoch's current word, before the block's status is published)
    if (lane == 0) {
        s_agg[wv] = agg;
        if (mx) atomicMax(&s_max, mx);
    }
    __syncthreads();
    uint32_t bagg = 0, wpre = 0;
    sfor<kS1W>([&](auto W) {
        const uint32_t x = s_agg[W];
        wpre += W < wv ? x : 0u;
        bagg += x;
    });
    pc.mark(3);  // block aggregate
    if (wv == 0) {
        const uint32_t bmx = s_max;
        if (lane == 0 && bmx) {
            unsigned long long *w = &maxw[(size_t)kDoneStride * (blockIdx.x % kDoneGroups)];
            const unsigned long long cur = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)(cur >> 32) != epoch || (uint32_t)cur < bmx) {
                const unsigned long long old = atomicMax(w, ((unsigned long long)epoch << 32) | bmx);
                asm volatile("" ::"v"(old));  // in place before this block's status is
            }
        }
        lookback_publish(status, blockIdx.x, epoch, bagg);
#if SLAT_1P_NOWALK  // timing experiment only (offsets wrong): the kernel without the look-back's wait
        const unsigned long long ex = 0;
#else
        const unsigned long long ex = walk1p<4>(status, blockIdx.x, epoch, bagg);
#endif
        if (lane == 0) s_off = ex;
        if (blockIdx.x == gridDim.x - 1) {
            const unsigned long long mxr = maxw_read(maxw, epoch);
            if (lane == 0) {
                const unsigned long long o0 =
                    __hip_atomic_exchange(&p.host_out[0], ex + bagg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                const unsigned long long o1 =
                    __hip_atomic_exchange(&p.host_out[1], mxr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                asm volatile("" ::"v"(o0), "v"(o1));
            }
        }
    }
    __syncthreads();
    const unsigned long long excl = s_off + wpre;
    pc.mark(4);  // look-back
    if (ov || spare) return;
    if (lane < nt) {
        p.c_rp[r0 + lane + 1] = excl + re;
        p.counts[r0 + lane] = cnt - zc[lane];
    }
    if (tile == 0 && lane == 0) p.c_rp[0] = 0;
    const uint32_t cmask = (1u << cb) - 1;
    sfor<kT1>([&](auto Bi) {
        if (nkb[Bi] == 0) return;
        const uint64_t o = excl + bbase[Bi];
        sfor<4>([&](auto E) {
            const uint32_t i = lane * nplb[Bi] + E;
            if (E < nplb[Bi] && i < nkb[Bi]) {
                p.c_col[o + i] = ck[Bi][E] & cmask;
                ((S *)p.c_val)[o + i] = cv[Bi][E];
            }
        });
    });
    const uint32_t zr = wave_sum_u32(lane < nt && zc[lane] ? 1u : 0u);
    add_zero_rows(&p.host_out[2], zr, false);
    pc.mark(5);  // stores
    if constexpr (SLAT_PHASES) {
        if (lane == 0) {
            unsigned long long *dst = p.shards + 512 + (tile % 64) * kPhaseSlots;
            for (int i = 0; i < kPhaseSlots; ++i) atomicAdd(&dst[i], (unsigned long long)pc.ph[i]);
        }
    }
}

}  // namespace

uint32_t slat_short1p_rows() { return kT1 * kS1W; }
size_t slat_short1p_lds() { return (size_t)s1p_wave_bytes() * kS1W; }

hipError_t slat_launch_short1p(dim3 grid, hipStream_t s, const Args &a, unsigned long long *status, uint32_t epoch,
                               unsigned long long *maxw) {
    hipLaunchKernelGGL(k_short1p, grid, dim3(kWave * kS1W), slat_short1p_lds(), s, a, status, epoch, maxw);
    return hipGetLastError();
}
