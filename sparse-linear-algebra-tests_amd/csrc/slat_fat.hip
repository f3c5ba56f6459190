// slat_fat.hip — the fat-row category of the SpGEMM (MAGNUS's dense accumulation for rows whose
// products outgrow a wavefront's LDS slots), SURVEY.md §8(a) row a7.
//
// A row of C = A·B with many products (power-law hubs, dense powers of a graph: thousands of
// outputs per row) would take the wavefront kernels many rank chunks or column windows, each a full
// re-walk of the row. Here such rows get a workgroup of 512 threads and the whole 160 KB LDS:
//
//   k_fr_select   one thread per row: products = sum over the row's entries k of nnz(B row k),
//                 cut off at slat_fat_min(); rows at or above it are marked (the other kernels skip them)
//                 and listed.
//   k_fr_symbolic one block per listed row: a column bitmap over 2^20 columns per pass (128 KB),
//                 one bit per product, popcount -> the row's structural count; also the mask of
//                 touched accumulator chunks, so the numeric pass visits only those.
//   k_fr_numeric  one block per listed row, per touched chunk of kChunk columns: a dense LDS
//                 accumulator indexed by column (no hash, no ranks), a bitmap of touched columns,
//                 then the emit: a block scan of the words' popcounts gives every column its
//                 position, so the row comes out sorted (the reference sorts nz_cols,
//                 src/graph_csr.rs:331,449). Integer semirings and f64 in any order add with LDS
//                 atomics, lanes spread over the row's A entries (a long B row is walked by the
//                 whole wave). f64 in the reference's order (the left fold of linalg/src/csr.rs:
//                 325-337) gives each wave its own slice of the chunk's columns and walks the A
//                 entries in order, lanes over one B row: one writer per column, in A order.
//
// B is read in its CSR form; the B-row part inside a column range is found by a 64-ary search.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstring>

#include "slat.h"
#include "slat_internal.hpp"
#include "spgemm_kernels.hpp"
#include "slat_fat.hpp"

namespace slat {

constexpr int kFB = 512;                 // threads per fat-row block
constexpr int kFW = kFB / kWave;         // waves per block

constexpr uint32_t kSymBits = 1u << 20;  // symbolic bitmap columns per pass (128 KB)

// columns per accumulator chunk: fr_kb<Sem>() KB of V slots + the chunk's bitmap. 64 KB (two blocks
// per CU, twice the chunks per row) for the semirings that add with atomics: R-MAT 2^16 A^2
// 11.7 -> 10.6 ms, C5 2^18 any order 92.5 -> 81.5 ms; 128 KB (one block per CU) for f64 in the
// reference's fold order, whose wave slices halve with the chunk (C5 2^18 fold 110 -> 256 ms at 64 KB),
// profiles/r03_ab_fr64.txt. SLAT_FR_KB overrides the 64.
#ifndef SLAT_FR_KB
#define SLAT_FR_KB 64
#endif
template <typename Sem>
__host__ __device__ constexpr uint32_t fr_kb() {
    return Sem::kOrdered ? 128u : (uint32_t)SLAT_FR_KB;
}
template <typename Sem>
__host__ __device__ constexpr uint32_t fr_chunk() {
    return (fr_kb<Sem>() * 1024u) / (uint32_t)(sizeof(typename Sem::V) * Sem::kSlots);
}
constexpr uint32_t kMaxBuckets = 256;  // accumulator chunks a bucketed row may span (LDS counters)
// LDS per wave of the flattened walk (fr_flat below): entry bases I[64] | A values S[64] (VALS) |
// markers u8[256]
template <typename S, bool VALS, typename I>
__host__ __device__ constexpr uint32_t fr_flat_bytes() {
    return kWave * (uint32_t)(sizeof(I) + (VALS ? sizeof(S) : 0)) + 4 * kWave;
}
template <typename Sem>
__host__ __device__ constexpr size_t fr_lds() {
    return (size_t)fr_chunk<Sem>() * sizeof(typename Sem::V) * Sem::kSlots + fr_chunk<Sem>() / 8 + 64 * 8 +
           (Sem::kOrdered ? 0 : 2 * kMaxBuckets * 4) + kFW * fr_flat_bytes<typename Sem::S, true, uint64_t>();
}

__device__ __forceinline__ uint32_t cap63(uint64_t x) { return x < 63 ? (uint32_t)x : 63u; }

#ifndef SLAT_FAT_TICKET
#define SLAT_FAT_TICKET 1
#endif
// The list's rows by block tickets instead of a fixed stride (power-law rows differ 40x in cost, so a
// stride leaves blocks idle behind the ones that drew several hubs): block b starts on row b without a
// ticket, each later row is a ticket (TicketQueue's protocol at block level: every block that had a
// row takes exactly one ticket past the end, and the last taker zeroes the counter for the next
// launch). Callers end each row with a block barrier.
struct BlockTickets {
    unsigned long long *ctr;
    uint64_t total;
    __device__ __forceinline__ BlockTickets(unsigned long long *c, uint64_t n)
        : ctr(SLAT_FAT_TICKET ? c : nullptr),
          total((n > gridDim.x ? n - gridDim.x : 0) + (n < gridDim.x ? n : (uint64_t)gridDim.x)) {}
    __device__ __forceinline__ uint64_t next(uint64_t li, unsigned long long *sh) const {
        if (!ctr) return li + gridDim.x;
        if (threadIdx.x == 0) {
            const unsigned long long t = atomicAdd(ctr, 1ull);
            if (t == total - 1) __hip_atomic_store(ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *sh = t;
        }
        __syncthreads();
        const uint64_t v = gridDim.x + *sh;
        __syncthreads();
        return v;
    }
};


// products of each row, cut off at f.fat_min; fat rows marked and listed
__global__ __launch_bounds__(kBlock) void k_fr_select(FatArgs f) {
    const Args &p = f.a;
    for (uint64_t r = (uint64_t)blockIdx.x * kBlock + threadIdx.x; r - threadIdx.x < p.nrows;
         r += (uint64_t)gridDim.x * kBlock) {
        bool fat = false;
        if (r < p.nrows) {
            uint64_t fl = 0;
            for (uint64_t i = p.a_rp[r], e = p.a_rp[r + 1]; i < e && fl < f.fat_min; ++i) {
                const uint32_t k = p.a_col[i];
                if (k < p.b_nrows) fl += p.b_rp[k + 1] - p.b_rp[k];
            }
            fat = fl >= f.fat_min;
            f.mark[r] = fat ? 1 : 0;
        }
        const unsigned long long m = __ballot(fat);
        if (m) {
            unsigned int base = 0;
            if (lane_id() == 0) base = atomicAdd(f.cnt, (unsigned int)__popcll(m));
            base = __builtin_amdgcn_readfirstlane(base);
            if (fat) f.list[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = (uint32_t)r;
        }
    }
}

// [s, e) = the entries of B row [bs, be) with columns in [lo, hi), by the whole wave: a 64-ary
// search (64 pivots per round, one per lane) while the range is longer than a wave
template <typename I>
__device__ __forceinline__ void b_range(const uint32_t *bcol, I bs, I be, uint32_t lo, uint32_t hi, I &s, I &e) {
    const int lane = lane_id();
    auto lower = [&](uint32_t key) -> I {  // first index in [bs, be) with col >= key
        I a = bs, b = be;
        while (b - a > (I)kWave) {
            const I step = (b - a + (I)kWave - 1) / (I)kWave;
            const I at = a + (I)lane * step;
            const bool below = at < b && bcol[at] < key;
            const uint32_t nb = __popcll(__ballot(below));  // pivots below key: a prefix of lanes
            const I na = nb ? a + (I)(nb - 1) * step + 1 : a;
            const I nbd = min(b, a + (I)nb * step + 1);
            a = na;
            b = nbd;
        }
        const I at = a + (I)lane;
        const bool below = at < b && bcol[at] < key;
        return a + (I)__popcll(__ballot(below));
    };
    s = lo == 0 ? bs : lower(lo);
    e = lower(hi);
}

// every product of A row [a0, a1) with column j in [lo, hi), by one block: fn(j, a, b) with the A and
// B values (VALS; else zeros). Lanes take kQ A entries at a time (their B-row bounds loaded together);
// a B row of at most kLongB entries is walked by its lane, two entries per step for all kQ rows at
// once (2 kQ independent loads in flight), a longer one by the whole wave over its part in [lo, hi).
constexpr int kQ = 4;
template <typename S, bool VALS, typename I, typename F>
__device__ __forceinline__ void fr_walk(const Args &p, I a0, I a1, uint32_t lo, uint32_t hi, bool all_cols, F &&fn,
                                        const uint32_t *split = nullptr, uint32_t nch1 = 0, uint32_t g0 = 0,
                                        uint32_t g1 = 0, uint32_t split_abs = 0) {
    const int lane = lane_id();
    const int wv = threadIdx.x / kWave;
    const S *av = (const S *)p.a_val;
    const S *bv = (const S *)p.b_val;
    for (I base = a0 + (I)wv * kWave; base < a1; base += (I)kFB * kQ) {
        uint32_t k[kQ];
        S a[kQ];
        I bs[kQ], be[kQ];
        sfor<kQ>([&](auto Q) {
            const I i = base + (I)(Q * kFB) + (I)lane;
            k[Q] = kSent;
            a[Q] = S(0);
            if (i < a1) {
                k[Q] = p.a_col[i];
                if constexpr (VALS) a[Q] = av[i];
            }
        });
        sfor<kQ>([&](auto Q) {
            bs[Q] = be[Q] = 0;
            if (k[Q] < p.b_nrows) {
                if (split) {  // only the chunk's part of the B row: no filtering, no search
                    const I r = split_abs ? (I)0 : (I)p.b_rp[k[Q]];
                    const uint32_t *sp = split + (uint64_t)k[Q] * nch1;
                    bs[Q] = r + (I)sp[g0];
                    be[Q] = r + (I)sp[g1];
                } else {
                    bs[Q] = (I)p.b_rp[k[Q]];
                    be[Q] = (I)p.b_rp[k[Q] + 1];
                }
            }
        });
        if (split) all_cols = true;
        uint32_t len[kQ], mx = 0;
        sfor<kQ>([&](auto Q) {
            const uint64_t l = (uint64_t)(be[Q] - bs[Q]);
            len[Q] = l > kLongB ? 0u : (uint32_t)l;
            mx = max(mx, len[Q]);
            // a long B row: the whole wave over its part in [lo, hi)
            for (unsigned long long m = __ballot(l > kLongB); m; m &= m - 1) {
                const int l0 = (int)__builtin_ctzll(m);
                const I s0 = (I)readlane_u64((uint64_t)bs[Q], l0), e0 = (I)readlane_u64((uint64_t)be[Q], l0);
                const S at = readlane_val(a[Q], l0);
                I s1 = s0, e1 = e0;
                if (!all_cols) b_range<I>(p.b_col, s0, e0, lo, hi, s1, e1);
                if constexpr (SLAT_LONG_UNROLL > 1) {
                    // several 64-entry stretches per step: their loads in flight together
                    constexpr int kLU = SLAT_LONG_UNROLL > 1 ? SLAT_LONG_UNROLL : 2;
                    for (I j0 = s1 + (I)lane; j0 < e1; j0 += (I)(kLU * kWave)) {
                        uint32_t cc[kLU];
                        S vv[kLU];
                        sfor<kLU>([&](auto U) {
                            const I j = j0 + (I)(U * kWave);
                            cc[U] = 0;
                            vv[U] = S(0);
                            if (j < e1) {
                                cc[U] = p.b_col[j];
                                if constexpr (VALS) vv[U] = bv[j];
                            }
                        });
                        sfor<kLU>([&](auto U) {
                            if (j0 + (I)(U * kWave) < e1) fn(cc[U], at, vv[U]);
                        });
                    }
                } else {
                    for (I j = s1 + (I)lane; j < e1; j += (I)kWave) fn(p.b_col[j], at, VALS ? bv[j] : S(0));
                }
            }
        });
        mx = wave_max_u32(mx);
        for (uint32_t t = 0; t < mx; t += 2) {
            uint32_t c[kQ][2];
            S b[kQ][2];
            sfor<kQ>([&](auto Q) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    c[Q][u] = kSent;
                    b[Q][u] = S(0);
                    if (t + u < len[Q]) {
                        c[Q][u] = p.b_col[bs[Q] + (I)(t + u)];
                        if constexpr (VALS) b[Q][u] = bv[bs[Q] + (I)(t + u)];
                    }
                }
            });
            sfor<kQ>([&](auto Q) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const uint32_t cc = c[Q][u];
                    if (cc != kSent && (all_cols || (cc >= lo && cc < hi))) fn(cc, a[Q], b[Q][u]);
                }
            });
        }
    }
}

// The flattened walk (SLAT_FR_FLAT; variant builds -DSLAT_FR_FLAT=0 keep fr_walk): every product of A
// row [a0, a1) by one block, wave w taking A entries w + 8 * lane, + 512, ... one per lane. The
// entries' B parts [bs, bs + len) are laid end to end and walked 256 products per pass, four per
// lane (product j = e*64 + lane of the pass: consecutive lanes on consecutive entries of a part), so
// every lane is busy whatever the parts' lengths (a hub's long B row and many one-entry parts alike)
// and a pass's loads are in flight together. fr_walk instead gives each lane its own entries and
// the wave waits on the longest; with R-MAT's skewed part lengths most lanes sat idle. Lane -> entry
// by markers: each part's first product in the pass marks its entry (lane + 1) and a running max
// over the pass's positions spreads it. part(k, bs, len): entry k's B part. wl: the wave's LDS,
// fr_flat_bytes<S, VALS, I>(): entry bases I[64] | A values S[64] (VALS) | markers u8[256].
#ifndef SLAT_FR_FLAT
#define SLAT_FR_FLAT 1
#endif
#ifndef SLAT_FOLD_DEPTH
#define SLAT_FOLD_DEPTH 16  // fold-order walk: entries whose B loads are in flight together (variant builds: 1, 4, 8)
#endif
constexpr uint32_t kFlatHuge = 1u << 24;  // parts at least this long: walked by the whole wave alone
// fn(c, a, b) per product.
template <typename S, bool VALS, typename I, typename Part, typename F>
__device__ __forceinline__ void fr_flat(const Args &p, I a0, I a1, Part &&part, F &&fn, uint8_t *wl) {
    const int lane = lane_id();
    const int wv = threadIdx.x / kWave;
    I *eb = (I *)wl;
    S *ea = (S *)(wl + kWave * sizeof(I));
    uint8_t *mk = wl + kWave * (sizeof(I) + (VALS ? sizeof(S) : 0));
    const S *av = (const S *)p.a_val;
    const S *bv = (const S *)p.b_val;
    const auto plus = [](uint32_t x, uint32_t y) { return x + y; };
    const auto mx = [](uint32_t x, uint32_t y) { return max(x, y); };
    // wave w's entries: w, w + 8, w + 16, ... (a row of 100 entries keeps all 8 waves busy)
    for (I base = a0 + (I)wv; base < a1; base += (I)kFB) {
        const I i = base + (I)lane * (I)kFW;
        I bs = 0;
        uint32_t len = 0;
        S a = S(0);
        if (i < a1) {
            const uint32_t k = p.a_col[i];
            if constexpr (VALS) a = av[i];
            if (k < p.b_nrows) part(k, bs, len);
        }
        // a part of 2^24 or more entries on its own (the flat offsets stay below 2^30)
        for (unsigned long long m = __ballot(len >= kFlatHuge); m; m &= m - 1) {
            const int l0 = (int)__builtin_ctzll(m);
            const I s0 = (I)readlane_u64((uint64_t)bs, l0);
            const I e0 = s0 + (I)readlane_u32(len, l0);
            const S at = readlane_val(a, l0);
            for (I j = s0 + (I)lane; j < e0; j += (I)kWave) fn(p.b_col[j], at, VALS ? bv[j] : S(0));
        }
        if (len >= kFlatHuge) len = 0;
        const uint32_t incl = wave_incl_scan(len, 0u, plus);
        const uint32_t tot = readlane_u32(incl, kWave - 1);
        if (tot == 0) continue;  // wave-uniform
        const uint32_t off = incl - len;
        eb[lane] = bs - (I)off;  // product j of the entry: B index eb + j
        if constexpr (VALS) ea[lane] = a;
        for (uint32_t p0 = 0; p0 < tot; p0 += 4 * kWave) {
            if (len && off < p0 + 4 * kWave && off + len > p0) mk[max(off, p0) - p0] = (uint8_t)(lane + 1);
            wave_sync();
            uint32_t L[4], carry = 0;
            sfor<4>([&](auto E) {
                const uint32_t m = mk[E * kWave + lane];
                L[E] = max(wave_incl_scan(m, 0u, mx), carry);
                carry = readlane_u32(L[E], kWave - 1);
            });
            sfor<4>([&](auto E) { mk[E * kWave + lane] = 0; });
            uint32_t c[4];
            S v[4], aa[4];
            sfor<4>([&](auto E) {
                const uint32_t j = p0 + E * kWave + (uint32_t)lane;
                c[E] = kSent;
                v[E] = aa[E] = S(0);
                if (j < tot) {
                    const uint32_t l = L[E] - 1;  // position 0 is always marked: L >= 1
                    const I bi = eb[l] + (I)j;
                    c[E] = p.b_col[bi];
                    if constexpr (VALS) {
                        v[E] = bv[bi];
                        aa[E] = ea[l];
                    }
                }
            });
            sfor<4>([&](auto E) {
                if (c[E] != kSent) fn(c[E], aa[E], v[E]);
            });
            wave_sync();  // the markers clear before the next pass writes them
        }
    }
}

// the split table of B by accumulator chunk (FatArgs::split): thread per (row k, boundary c), a
// binary search in the sorted row; boundary 0 is 0 and boundary nch1 - 1 the row length
// (abs: the absolute offset in B instead, B of < 2^32 entries)
__global__ __launch_bounds__(kBlock) void k_fr_splits(const uint64_t *b_rp, const uint32_t *b_col, uint64_t nb,
                                                       uint32_t nch1, uint32_t chunk_shift, uint32_t *split,
                                                       uint32_t abs = 0) {
    const uint64_t total = nb * nch1;
    for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g < total; g += (uint64_t)gridDim.x * kBlock) {
        const uint64_t k = g / nch1;
        const uint32_t c = (uint32_t)(g - k * nch1);
        const uint64_t s = b_rp[k], e = b_rp[k + 1];
        uint64_t lo = s, hi = e;
        if (c == 0) {
            hi = s;
        } else if (c + 1 < nch1) {
            const uint64_t key = (uint64_t)c << chunk_shift;  // first index with col >= key
            while (lo < hi) {
                const uint64_t mid = lo + (hi - lo) / 2;
                if ((uint64_t)b_col[mid] < key)
                    lo = mid + 1;
                else
                    hi = mid;
            }
        }
        split[g] = (uint32_t)(abs ? hi : hi - s);
    }
}

// block-wide exclusive scan of one u32 per thread (512 threads); returns the block total via *tot
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *sh, uint32_t &tot) {
    const int lane = lane_id(), wv = threadIdx.x / kWave;
    const uint32_t incl = wave_incl_scan(v, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    if (lane == kWave - 1) sh[wv] = incl;
    __syncthreads();
    uint32_t pre = 0;
    tot = 0;
#pragma unroll
    for (int w = 0; w < kFW; ++w) {
        const uint32_t x = sh[w];
        pre += w < wv ? x : 0u;
        tot += x;
    }
    __syncthreads();
    return pre + incl - v;
}

template <typename I>
__global__ __launch_bounds__(kFB) void k_fr_symbolic(FatArgs f) {
    const Args &p = f.a;
    // the pass width: f.sym_bits columns (a multiple of 2048, at most kSymBits), so a matrix narrower
    // than 2^20 columns takes a smaller bitmap and several blocks per CU
    const uint32_t SB = f.sym_bits, kWords = SB / 32;
    // dynamic LDS only (16-byte aligned carve): bitmap | block-scan words | chunk-mask words
    extern __shared__ __attribute__((aligned(16))) uint32_t bits[];
    uint32_t *sh = bits + kWords;
    unsigned long long *shm = (unsigned long long *)(bits + kWords + kFW);
    // the flattened walk's per-wave region (one pass over all columns), markers clear
    constexpr uint32_t kFlat = fr_flat_bytes<uint32_t, false, I>();
    uint8_t *wl = (uint8_t *)(shm + kFW) + (threadIdx.x / kWave) * kFlat;
    ((uint32_t *)(wl + kFlat - 4 * kWave))[lane_id()] = 0;
    const unsigned int nl = *(volatile unsigned int *)f.cnt;
    for (uint32_t w = threadIdx.x; w < kWords; w += kFB) bits[w] = 0;
    __syncthreads();
    __shared__ unsigned long long s_tk;
    const BlockTickets bt(f.tq, nl);
    for (uint64_t li = blockIdx.x; li < nl; li = bt.next(li, &s_tk)) {
        const uint64_t row = f.list[li];
        const I a0 = (I)p.a_rp[row], a1 = (I)p.a_rp[row + 1];
        uint64_t count = 0;
        unsigned long long cm = 0;
        for (uint64_t lo = 0; lo < p.ncols; lo += SB) {
            const uint32_t hi = (uint32_t)min<uint64_t>(p.ncols, lo + SB);
            const bool all = lo == 0 && hi == p.ncols;
            auto mark = [&](uint32_t c, uint32_t, uint32_t) {
                const uint32_t o = c - (uint32_t)lo;
                atomicOr(&bits[o >> 5], 1u << (o & 31));
            };
            if (SLAT_FR_FLAT && all)
                fr_flat<uint32_t, false, I>(
                    p, a0, a1,
                    [&](uint32_t k, I &bs, uint32_t &len) {
                        bs = (I)p.b_rp[k];
                        len = (uint32_t)min<uint64_t>((uint64_t)((I)p.b_rp[k + 1] - bs), 0xFFFFFFFFull);
                    },
                    mark, wl);
            else
                fr_walk<uint32_t, false, I>(p, a0, a1, (uint32_t)lo, hi, all, mark);
            __syncthreads();
            uint32_t pc = 0;
            for (uint32_t w = threadIdx.x; w < kWords; w += kFB) {
                const uint32_t x = bits[w];
                if (x) {
                    pc += __popc(x);
                    cm |= 1ull << cap63((lo + (uint64_t)w * 32) >> f.csh);
                    bits[w] = 0;
                }
            }
            uint32_t tot;
            (void)block_excl_scan(pc, sh, tot);
            count += tot;
        }
        // the touched-chunk mask: OR over the block
        cm = readlane_u64(wave_or_u32((uint32_t)cm) | ((uint64_t)wave_or_u32((uint32_t)(cm >> 32)) << 32), 0);
        if (lane_id() == 0) shm[threadIdx.x / kWave] = cm;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long all = 0;
            for (int w = 0; w < kFW; ++w) all |= shm[w];
            f.cmask[li] = all;
            p.counts[row] = count;
        }
        __syncthreads();
    }
}

// f64 in the reference's order: acc[o] += p. SLAT_FOLD_ATOMIC (default): one LDS atomic add
// (ds_add_f64: an IEEE double add, round to nearest even, as v_add_f64). A wave's LDS instructions
// execute in issue order, so the adds of successive A entries to one column still land in A order —
// the left fold bit for bit — with no wait between entries; otherwise a read, an add and a write, then
// an LDS fence before the next entry (same columns are possible). A wave owns its column slice, so no
// other wave touches these slots.
__device__ __forceinline__ void fold_add(double *acc, uint32_t o, double p) {
    if constexpr (SLAT_FOLD_ATOMIC)
        (void)__hip_atomic_fetch_add(&acc[o], p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else
        acc[o] = __dadd_rn(acc[o], p);
}
__device__ __forceinline__ void fold_sync() {
    if constexpr (!SLAT_FOLD_ATOMIC) wave_sync();
    fold_order_point();  // the atomic adds: issue order made explicit to the compiler
}

// The chunk's products into the dense accumulator. Integer semirings / f64 any order: LDS atomics,
// lanes over A entries. f64 in the reference's order: wave w owns columns [c0 + w*span, ...) and
// walks the A entries in order, lanes over one B row (distinct columns): one writer per column.
template <typename Sem, typename I>
__device__ __forceinline__ void fr_accumulate(const FatArgs &f, I a0, I a1, uint32_t c0, uint32_t c1,
                                              typename Sem::V *acc, uint32_t *bits, uint8_t *wl) {
    using S = typename Sem::S;
    const Args &p = f.a;
    const S *av = (const S *)p.a_val;
    const S *bv = (const S *)p.b_val;
    // the chunk's granules in the split table: [g0, g1)
    const uint32_t g0 = c0 >> f.gsh, g1 = min(f.nch1 - 1, (c1 + (1u << f.gsh) - 1) >> f.gsh);
    if constexpr (!Sem::kOrdered && SLAT_FR_FLAT) {
        if (f.split) {  // the chunk's part of each B row from the split table: no filtering
            fr_flat<S, true, I>(
                p, a0, a1,
                [&](uint32_t k, I &bs, uint32_t &len) {
                    const uint32_t *sp = f.split + (uint64_t)k * f.nch1;
                    const uint32_t s0 = sp[g0];
                    bs = (f.split_abs ? (I)0 : (I)p.b_rp[k]) + (I)s0;
                    len = sp[g1] - s0;
                },
                [&](uint32_t c, S a, S b) {
                    const uint32_t o = c - c0;
                    Sem::acc(acc, o, Sem::prod(a, b));
                    atomicOr(&bits[o >> 5], 1u << (o & 31));
                },
                wl);
            return;
        }
    }
    if constexpr (!Sem::kOrdered) {
        const bool all = c0 == 0 && c1 == p.ncols;
        fr_walk<S, true, I>(p, a0, a1, c0, c1, all, [&](uint32_t c, S a, S b) {
            const uint32_t o = c - c0;
            Sem::acc(acc, o, Sem::prod(a, b));
            atomicOr(&bits[o >> 5], 1u << (o & 31));
        }, f.split, f.nch1, g0, g1, f.split_abs);
    } else if (f.split && (1u << f.gsh) * kFW == fr_chunk<Sem>()) {
        // the split table's granule is one wave's slice: each A entry's part of the B row is two
        // loads, no search. Entries with a non-empty part, in A order; the next one's B entries
        // load while this one's products are added.
        const int lane = lane_id(), wv = threadIdx.x / kWave;
        const uint32_t g = g0 + (uint32_t)wv;
        if ((c0 + ((uint32_t)wv << f.gsh)) >= c1) return;
        // 64 entries at a time, the next groups' loads in flight under this group's products: the
        // entries two groups ahead, the B parts (bounds + split) one group ahead
        auto load_k = [&](I base, uint32_t &k, S &a) {
            const I i = base + (I)lane;
            k = kSent;
            a = S(0);
            if (i < a1) {
                k = p.a_col[i];
                a = av[i];
            }
        };
        auto load_part = [&](uint32_t k, I &bs, I &be) {
            bs = be = 0;
            if (k < p.b_nrows) {
                const I r = f.split_abs ? (I)0 : (I)p.b_rp[k];
                const uint32_t *sp = f.split + (uint64_t)k * f.nch1 + g;
                bs = r + (I)sp[0];
                be = r + (I)sp[1];
            }
        };
        uint32_t kA, kB;
        S aA, aB;
        I bsA, beA;
        load_k(a0, kA, aA);
        load_k(a0 + (I)kWave, kB, aB);
        load_part(kA, bsA, beA);
        for (I base = a0; base < a1; base += (I)kWave) {
            S a_now = aA;
            I bs_now = bsA, be_now = beA;
            I bsB, beB;
            uint32_t kC;
            S aC;
            load_part(kB, bsB, beB);
            load_k(base + (I)(2 * kWave), kC, aC);
            bsA = bsB;
            beA = beB;
            aA = aB;
            kB = kC;
            aB = aC;
            unsigned long long m = __ballot(bs_now != be_now);
            // the group's entries with a non-empty part, in A order, kFD at a time: the next kFD
            // entries' B loads are issued before this kFD's products are added (adds stay in entry
            // order; only the loads move ahead)
            constexpr int kFD = SLAT_FOLD_DEPTH;
            // an entry ahead holds only its lane in the group: its bounds and A value are read again
            // from the group's registers when it is applied (holding them took 16 x 2 x 4 SGPRs,
            // 192 spilled: C5 2^18 fold 77.8 -> 73.2 ms, profiles/r05_fold_lane_ab18.txt)
            struct Ent {
                uint32_t c[kFD];
                S v[kFD];
                int t[kFD];
            };
            auto fetch = [&](Ent &q) {
                sfor<kFD>([&](auto U) {
                    q.t[U] = -1;
                    q.v[U] = S(0);
                    q.c[U] = 0;
                    if (m) {
                        const int t = (int)__builtin_ctzll(m);
                        m &= m - 1;
                        q.t[U] = t;
                        const I s0 = (I)readlane_u64((uint64_t)bs_now, t), e0 = (I)readlane_u64((uint64_t)be_now, t);
                        if (s0 + (I)lane < e0) {
                            q.c[U] = p.b_col[s0 + (I)lane];
                            q.v[U] = bv[s0 + (I)lane];
                        }
                    }
                });
            };
            auto apply = [&](const Ent &q) {
                sfor<kFD>([&](auto U) {
                    const int t = q.t[U];
                    if (t >= 0) {  // wave-uniform
                        const I s = (I)readlane_u64((uint64_t)bs_now, t), e = (I)readlane_u64((uint64_t)be_now, t);
                        const S a = readlane_val(a_now, t);
                        if (s + (I)lane < e) {
                            const uint32_t o = q.c[U] - c0;
                            fold_add(acc, o, __dmul_rn(a, q.v[U]));
                            atomicOr(&bits[o >> 5], 1u << (o & 31));
                        }
                        fold_sync();
                        for (I j0 = s + (I)kWave; j0 < e; j0 += (I)kWave) {
                            const I j = j0 + (I)lane;
                            if (j < e) {
                                const uint32_t o = p.b_col[j] - c0;
                                fold_add(acc, o, __dmul_rn(a, bv[j]));
                                atomicOr(&bits[o >> 5], 1u << (o & 31));
                            }
                            fold_sync();
                        }
                    }
                });
            };
            if (m) {
                Ent qa, qb;
                fetch(qa);
                for (;;) {
                    const bool mb = m != 0;
                    if (mb) fetch(qb);
                    apply(qa);
                    if (!mb) break;
                    const bool ma = m != 0;
                    if (ma) fetch(qa);
                    apply(qb);
                    if (!ma) break;
                }
            }
        }
    } else {
        const int lane = lane_id(), wv = threadIdx.x / kWave;
        const uint32_t span = (c1 - c0 + kFW - 1) / kFW;
        const uint32_t lo = c0 + (uint32_t)wv * span, hi = min(c1, lo + span);
        if (lo >= hi) return;
        for (I base = a0; base < a1; base += (I)kWave) {
            const I i = base + (I)lane;
            uint32_t k = kSent;
            S a = S(0);
            I bs = 0, be = 0;
            if (i < a1) {
                k = p.a_col[i];
                a = av[i];
                if (k < p.b_nrows) {
                    const I r = (f.split && f.split_abs) ? (I)0 : (I)p.b_rp[k];
                    if (f.split) {  // the chunk's part of the B row
                        const uint32_t *sp = f.split + (uint64_t)k * f.nch1;
                        bs = r + (I)sp[g0];
                        be = r + (I)sp[g1];
                    } else {
                        bs = r;
                        be = (I)p.b_rp[k + 1];
                    }
                }
            }
            const int cnt = (int)min<uint64_t>((uint64_t)kWave, (uint64_t)(a1 - base));
            for (int t = 0; t < cnt; ++t) {  // A entries in order: the left fold
                const I s0 = (I)readlane_u64((uint64_t)bs, t), e0 = (I)readlane_u64((uint64_t)be, t);
                if (s0 == e0) continue;
                const S at = readlane_val(a, t);
                I s, e;
                b_range<I>(p.b_col, s0, e0, lo, hi, s, e);
                for (I j = s + (I)lane; j < e; j += (I)kWave) {
                    const uint32_t o = p.b_col[j] - c0;
                    fold_add(acc, o, __dmul_rn(at, bv[j]));
                    atomicOr(&bits[o >> 5], 1u << (o & 31));
                }
                fold_sync();  // this entry's adds land before the next entry's (same columns)
            }
        }
    }
}

// MAGNUS's long-row category with the products bucketed: one walk counts each accumulator chunk's
// products, a second writes them (column, product) into the chunk's bucket in the block's global
// region, and each chunk then accumulates from its bucket alone. Two walks of the row instead of one
// per touched chunk, each of which pays every A entry's B-row bounds again (a hub row touching 16
// chunks walked 16 times), for one write and one read of the products. Returns false (nothing
// written) when the row's products outgrow the block's region.
template <typename Sem, typename I, typename Emit>
__device__ __forceinline__ bool fr_bucketed(const FatArgs &f, I a0, I a1, uint32_t nbk, uint32_t *bcnt, uint32_t *boff,
                                            typename Sem::V *acc, uint32_t *bits, uint32_t *sh, Emit &&emit) {
    using S = typename Sem::S;
    using P = typename Sem::P;
    constexpr uint32_t CH = fr_chunk<Sem>();
    constexpr uint32_t csh = __builtin_ctz(CH);
    const Args &p = f.a;
    const uint32_t t = threadIdx.x;
    for (uint32_t c = t; c < nbk; c += kFB) bcnt[c] = 0;
    __syncthreads();
    fr_walk<S, false, I>(p, a0, a1, 0u, (uint32_t)p.ncols, true, [&](uint32_t c, S, S) { atomicAdd(&bcnt[c >> csh], 1u); });
    __syncthreads();
    uint32_t tot;
    const uint32_t ex = block_excl_scan(t < nbk ? bcnt[t] : 0u, sh, tot);
    if (tot > f.bcap) return false;  // block-uniform
    if (t < nbk) {
        boff[t] = ex;
        bcnt[t] = ex;  // from here the chunk's write cursor
    }
    __syncthreads();
    uint32_t *bc = f.bcol + (uint64_t)blockIdx.x * f.bcap;
    P *bv = (P *)f.bval + (uint64_t)blockIdx.x * f.bcap;
    fr_walk<S, true, I>(p, a0, a1, 0u, (uint32_t)p.ncols, true, [&](uint32_t c, S a, S b) {
        const uint32_t at = atomicAdd(&bcnt[c >> csh], 1u);
        bc[at] = c;
        bv[at] = Sem::prod(a, b);
    });
    __syncthreads();
    for (uint32_t k = 0; k < nbk; ++k) {
        const uint32_t s0 = boff[k], s1 = k + 1 < nbk ? boff[k + 1] : tot;
        if (s0 == s1) continue;  // block-uniform
        const uint32_t c0 = k << csh;
        for (uint32_t i = s0 + t; i < s1; i += kFB) {
            const uint32_t o = bc[i] - c0;
            Sem::acc(acc, o, bv[i]);
            atomicOr(&bits[o >> 5], 1u << (o & 31));
        }
        __syncthreads();
        emit(c0);
    }
    return true;
}

template <typename Sem, typename I>
__global__ __launch_bounds__(kFB) void k_fr_numeric(FatArgs f) {
    using S = typename Sem::S;
    using V = typename Sem::V;
    const Args &p = f.a;
    constexpr uint32_t CH = fr_chunk<Sem>();
    constexpr uint32_t kWords = CH / 32;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    V *acc = (V *)smem;
    uint32_t *bits = (uint32_t *)(smem + (size_t)CH * sizeof(V) * Sem::kSlots);
    uint32_t *sh = bits + kWords;
    uint32_t *bcnt = sh + 128, *boff = bcnt + kMaxBuckets;  // (bucketed rows; past the scan words)
    // the flattened walk's per-wave region (its markers start clear), past the bucket counters
    constexpr uint32_t kFlat = fr_flat_bytes<S, true, I>();
    uint8_t *wl = (uint8_t *)(Sem::kOrdered ? bcnt : boff + kMaxBuckets) + (threadIdx.x / kWave) * kFlat;  // (fr_lds)
    ((uint32_t *)(wl + kFlat - 4 * kWave))[lane_id()] = 0;
    for (uint32_t w = threadIdx.x; w < CH * Sem::kSlots; w += kFB) acc[w] = V(0);
    for (uint32_t w = threadIdx.x; w < kWords; w += kFB) bits[w] = 0;
    __syncthreads();
    S *cval = (S *)p.c_val;
    const unsigned int nl = *(volatile unsigned int *)f.cnt;
    const uint32_t nbk = (uint32_t)((p.ncols + CH - 1) / CH);
    uint32_t zrows = 0;
    __shared__ unsigned long long s_tk;
    const BlockTickets bt(f.tq, nl);
    for (uint64_t li = blockIdx.x; li < nl; li = bt.next(li, &s_tk)) {
        const uint64_t row = f.list[li];
        const I a0 = (I)p.a_rp[row], a1 = (I)p.a_rp[row + 1];
        const uint64_t ob = p.c_rp[row], oe = p.c_rp[row + 1];
        const unsigned long long cm = f.cmask[li];
        uint64_t pos = 0;
        uint32_t zeros = 0;
        // emit of the chunk at c0 from the accumulator: thread t owns bitmap word t (32 columns),
        // positions by a block scan; leaves the accumulator and bitmap clear
        auto emit = [&](uint32_t c0) {
            uint32_t x = 0;
            if (threadIdx.x < kWords) x = bits[threadIdx.x];
            uint32_t tot;
            const uint32_t pre = block_excl_scan(__popc(x), sh, tot);
            uint32_t q = 0;
            for (uint32_t m = x; m; m &= m - 1, ++q) {
                const uint32_t o = threadIdx.x * 32 + (uint32_t)__builtin_ctz(m);
                S v = Sem::finish(acc, o);
#pragma unroll
                for (int w = 0; w < Sem::kSlots; ++w) acc[o * Sem::kSlots + w] = V(0);
                zeros += Sem::is_zero(v) ? 1u : 0u;
                const uint64_t at = ob + pos + pre + q;
                if (at < oe) {  // never write past the row's slice
                    p.c_col[at] = c0 + o;
                    cval[at] = v;
                }
            }
            if (threadIdx.x < kWords) bits[threadIdx.x] = 0;
            pos += tot;
            __syncthreads();
        };
        bool done = false;
        if constexpr (!Sem::kOrdered)
            // bucketed when the row spans 3 or more chunks (fewer: the re-walks cost no more)
            if (f.bcol && nbk <= kMaxBuckets && __popcll(cm) >= 3)
                done = fr_bucketed<Sem, I>(f, a0, a1, nbk, bcnt, boff, acc, bits, sh, emit);
        if (!done) {
            for (uint64_t c0 = 0; c0 < p.ncols; c0 += CH) {
                // skip chunks with no product (mask granule 2^csh columns, a multiple of CH or the last)
                if (!((cm >> cap63(c0 >> f.csh)) & 1ull)) continue;
                const uint32_t c1 = (uint32_t)min<uint64_t>(p.ncols, c0 + CH);
                fr_accumulate<Sem, I>(f, a0, a1, (uint32_t)c0, c1, acc, bits, wl);
                __syncthreads();
                emit((uint32_t)c0);
            }
        }
        uint32_t zt;
        (void)block_excl_scan(zeros, sh, zt);
        if (threadIdx.x == 0) {
            p.counts[row] = pos - zt;
            zrows += zt ? 1u : 0u;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0 && zrows)
        __hip_atomic_fetch_add(&p.host_out[2], (unsigned long long)zrows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace slat

using namespace slat;

// products per row from which a row is fat. B in CSR form (rows past the ELL limit: power-law
// graphs) and a semiring that adds with atomics: 2048 since the flattened walk (round 4: R-MAT 2^16
// A^2 7.56 -> 6.65 ms, C5 2^16 any order 8.51 -> 6.98, 2^18 any 45.7 -> 45.1 against 8192; 1024 and
// 512 measured between, profiles/r04_inv1.txt). Otherwise 8192 (16384 until round 3,
// r03_ab_fat_min.txt): f64 in the reference's fold order keeps the ordered per-slice walk, and ELL
// launches (short B rows, the 30^3 chain) keep their rows in the window kernels.
// SLAT_FAT_MIN: A/B knob (both cases)
uint64_t slat_fat_min(bool flat) {
    static const uint64_t v = [] {
        const char *e = slat_ab_knob("SLAT_FAT_MIN");
        return e ? std::max<uint64_t>(256, std::strtoull(e, nullptr, 10)) : 0ull;
    }();
    return v ? v : flat ? 2048ull : 8192ull;
}

// workspace bytes of the fat-row category for n rows
hipError_t slat_launch_splits(slat_ctx *ctx, const uint64_t *b_rp, const uint32_t *b_col, uint64_t nb, uint32_t nch1,
                              uint32_t shift, uint32_t *split, hipStream_t s, uint32_t abs) {
    const unsigned gs = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nb * nch1 + kBlock - 1) / kBlock,
                                                                           (uint64_t)ctx->cu_count * 16));
    hipLaunchKernelGGL(k_fr_splits, dim3(gs), dim3(kBlock), 0, s, b_rp, b_col, nb, nch1, shift, split, abs);
    return hipGetLastError();
}

size_t slat_fat_ws(uint64_t n) { return ((n + 255) & ~255ull) * (1 + 4 + 8) + 256; }

// Select the fat rows (marks into a.fr_mark's buffer) and count them on the device; nothing to do on
// the host. `ws` = slat_fat_ws(n) bytes of workspace.
slat_status slat_fat_select(slat_ctx *ctx, Args &a, void *ws, uint64_t fat_min, FatArgs *out) {
    const hipStream_t s = ctx->stream;
    const uint64_t n = a.nrows;
    const uint64_t nn = (n + 255) & ~255ull;
    uint8_t *w = (uint8_t *)ws;
    FatArgs f;
    f.mark = w;
    f.list = (uint32_t *)(w + nn);
    f.cmask = (unsigned long long *)(w + nn * 5);
    f.cnt = (unsigned int *)(w + nn * 13);
    // the chunk mask's granule: at least the largest accumulator chunk (2^14 columns), at most 64
    // granules over the columns
    uint32_t csh = 14;
    while (csh < 63 && (a.ncols >> csh) > 63) ++csh;
    f.csh = csh;
    f.split = nullptr;
    f.nch1 = 0;
    f.gsh = 0;
    f.bcol = nullptr;
    f.bval = nullptr;
    f.bcap = 0;
    f.tq = ctx->d_words + 5;
    f.fat_min = fat_min;
    f.buckets = 0;
    SLAT_HIP(ctx, hipMemsetAsync(f.cnt, 0, 4, s));
    a.fr_mark = f.mark;
    f.a = a;
    const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + kBlock - 1) / kBlock, (uint64_t)ctx->cu_count * 8));
    hipLaunchKernelGGL(k_fr_select, dim3(g), dim3(kBlock), 0, s, f);
    SLAT_HIP(ctx, hipGetLastError());
    *out = f;
    return SLAT_OK;
}

slat_status slat_fat_symbolic(slat_ctx *ctx, FatArgs &f, const Args &a, bool idx32) {
    f.a = a;
    // the bitmap covers min(2^20, columns rounded up to 2048) per pass; narrower matrices fit more
    // blocks per CU (SLAT_FAT_SYM_FULL=1: always 2^20, one block per CU)
    static const bool kFull = slat_ab_knob("SLAT_FAT_SYM_FULL") != nullptr;
    const uint64_t sb = kFull ? kSymBits : std::min<uint64_t>(kSymBits, (a.ncols + 2047) / 2048 * 2048);
    f.sym_bits = (uint32_t)sb;
    const size_t flat = (size_t)kFW * fr_flat_bytes<uint32_t, false, uint64_t>();
    const size_t lds = sb / 8 + kFW * 4 + kFW * 8 + flat, lds_max = kSymBits / 8 + kFW * 4 + kFW * 8 + flat;
    const unsigned per_cu = (unsigned)std::max<size_t>(1, std::min<size_t>(4, (160u * 1024u) / lds));
    const dim3 g((unsigned)ctx->cu_count * per_cu);
    static std::atomic<uint64_t> attr{0};  // devices whose attribute is set (idempotent, so a race is harmless)
    if (!(attr.load(std::memory_order_relaxed) >> (ctx->device & 63) & 1)) {  // > 64 KB of dynamic LDS per block
        (void)hipFuncSetAttribute((const void *)k_fr_symbolic<uint32_t>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max);
        (void)hipFuncSetAttribute((const void *)k_fr_symbolic<uint64_t>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max);
        attr.fetch_or(1ull << (ctx->device & 63), std::memory_order_relaxed);
    }
    if (idx32)
        hipLaunchKernelGGL(k_fr_symbolic<uint32_t>, g, dim3(kFB), lds, ctx->stream, f);
    else
        hipLaunchKernelGGL(k_fr_symbolic<uint64_t>, g, dim3(kFB), lds, ctx->stream, f);
    SLAT_HIP(ctx, hipGetLastError());
    return SLAT_OK;
}

// split tables above this size are not built (the walks then filter B rows by column range)
static const uint64_t kSplitBytes = [] {
    const char *e = slat_ab_knob("SLAT_FAT_SPLIT_BYTES");
    return e ? std::strtoull(e, nullptr, 10) : (256ull << 20);
}();

template <typename Sem>
static hipError_t fr_num(slat_ctx *ctx, const FatArgs &f, bool idx32) {
    const dim3 g((unsigned)ctx->cu_count * (128u / fr_kb<Sem>()));  // the resident blocks
    const size_t lds = fr_lds<Sem>();
    // the chunk mask's granule must be a multiple of this instance's chunk
    FatArgs h = f;
    if ((1ull << h.csh) < fr_chunk<Sem>()) return hipErrorInvalidValue;
    // B split by this instance's accumulator chunk, so each chunk's walk loads only its own entries
    // (MAGNUS's column-chunk reordering, applied to B once instead of to every fat row's products)
    // (f64 in the reference's order: granules of one wave's slice of a chunk when that table fits,
    // so no wave searches its slice in a B row)
    const uint64_t nb = h.a.b_nrows;
    uint32_t sh = (uint32_t)__builtin_ctz(fr_chunk<Sem>());
    static const bool kNoSlices = slat_ab_knob("SLAT_NO_FAT_SLICES") != nullptr;  // A/B knob
    if (Sem::kOrdered && !kNoSlices) {
        const uint32_t fine = sh - (uint32_t)__builtin_ctz((uint32_t)kFW);
        const uint64_t ng = (h.a.ncols + (1ull << fine) - 1) >> fine;
        if (nb * (ng + 1) * 4 <= kSplitBytes) sh = fine;
    }
    const uint64_t nch = (h.a.ncols + (1ull << sh) - 1) >> sh;  // granules
    uint32_t *split = nullptr;
    h.split = nullptr;
    h.nch1 = 0;
    h.gsh = sh;
    static const bool kNoSplit = slat_ab_knob("SLAT_NO_FAT_SPLIT") != nullptr;  // A/B knob
    if (nch > 1 && nb * (nch + 1) * 4 <= kSplitBytes && !kNoSplit) {
        if (slat_dev_alloc(ctx, (void **)&split, nb * (nch + 1) * 4, ctx->stream) == hipSuccess) {
            const unsigned gs = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nb * (nch + 1) + kBlock - 1) / kBlock,
                                                                                   (uint64_t)ctx->cu_count * 16));
            // (f.split_abs on entry: the host's permission, B has < 2^32 entries)
            hipLaunchKernelGGL(k_fr_splits, dim3(gs), dim3(kBlock), 0, ctx->stream, h.a.b_rp, h.a.b_col, nb,
                               (uint32_t)(nch + 1), sh, split, h.split_abs);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) {
                slat_dev_free(ctx, split, ctx->stream);
                return e;
            }
            h.split = split;
            h.nch1 = (uint32_t)(nch + 1);
        } else {
            (void)hipGetLastError();
        }
    }
    // product buckets (not for the fold order): bcap pairs per block, dropped when the memory is not there
    uint32_t *bcol = nullptr;
    void *bval = nullptr;
    h.bcol = nullptr;
    h.bval = nullptr;
    h.bcap = 0;
    // (off by default: with the long B rows' loads in flight together, the per-chunk walks over B split
    // by chunk beat the bucket scatter, which moves 4x the bytes: R-MAT 2^16 A^2 fat rows 7.4 GB /
    // 6.9 ms against 1.8 GB / 3.6 ms, profiles/r03_fat_bucket_vs_rewalk.txt; SLAT_FLAG_FAT_BUCKETS: on)
    if (!Sem::kOrdered && f.buckets && (h.a.ncols + fr_chunk<Sem>() - 1) / fr_chunk<Sem>() <= kMaxBuckets) {
        const uint32_t cap = 1u << 19;
        const size_t nbk = (size_t)g.x * cap;
        if (slat_dev_alloc(ctx, (void **)&bcol, nbk * 4, ctx->stream) == hipSuccess &&
            slat_dev_alloc(ctx, &bval, nbk * sizeof(typename Sem::P), ctx->stream) == hipSuccess) {
            h.bcol = bcol;
            h.bval = bval;
            h.bcap = cap;
        } else {
            (void)hipGetLastError();
            if (bcol) slat_dev_free(ctx, bcol, ctx->stream);
            bcol = nullptr;
        }
    }
    static std::atomic<uint64_t> attr{0};  // per device, as above
    if (!(attr.load(std::memory_order_relaxed) >> (ctx->device & 63) & 1)) {  // > 64 KB of dynamic LDS per block
        (void)hipFuncSetAttribute((const void *)k_fr_numeric<Sem, uint32_t>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void *)k_fr_numeric<Sem, uint64_t>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr.fetch_or(1ull << (ctx->device & 63), std::memory_order_relaxed);
    }
    if (idx32)
        hipLaunchKernelGGL((k_fr_numeric<Sem, uint32_t>), g, dim3(kFB), lds, ctx->stream, h);
    else
        hipLaunchKernelGGL((k_fr_numeric<Sem, uint64_t>), g, dim3(kFB), lds, ctx->stream, h);
    const hipError_t e = hipGetLastError();
    if (split) slat_dev_free(ctx, split, ctx->stream);  // stream-ordered: reused only by later work
    if (bcol) slat_dev_free(ctx, bcol, ctx->stream);
    if (bval) slat_dev_free(ctx, bval, ctx->stream);
    return e;
}

slat_status slat_fat_numeric(slat_ctx *ctx, FatArgs &f, const Args &a, int32_t dtype, bool f64any, bool idx32) {
    f.a = a;
    hipError_t e;
    if (dtype == SLAT_U32) e = fr_num<SemU32>(ctx, f, idx32);
    else if (dtype == SLAT_SAT64) e = fr_num<SemSat64>(ctx, f, idx32);
    else if (f64any) e = fr_num<SemF64Any>(ctx, f, idx32);
    else e = fr_num<SemF64>(ctx, f, idx32);
    SLAT_HIP(ctx, e);
    return SLAT_OK;
}
