// spgemm_kernels.hpp — gfx950 device code for row-wise (Gustavson) SpGEMM C = A·B.
//
// Data layout in HBM (the reference's CSR, src/graph_csr.rs:42-53): row_ptr u64[n+1],
// col_idx u32[nnz] (sorted, unique per row), values u32 | u64 | f64 [nnz].
//
// Pipeline (the reference's matmul_par structure, src/graph_csr.rs:360-476, re-designed):
//   k_symbolic  one wavefront per row: structural nnz via an LDS column bitmap
//   k_scan_rows single-pass decoupled look-back scan -> C.row_ptr
//   k_numeric   one row GROUP (1 or 4 wavefronts) per row:
//                 1. gather: every scalar product (j, a_ik*b_kj) of the row, loaded with batched
//                    independent loads (Q A-entries x U B-entries per lane in flight), into an LDS
//                    product cache (one global traversal per row);
//                 2. bitmap: the row's column set over an LDS window of 32*ww columns;
//                 3. ranks: word prefix popcounts -> rank(j) = wbase[w] + popc(bits below j),
//                    so the output is emitted already sorted (the reference sorts nz_cols,
//                    src/graph_csr.rs:449);
//                 4. values: accumulate cached products into LDS slots indexed by rank;
//                 5. emit: coalesced stores of (col, value) at C.row_ptr[i] + rank.
//               Rows whose products exceed the cache re-traverse global memory instead; rows with
//               more distinct columns than the LDS slots run several rank chunks; rows wider
//               than a window run several windows (MAGNUS-style fine-level column chunking).
//   k_compact   only when an emitted value is exactly zero (f64 cancellation or explicit zero
//               inputs): drops those entries, rebuilding exact row slices (matmul's `v != 0`).
//
// Semantics kept bit-exact (SURVEY.md §8(a) rules 1-4):
//   u32   : product clamped to u32::MAX, u32 LDS atomic adds, a wrap of the running sum sets a
//           per-slot saturation bit (a wrap happens iff the exact sum >= 2^32) == sadd/smul
//           (src/graph_csr.rs:29-37), valid in any order because all values are non-negative.
//   Sat64 : the same with u64 and __umul64hi overflow detection == Sat64 (src/graph_sprs.rs:29-51).
//   f64   : each wavefront walks A's row entries in order with lanes spread over one B row
//           (distinct columns) and owns a disjoint quarter of the rank range, non-atomic
//           __dmul_rn/__dadd_rn: the left fold from 0.0 in A-row order of linalg/src/csr.rs:325-337.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

namespace slat {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kShards = 64;      // sharded status words (avoid one hot atomic address)
constexpr uint32_t kSent = 0xFFFFFFFFu;  // ELL padding (column ids are < n_cols <= 2^32 - 1)
// words of the B-value summary block (context memory, epoch-tagged): max B value, ~min B value
constexpr int kVMaxWord = 0, kVMinInvWord = 3;
constexpr int kRegQ = 4;  // A entries per lane kept in registers across the numeric passes
constexpr int kShardStride = 4;  // [0] total nnz (shard 0), [1] max row nnz, [2] rows with zeros, [3] flops

#ifndef SLAT_PHASES
#define SLAT_PHASES 0  // diagnostic builds: per-phase s_memtime cycles of k_numeric
#endif
#ifndef SLAT_FOLD_ATOMIC
#define SLAT_FOLD_ATOMIC 1  // f64 in the fold order: slot adds as in-order LDS atomics (variant builds: 0)
#endif
#ifndef SLAT_SHORT_PACK
#define SLAT_SHORT_PACK 1  // k_numeric_short: payload-free emit sort of (key << 9 | slot) when it fits 32 bits
#endif
#ifndef SLAT_LONG_UNROLL
#define SLAT_LONG_UNROLL 4  // long B rows walked by the whole wave: 64-entry stretches per step (1, 4 or 8)
#endif
#ifndef SLAT_ACC_Q
#define SLAT_ACC_Q 4  // k_numeric's accumulate, 32-bit values: groups per batch of rank lookups (1, 2 or 4)
#endif
#ifndef SLAT_MK_HOIST
#define SLAT_MK_HOIST 1  // short-row batches: the entry -> row marker reads issued together
#endif
#ifndef SLAT_SYM_CAP_PCT
#define SLAT_SYM_CAP_PCT 70  // k_symbolic_short: a batch's product bound, % of the table's slots
#endif
#ifndef SLAT_AEARLY
#define SLAT_AEARLY 1  // k_numeric: a long row's A values for the narrow bound loaded with its stored bitmap
#endif
#ifndef SLAT_SAT64_NARROW
#define SLAT_SAT64_NARROW 1  // Sat64 rows under the u32 bound accumulate in u32 slots (variant builds: 0)
#endif

#ifndef SLAT_NUM_UNI
#define SLAT_NUM_UNI 1  // k_numeric / k_numeric_short: no B-value loads for a pattern B (variant builds: 0)
#endif
#ifndef SLAT_SYM_PREFETCH
#define SLAT_SYM_PREFETCH 1  // k_symbolic (single-window): the next row's bounds loaded ahead (variant builds: 0)
#endif
constexpr int kPhaseSlots = 16;  // [0..12] phases, [15] rows

// diagnostic builds: s_memtime phase accumulator (compiled away otherwise)
struct PhaseClock {
    uint64_t ph[kPhaseSlots];
    uint64_t t;
    __device__ __forceinline__ void mark(int i) {
        if constexpr (SLAT_PHASES) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            ph[i] += now - t;
            t = now;
        }
    }
};

struct Args {
    const uint64_t *a_rp;
    const uint32_t *a_col;
    const void *a_val;
    const uint64_t *b_rp;
    const uint32_t *b_col;
    const void *b_val;
    uint64_t nrows, ncols;
    uint64_t b_nrows;  // column ids of A index rows of B: anything >= b_nrows is ignored
    uint32_t ww;     // bitmap words per window
    uint32_t area;   // LDS bytes per wave for rank slots (value + u16 column offset)
    uint32_t wide;   // 0 = one window at column 0 covers all columns; 1 = row-span windows
    uint32_t stats;  // count products into shard[3]
    uint32_t ell_wq; // groups of 4 per row in the padded ELL copy of B (0: CSR only)
    uint32_t ablate; // experiments only (SLAT_ABLATE): 1 = symbolic skips its LDS bitmap
    const uint32_t *ell_col;  // [n_B][ell_wq*4] columns, kSent padded
    const void *ell_val;      // [n_B][ell_wq*4] values
    const uint8_t *ell_ng;    // [n_B] groups of 4 holding real entries: ceil(len / 4)
    unsigned long long *b_vmax;  // B-value summary from k_build_ell (u32 only; else null): [kVMaxWord]
                                 // (epoch << 32) | max, [kVMinInvWord] (epoch << 32) | ~min
    uint32_t epoch;
    // stored bitmaps (single-window launches, else null): symbolic keeps row r's touched 64-word
    // blocks at sbm[r * nblk * 64 + w] and their mask at smask[r]; numeric loads them instead of
    // rebuilding the bitmap
    uint32_t *sbm;
    uint32_t *smask;
    uint32_t nblk;
    uint32_t b_maxrow;
    uint32_t cbits;     // k_*_short: column bits of the composite (row, column) keys (0: one row per batch)
    // rows of the window category, appended by the short-row kernels (symbolic / numeric lists)
    // and walked by the MODE 2 launches instead of every row
    uint32_t *list;
    // the list's length (a context word, zero when the call starts: no per-call memset launch, which
    // was 4.8 us of a C4 row block's ~220); list_reset: a word k_symbolic_short's block 0 zeroes
    // (the numeric list's length, appended to by a later kernel of the same call); scan_reset: the
    // word k_scan_rows zeroes for the next call (the other of two alternating symbolic list words)
    unsigned int *list_cnt;
    unsigned int *list_reset;
    unsigned long long *host_out;  // mapped pinned host words: [0] nnz, [1] max row nnz, [2] rows with zeros
    uint64_t *counts;  // symbolic: structural nnz per row; numeric: non-zero nnz per row
    uint64_t *c_rp;    // C.row_ptr (n+1)
    uint32_t *c_col;
    void *c_val;
    unsigned long long *shards;
    // rows of the fat-row category (slat_fat.hip: a workgroup and a dense LDS accumulator per row),
    // which the kernels here skip; null = none
    const uint8_t *fr_mark;
    // rows of the wide launches' window / hash passes (k_symbolic, k_numeric MODE 1 / 2) from a
    // ticket counter instead of a fixed stride over the grid (null)
    unsigned long long *tq;
    // the call's completion (seq != 0: this launch is the call's last kernel; signal_done)
    unsigned long long *done;
    unsigned long long seq;
    // k_symbolic (single-window launches): each block's max row count at bmax[blockIdx.x], so the
    // scan that follows need not reduce it across its tiles (null: the scan does)
    uint32_t *bmax;
    // B (CSR form) bucketed by column chunk of the wide launches' window passes: wsplit[k * wnch1 + g]
    // = the offset in B row k of its first column >= g << chunk_shift(ncols) (null: none). A window
    // walks only its chunks' part of each B row instead of the whole row with a column filter
    const uint32_t *wsplit;
    uint32_t wsplit_abs;  // its entries are absolute offsets in B (no row-pointer load per entry)
    uint32_t wnch1;
    // k_symbolic_short: a batch's product bound (0: kSymHashT * SLAT_SYM_CAP_PCT %). Single-window
    // launches take kHashT / 2, so every row it counts fits k_numeric_short's table and every row it
    // lists (the workgroup kernels') gets a stored bitmap
    uint32_t sym_cap;
    // k_symbolic_short / k_numeric_short: rows per wave tile (0: 64). Fewer when the launch has too
    // few rows to give every resident wave a 64-row tile (the 30^3 chain's 27 000 rows: 422 tiles)
    uint32_t tile_rows;
    // speculative wide launch (null: none): the listed-row launches were not queued, as if every row
    // were short; a short-row kernel that lists a row stores 1 here (a mapped host word) and the host
    // reruns the call with them. k_symbolic_short gives such a row 0 outputs, so the scan and the
    // numeric batches stay inside C's bound-sized arrays
    unsigned long long *spec_flag;
};

__device__ __forceinline__ bool fat_row(const Args &p, uint64_t row) { return p.fr_mark && p.fr_mark[row]; }

// the length of the window-category list the short-row kernels appended to
__device__ __forceinline__ uint64_t list_len(const Args &p) {
    return (uint64_t)__builtin_amdgcn_readfirstlane(*(volatile unsigned int *)p.list_cnt);
}

// End of the call's last kernel (p.seq != 0): the last block to finish stores seq into the mapped host
// word the host spins on (host_out[7]), in place of a one-thread kernel queued behind this one (a
// dispatch of its own, ~4 us per call). Stream order still covers everything after the call; the
// host learns of the end a few hundred ns before the grid has retired.
// The done count is two-level (p.done: [0] groups done, [kDoneStride * (g + 1)] blocks done of group
// g = blockIdx % 8, each word on its own 512-byte stretch): device-scope atomics on one word serialise
// across the XCDs, ~15 ns each, so one word per block cost a 768-block launch ~10 us (C4's empty
// window pass: 11 us); eight group words take an eighth of the blocks each, and the block that ends
// a group adds to [0]. Every word is back at 0 when the launch has signalled.
constexpr uint32_t kDoneStride = 64, kDoneGroups = 8;
constexpr size_t kDoneBytes = (size_t)kDoneStride * (kDoneGroups + 1) * 8;
__device__ __forceinline__ void signal_done(const Args &p) {
    if (p.seq == 0) return;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t G = gridDim.x, g = blockIdx.x % kDoneGroups;
        const uint32_t groups = min(G, kDoneGroups), members = (G - g + kDoneGroups - 1) / kDoneGroups;
        unsigned long long *gw = p.done + (size_t)kDoneStride * (g + 1);
        if (__hip_atomic_fetch_add(gw, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != members - 1) return;
        __hip_atomic_store(gw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_fetch_add(p.done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != groups - 1) return;
        __hip_atomic_store(p.done, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&p.host_out[7], p.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The call's max row count in the one-kernel paths (k_tiny, k_lane), two-level like the done count:
// block b raises word b % 8 (kDoneStride apart) with an epoch-tagged atomicMax and waits for it, so
// the max is in place before any later block can see this block's look-back status; the last block
// takes the max over the eight words of this epoch after its walk. (One word took the launch's ~420
// blocks' atomics in a row, ~15 ns each, all arriving after their sorts: the last blocks' look-back
// publishes waited up to ~6 us behind them.)
constexpr size_t kMaxwBytes = (size_t)kDoneStride * kDoneGroups * 8;
__device__ __forceinline__ void maxw_raise(unsigned long long *maxw8, uint32_t epoch, uint32_t mx) {
    const unsigned long long old =
        atomicMax(&maxw8[(size_t)kDoneStride * (blockIdx.x % kDoneGroups)], ((unsigned long long)epoch << 32) | mx);
    asm volatile("" ::"v"(old));  // wait for it
}
// (a whole wave) the max over the eight words raised in this epoch
__device__ __forceinline__ uint32_t maxw_read(unsigned long long *maxw8, uint32_t epoch);

// ------------------------------------------------------------------------------------------------
// value semirings: S storage type, P cached product, V LDS accumulator
// ------------------------------------------------------------------------------------------------
struct SemU32 {
    using S = uint32_t;
    using P = uint32_t;
    using V = unsigned long long;
    static constexpr int kSlots = 1;  // V words per output slot
    static constexpr bool kOrdered = false;
    static constexpr bool kNarrowable = true;  // u32 slots when a row cannot overflow 2^32
    __device__ static __forceinline__ P prod(S a, S b) {
        const unsigned long long p = (unsigned long long)a * b;
        return p > 0xFFFFFFFFull ? 0xFFFFFFFFu : (P)p;  // Saturating<u32> product
    }
    // exact u64 sum of < 2^32 clamped products, no returned value: the atomics pipeline freely
    __device__ static __forceinline__ void acc(V *vals, uint32_t r, P p) { atomicAdd(&vals[r], (V)p); }
    __device__ static __forceinline__ S finish(const V *vals, uint32_t t) {
        const V v = vals[t];
        return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (S)v;  // the saturating sum
    }
    __device__ static __forceinline__ bool is_zero(S v) { return v == 0; }
};

struct SemSat64 {
    using S = unsigned long long;
    using P = unsigned long long;
    using V = unsigned long long;
    static constexpr int kSlots = 2;  // low / high 32-bit halves of the products, summed apart
    static constexpr bool kOrdered = false;
    // u32 slots when a row cannot reach 2^32 (the same bound as u32: every product and sum is exact
    // in 32 bits, so no saturation can happen): 6 B per output slot instead of 18 B
    static constexpr bool kNarrowable = SLAT_SAT64_NARROW;
    __device__ static __forceinline__ P prod(S a, S b) {
        return __umul64hi(a, b) != 0 ? ~0ull : a * b;  // Saturating<u64> product
    }
    __device__ static __forceinline__ void acc(V *vals, uint32_t r, P p) {
        atomicAdd(&vals[2 * r], p & 0xFFFFFFFFull);
        atomicAdd(&vals[2 * r + 1], p >> 32);
    }
    __device__ static __forceinline__ S finish(const V *vals, uint32_t t) {
        const V lo = vals[2 * t], hi = vals[2 * t + 1] + (vals[2 * t] >> 32);
        return hi > 0xFFFFFFFFull ? ~0ull : ((hi << 32) | (lo & 0xFFFFFFFFull));  // exact sum, saturated
    }
    __device__ static __forceinline__ bool is_zero(S v) { return v == 0; }
};

struct SemF64 {
    using S = double;
    using P = double;
    using V = double;
    static constexpr int kSlots = 1;
    static constexpr bool kOrdered = true;
    static constexpr bool kNarrowable = false;
    __device__ static __forceinline__ P prod(S a, S b) { return __dmul_rn(a, b); }
    // no FMA contraction: Rust's a*b then +. One LDS atomic add (ds_add_f64, an IEEE double add,
    // round to nearest even) instead of a read, an add and a write: the ordered walks give a row's
    // slots to one wave and add its A entries in order, and a wave's LDS instructions execute in
    // issue order, so the adds to one slot land in A order (the left fold) without each entry waiting
    // for the previous one's write (SLAT_FOLD_ATOMIC=0: the read-add-write)
    __device__ static __forceinline__ void acc(V *vals, uint32_t r, P p) {
#if SLAT_FOLD_ATOMIC
        (void)__hip_atomic_fetch_add(&vals[r], p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
        vals[r] = __dadd_rn(vals[r], p);
#endif
    }
    __device__ static __forceinline__ S finish(const V *vals, uint32_t t) { return vals[t]; }
    __device__ static __forceinline__ bool is_zero(S v) { return v == 0.0; }
};

// f64 in any order (SLAT_FLAG_F64_ANY_ORDER; BASELINE config C5 is tolerance-checked): LDS atomic
// adds like the integer semirings, so every traversal, category and batch applies; rows with more
// outputs than the LDS slots accumulate straight into their C slice with global atomics instead of
// re-traversing the row once per rank chunk (kGlobalOverflow).
struct SemF64Any {
    using S = double;
    using P = double;
    using V = double;
    static constexpr int kSlots = 1;
    static constexpr bool kOrdered = false;
    static constexpr bool kNarrowable = false;
    static constexpr bool kGlobalOverflow = true;
    __device__ static __forceinline__ P prod(S a, S b) { return __dmul_rn(a, b); }
    __device__ static __forceinline__ void acc(V *vals, uint32_t r, P p) { atomicAdd(&vals[r], p); }
    __device__ static __forceinline__ S finish(const V *vals, uint32_t t) { return vals[t]; }
    __device__ static __forceinline__ bool is_zero(S v) { return v == 0.0; }
};
template <typename Sem, typename = void>
struct GlobalOverflow : std::false_type {};
template <typename Sem>
struct GlobalOverflow<Sem, std::void_t<decltype(Sem::kGlobalOverflow)>> : std::bool_constant<Sem::kGlobalOverflow> {};

// compile-time loop: f(std::integral_constant<int, i>) for i in [0, N) — indices stay constants, so
// register arrays indexed by them are never demoted to scratch
template <typename F, int... Is>
__device__ __forceinline__ void sfor_impl(F &&f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F &&f) {
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// ------------------------------------------------------------------------------------------------
// wave / group helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// LDS written by some lanes and read by others within one wave: DS instructions of a wave execute
// in order; the fences stop the compiler from reordering across the hand-off.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave64 reductions and scans on DPP (row shifts + row broadcasts): no LDS round trips, unlike
// __shfl_* (ds_bpermute + a wait per step).
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp(uint32_t v, uint32_t identity) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, CTRL, ROW_MASK, 0xf, false);
}
template <typename Op>
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t id, Op op) {
    v = op(v, dpp<0x111>(v, id));         // row_shr:1
    v = op(v, dpp<0x112>(v, id));         // row_shr:2
    v = op(v, dpp<0x114>(v, id));         // row_shr:4
    v = op(v, dpp<0x118>(v, id));         // row_shr:8
    v = op(v, dpp<0x142, 0xa>(v, id));    // row_bcast:15 -> rows 1, 3
    v = op(v, dpp<0x143, 0xc>(v, id));    // row_bcast:31 -> rows 2, 3
    return v;
}
__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, int l);
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    return readlane_u32(wave_incl_scan(v, 0u, [](uint32_t a, uint32_t b) { return a + b; }), kWave - 1);
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    return readlane_u32(wave_incl_scan(v, 0u, [](uint32_t a, uint32_t b) { return max(a, b); }), kWave - 1);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    return readlane_u32(wave_incl_scan(v, 0xFFFFFFFFu, [](uint32_t a, uint32_t b) { return min(a, b); }), kWave - 1);
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
    return readlane_u32(wave_incl_scan(v, 0u, [](uint32_t a, uint32_t b) { return a | b; }), kWave - 1);
}
__device__ __forceinline__ uint32_t wave_excl_scan_u32(uint32_t x) {
    return wave_incl_scan(x, 0u, [](uint32_t a, uint32_t b) { return a + b; }) - x;
}
__device__ __forceinline__ unsigned long long wave_incl_scan_u64(unsigned long long v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const unsigned long long t = __shfl_up(v, d);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    return ((uint64_t)readlane_u32((uint32_t)(v >> 32), l) << 32) | readlane_u32((uint32_t)v, l);
}
__device__ __forceinline__ uint32_t maxw_read(unsigned long long *maxw8, uint32_t epoch) {
    uint32_t m = 0;
    if (lane_id() < (int)kDoneGroups) {
        const unsigned long long w =
            __hip_atomic_load(&maxw8[(size_t)kDoneStride * lane_id()], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        m = (uint32_t)(w >> 32) == epoch ? (uint32_t)w : 0u;
    }
    return wave_max_u32(m);
}

// Work items handed out by a ticket counter instead of a fixed stride, so waves that drew cheap items
// take more of them. Wave w starts on item w without a ticket (a wave with no item never touches
// the counter: one contended address costs ~11 ns per atomic, so 16k waves taking one failing
// ticket each would add ~180 us); after that, ticket t is item waves + t. One device-scope atomic per
// later item, issued one item ahead (its latency overlaps the current item's loads). Every wave
// that had an item takes exactly one ticket past the end, so the last taker knows it is last and
// zeroes the counter for the next launch on the stream.
struct TicketQueue {
    unsigned long long *ctr;
    uint64_t n, waves, total;  // items, waves in the grid, tickets this launch takes
    __device__ __forceinline__ TicketQueue(unsigned long long *c, uint64_t items, uint64_t nw)
        : ctr(c), n(items), waves(nw), total((items > nw ? items - nw : 0) + (items < nw ? items : nw)) {}
    __device__ __forceinline__ unsigned long long issue() const {
        unsigned long long t = 0;
        if (lane_id() == 0) t = atomicAdd(ctr, 1ull);
        return t;
    }
    // the item of a ticket (>= n: none left)
    __device__ __forceinline__ uint64_t resolve(unsigned long long t) const {
        const uint64_t v = readlane_u64(t, 0);
        if (v == total - 1 && lane_id() == 0) __hip_atomic_store(ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return waves + v;
    }
};
// Rows that lost explicit zeros (rare), counted straight into the mapped host word. In a launch that
// signals the call's end the add returns its old value, so it has completed before the wave reaches
// signal_done's barrier (the completion word must not overtake it).
__device__ __forceinline__ void add_zero_rows(unsigned long long *word, uint32_t zrows, bool signals) {
    if (lane_id() != 0 || zrows == 0) return;
    if (signals) {
        const unsigned long long old =
            __hip_atomic_fetch_add(word, (unsigned long long)zrows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("" ::"v"(old));  // wait for the value
    } else {
        __hip_atomic_fetch_add(word, (unsigned long long)zrows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Static tile order with each XCD on a contiguous eighth of the tiles: workgroups go to the 8 XCDs
// round-robin by blockIdx and every XCD has its own L2, so a plain stride over the grid spreads
// neighbouring tiles (rows that gather neighbouring B rows) over all eight L2s. Here XCD x's waves
// stride over [x * per, (x + 1) * per). SLAT_XCD=0: the plain stride.
#ifndef SLAT_XCD
#define SLAT_XCD 1
#endif
constexpr uint32_t kXcds = 8;
struct XcdStride {
    uint64_t first, end, stride;
    __device__ __forceinline__ XcdStride(uint64_t n, int wpb, int wv) {
        if (SLAT_XCD && gridDim.x >= 4 * kXcds) {
            const uint32_t x = blockIdx.x % kXcds, nb = (gridDim.x - x + kXcds - 1) / kXcds;  // blocks on XCD x
            const uint64_t per = (n + kXcds - 1) / kXcds;
            first = x * per + (uint64_t)(blockIdx.x / kXcds) * wpb + wv;
            end = min<uint64_t>(n, (x + 1) * per);
            stride = (uint64_t)nb * wpb;
        } else {
            first = (uint64_t)blockIdx.x * wpb + wv;
            end = n;
            stride = (uint64_t)gridDim.x * wpb;
        }
    }
};
template <typename S>
__device__ __forceinline__ S readlane_val(S v, int l) {
    if constexpr (sizeof(S) == 4) {
        return (S)readlane_u32((uint32_t)v, l);
    } else {
        return __builtin_bit_cast(S, readlane_u64(__builtin_bit_cast(uint64_t, v), l));
    }
}

// a value clamped to u32 (the narrow-slot bound's inputs: a u64 value >= 2^32 never passes it)
template <typename S>
__device__ __forceinline__ uint32_t sat32(S v) {
    if constexpr (sizeof(S) == 4)
        return (uint32_t)v;
    else
        return (uint64_t)v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)v;
}

// Ordered traversal (f64): A's row entries in order, lanes spread over one B row (distinct
// columns), 64 A entries' row pointers prefetched at a time. The first 64 elements of the B rows
// of kOrdAhead consecutive entries are loaded before any of them is visited, so the visits (in A
// order: the left fold of linalg/src/csr.rs:325-337) do not wait on one load chain per entry.
// (4 and 16 measured within 1 % of 8 on C5 2^18, profiles/r05_ord_ahead_ab18.txt)
constexpr int kOrdAhead = 8;
// between two A entries of an ordered walk: a compiler-only barrier, so the relaxed LDS atomic adds
// of one entry are issued before the next entry's (a wave's LDS instructions then execute in issue
// order: the left fold). No hardware wait.
__device__ __forceinline__ void fold_order_point() {
    if constexpr (SLAT_FOLD_ATOMIC) asm volatile("" ::: "memory");
}
template <typename I, typename S, typename F>
__device__ __forceinline__ void traverse_ordered(const Args &p, I a0, I a1, F &&visit) {
    const int lane = lane_id();
    const S *av_ = (const S *)p.a_val;
    const S *bv_ = (const S *)p.b_val;
    for (I base = a0; base < a1; base += kWave) {
        const I idx = base + (I)lane;
        I bs = 0, be = 0;
        S av = S(0);
        if (idx < a1) {
            const uint32_t k = p.a_col[idx];
            av = av_[idx];
            if (k < p.b_nrows) {
                bs = (I)p.b_rp[k];
                be = (I)p.b_rp[k + 1];
            }
        }
        const int cnt = (int)min<uint64_t>((uint64_t)kWave, (uint64_t)(a1 - base));
        struct Ahead {
            uint32_t c[kOrdAhead];
            S v[kOrdAhead];
        };
        auto fetch = [&](int t0, Ahead &q) {
            sfor<kOrdAhead>([&](auto G) {
                q.c[G] = kSent;
                q.v[G] = S(0);
                const int t = t0 + G;
                if (t < cnt) {
                    const I s = (I)readlane_u64((uint64_t)bs, t), e = (I)readlane_u64((uint64_t)be, t);
                    const I jdx = s + (I)lane;
                    if (jdx < e) {
                        q.c[G] = p.b_col[jdx];
                        q.v[G] = bv_[jdx];
                    }
                }
            });
        };
        auto visit_all = [&](int t0, const Ahead &q) {
            sfor<kOrdAhead>([&](auto G) {
                const int t = t0 + G;
                if (t < cnt) {
                    const I s = (I)readlane_u64((uint64_t)bs, t), e = (I)readlane_u64((uint64_t)be, t);
                    const S a = readlane_val(av, t);
                    if (q.c[G] != kSent) visit(q.c[G], a, q.v[G]);
                    for (I jdx = s + (I)kWave + (I)lane; jdx < e; jdx += (I)kWave) visit(p.b_col[jdx], a, bv_[jdx]);
                    fold_order_point();
                }
            });
        };
        // double-buffered: the next kOrdAhead entries' loads are issued before this kOrdAhead
        // are visited (visits stay in A order)
        Ahead qa, qb;
        if (cnt > 0) fetch(0, qa);
        for (int t0 = 0; t0 < cnt; t0 += 2 * kOrdAhead) {
            const bool hb = t0 + kOrdAhead < cnt;
            if (hb) fetch(t0 + kOrdAhead, qb);
            visit_all(t0, qa);
            if (!hb) break;
            const bool ha = t0 + 2 * kOrdAhead < cnt;
            if (ha) fetch(t0 + 2 * kOrdAhead, qa);
            visit_all(t0 + kOrdAhead, qb);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// padded ELL copy of B (rows of B short, e.g. the base adjacency of an A^k chain): row k holds
// ell_wq groups of 4 columns at ell_col[k*ell_wq ..], padded with kSent, and the matching values
// (4 per uint4 for 4-byte values, 4 per 2 uint4 for 8-byte values). One dwordx4 load brings four
// B entries, the B row pointers drop out of the dependent load chain (a_col -> ELL row), and
// rows are 16-byte aligned. Built per call into the context workspace (a few microseconds).
// ------------------------------------------------------------------------------------------------
template <typename S>
__global__ __launch_bounds__(kBlock) void k_build_ell(const uint64_t *rp, const uint32_t *col, const S *val,
                                                       uint32_t n, uint32_t wq, uint32_t *ecol, S *eval, uint8_t *eng,
                                                       unsigned long long *part) {
    // one thread per (row k, group t): 4 columns and 4 values, written as whole groups
    // 32-bit group index: the host keeps n < 2^24 and wq <= 8 for the ELL copy
    uint32_t mx = 0, mn = 0xFFFFFFFFu;
    const uint32_t total = n * wq;
    for (uint32_t g = blockIdx.x * kBlock + threadIdx.x; g < total; g += gridDim.x * kBlock) {
        const uint32_t k = g / wq;
        const uint32_t t = g - k * wq;
        const uint64_t s0 = rp[k], len = rp[k + 1] - s0;
        if (t == 0) eng[k] = (uint8_t)((len + 3) / 4);
        uint32_t c[4];
        S v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint64_t u = (uint64_t)t * 4 + e;
            c[e] = u < len ? col[s0 + u] : kSent;
            v[e] = u < len ? val[s0 + u] : S(0);
            if constexpr (!std::is_floating_point<S>::value)
                if (u < len) {
                    mx = max(mx, sat32(v[e]));
                    mn = min(mn, sat32(v[e]));
                }
        }
        ((uint4 *)ecol)[g] = make_uint4(c[0], c[1], c[2], c[3]);
        if constexpr (sizeof(S) == 4) {
            ((uint4 *)eval)[g] = make_uint4(__builtin_bit_cast(uint32_t, v[0]), __builtin_bit_cast(uint32_t, v[1]),
                                            __builtin_bit_cast(uint32_t, v[2]), __builtin_bit_cast(uint32_t, v[3]));
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) eval[(uint64_t)g * 4 + e] = v[e];
        }
    }
    if constexpr (!std::is_floating_point<S>::value) {
        // max and min B value of this block (clamped to u32), stored as one partial ((~min << 32) | max) that
        // k_scan_rows reduces into the epoch-tagged words: no same-address atomics and no
        // round trip at the end of every block
        __shared__ uint32_t bm[kBlock / kWave], bn[kBlock / kWave];
        mx = wave_max_u32(mx);
        mn = wave_min_u32(mn);
        if (lane_id() == 0) {
            bm[threadIdx.x / kWave] = mx;
            bn[threadIdx.x / kWave] = mn;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < kBlock / kWave; ++w) {
                mx = max(mx, bm[w]);
                mn = min(mn, bn[w]);
            }
            part[blockIdx.x] = ((unsigned long long)~mn << 32) | mx;
        }
    }
}

// k_build_ell's per-block partials ((~min << 32) | max) reduced by one wave into vmax[kVMaxWord] =
// (epoch << 32) | max and vmax[kVMinInvWord] = (epoch << 32) | ~min (a prepared B's summary)
static __global__ __launch_bounds__(kWave) void k_reduce_bparts(const unsigned long long *part, uint32_t n,
                                                                unsigned long long *vmax, uint32_t epoch) {
    uint32_t bx = 0, bn = 0;
    for (uint32_t i = threadIdx.x; i < n; i += kWave) {
        const unsigned long long q = part[i];
        bx = max(bx, (uint32_t)q);
        bn = max(bn, (uint32_t)(q >> 32));
    }
    bx = wave_max_u32(bx);
    bn = wave_max_u32(bn);
    if (threadIdx.x == 0) {
        vmax[kVMaxWord] = ((unsigned long long)epoch << 32) | bx;
        vmax[kVMinInvWord] = ((unsigned long long)epoch << 32) | bn;
    }
}

// the same B-value summary when B is walked in CSR form (no ELL copy): max and ~min of the u32
// values, epoch-tagged, one atomic pair per block
template <typename S>
__global__ __launch_bounds__(kBlock) void k_bvmax(const S *val, uint64_t nnz, unsigned long long *vmax, uint32_t epoch) {
    uint32_t mx = 0, mn = 0xFFFFFFFFu;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nnz; i += (uint64_t)gridDim.x * kBlock) {
        mx = max(mx, sat32(val[i]));
        mn = min(mn, sat32(val[i]));
    }
    __shared__ uint32_t bm[kBlock / kWave], bn[kBlock / kWave];
    mx = wave_max_u32(mx);
    mn = wave_min_u32(mn);
    if (lane_id() == 0) {
        bm[threadIdx.x / kWave] = mx;
        bn[threadIdx.x / kWave] = mn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / kWave; ++w) {
            mx = max(mx, bm[w]);
            mn = min(mn, bn[w]);
        }
        atomicMax(&vmax[kVMaxWord], ((unsigned long long)epoch << 32) | mx);
        atomicMax(&vmax[kVMinInvWord], ((unsigned long long)epoch << 32) | ~mn);
    }
}

template <typename S>
struct Quad {
    S v[4];
};

// the t-th group of 4 values / columns of ELL row k. The host keeps B's ELL image below 2^24 rows and
// 2^31 bytes, so the byte offset is one 24-bit multiply-add and the load takes the SGPR-base +
// 32-bit VGPR-offset form (no 64-bit address math per lane).
template <typename S>
__device__ __forceinline__ Quad<S> ell_vals(const Args &p, uint32_t k, uint32_t t) {
    constexpr uint32_t kGB = 4 * sizeof(S);  // bytes per group of 4 values
    const uint32_t off = __umul24(k, p.ell_wq * kGB) + t * kGB;
    const uint8_t *b = (const uint8_t *)p.ell_val + off;
    Quad<S> q;
    if constexpr (sizeof(S) == 4) {
        const uint4 x = *(const uint4 *)b;
        q.v[0] = __builtin_bit_cast(S, x.x);
        q.v[1] = __builtin_bit_cast(S, x.y);
        q.v[2] = __builtin_bit_cast(S, x.z);
        q.v[3] = __builtin_bit_cast(S, x.w);
    } else {
        const uint4 x = ((const uint4 *)b)[0], y = ((const uint4 *)b)[1];
        q.v[0] = __builtin_bit_cast(S, ((uint64_t)x.y << 32) | x.x);
        q.v[1] = __builtin_bit_cast(S, ((uint64_t)x.w << 32) | x.z);
        q.v[2] = __builtin_bit_cast(S, ((uint64_t)y.y << 32) | y.x);
        q.v[3] = __builtin_bit_cast(S, ((uint64_t)y.w << 32) | y.z);
    }
    return q;
}

__device__ __forceinline__ uint4 ell_cols(const Args &p, uint32_t k, uint32_t t) {
    const uint32_t off = __umul24(k, p.ell_wq * 16u) + t * 16u;
    return *(const uint4 *)((const uint8_t *)p.ell_col + off);
}

// The short-row kernels over B in CSR form (wide launches whose B rows outgrow the ELL image: power-law
// graphs): a "group" is up to 4 consecutive entries of a B row, staged as the offset of its first entry
// in B (u32: the host takes this form only for B of < 2^32 entries) and its entry count - 1 in bits
// 6-7 of the local-row byte. The entries are read where they lie, no image is built.
__device__ __forceinline__ uint4 csr_cols(const Args &p, uint32_t off, uint32_t cnt) {
    const uint32_t *c = p.b_col + off;
    uint4 r;
    r.x = c[0];
    r.y = cnt > 1 ? c[1] : kSent;
    r.z = cnt > 2 ? c[2] : kSent;
    r.w = cnt > 3 ? c[3] : kSent;
    return r;
}
template <typename S>
__device__ __forceinline__ Quad<S> csr_vals(const Args &p, uint32_t off, uint32_t cnt) {
    const S *v = (const S *)p.b_val + off;
    Quad<S> q;
    q.v[0] = v[0];
    q.v[1] = cnt > 1 ? v[1] : S(0);
    q.v[2] = cnt > 2 ? v[2] : S(0);
    q.v[3] = cnt > 3 ? v[3] : S(0);
    return q;
}
// an A entry's B row for the short-row kernels: ELL, its group count; CSR, k becomes the row's first
// entry offset and the count its length (groups = (len + 3) / 4). kSent / out of range: count 0
template <bool CSR>
__device__ __forceinline__ uint32_t short_brow(const Args &p, uint32_t &k) {
    if (k >= p.b_nrows) return 0u;
    if constexpr (CSR) {
        const uint64_t r0 = p.b_rp[k], r1 = p.b_rp[k + 1];
        k = (uint32_t)r0;
        return (uint32_t)min<uint64_t>(r1 - r0, 1u << 30);
    } else {
        return p.ell_ng[k];
    }
}
template <bool CSR>
__device__ __forceinline__ uint32_t short_groups(uint32_t cnt) {
    return CSR ? (cnt + 3) >> 2 : cnt;
}

// ------------------------------------------------------------------------------------------------
// group walks: the passes consume B entries four at a time (one ELL group, or a CSR entry padded
// with kSent), branch-free inside a group, so a wave issues every LDS access of a group before
// it waits on any.
// ------------------------------------------------------------------------------------------------
template <typename S>
__device__ __forceinline__ Quad<S> quad1(S v) {
    Quad<S> q{};
    q.v[0] = v;
    return q;
}

template <typename S>
__device__ __forceinline__ Quad<S> splat4(S v) {
    Quad<S> q;
#pragma unroll
    for (int e = 0; e < 4; ++e) q.v[e] = v;
    return q;
}

template <typename Sem>
__device__ __forceinline__ Quad<typename Sem::S> prods(typename Sem::S a, const Quad<typename Sem::S> &v) {
    Quad<typename Sem::S> pr;
#pragma unroll
    for (int e = 0; e < 4; ++e) pr.v[e] = Sem::prod(a, v.v[e]);
    return pr;
}

// products of a row whose bound max(A) * max(B) * len < 2^32 holds (u32 or Sat64 values): exact in
// 32 bits, no clamp needed
template <typename ST>
struct SemNarrowT {
    using S = ST;
    static constexpr bool kNarrowable = true;
    __device__ static __forceinline__ S prod(S a, S b) { return (S)((uint32_t)a * (uint32_t)b); }
};
using SemU32Narrow = SemNarrowT<uint32_t>;

// passes that need no values (symbolic, bitmap, column span) walk with this stand-in semiring
struct SemNone {
    using S = uint32_t;
    static constexpr bool kNarrowable = false;
    __device__ static __forceinline__ S prod(S, S) { return 0; }
};

// grp(c4, pr4) for every group of B row k, ELL groups from t0 on (CSR: one entry per group);
// pr4 = the products a * b of the group when VALS
template <typename Sem, bool ELL, bool VALS, typename I, typename G>
__device__ __forceinline__ void walk_brow(const Args &p, uint32_t k, typename Sem::S a, uint32_t t0, G &&grp) {
    using S = typename Sem::S;
    if constexpr (ELL) {
        for (uint32_t t = t0; t < p.ell_wq; ++t) {
            const uint4 c = ell_cols(p, k, t);
            Quad<S> pr{};
            if constexpr (VALS) pr = prods<Sem>(a, ell_vals<S>(p, k, t));
            grp(c, pr);
            if (c.w == kSent) break;
        }
    } else {
        const S *bv_ = (const S *)p.b_val;
        const I bs = (I)p.b_rp[k], be = (I)p.b_rp[k + 1];
        for (I jdx = bs; jdx < be; ++jdx)
            grp(make_uint4(p.b_col[jdx], kSent, kSent, kSent), quad1<S>(VALS ? Sem::prod(a, bv_[jdx]) : S(0)));
    }
}

// CSR walk of N A entries per lane (k = B row, kSent = none): a B row of at most kLongB entries is
// walked by its own lane, a longer one by the whole wave (lanes over its columns), so no lane walks
// thousands of entries alone (power-law B rows).
constexpr uint32_t kLongB = 32;
// [g0, g1) (g1 > 0): only the B entries of those column chunks (p.wsplit)
template <typename Sem, bool VALS, typename I, int N, typename G>
__device__ __forceinline__ void walk_csr(const Args &p, const uint32_t *k, const typename Sem::S *a, G &&grp,
                                         uint32_t g0 = 0, uint32_t g1 = 0) {
    using S = typename Sem::S;
    const int lane = lane_id();
    const S *bv_ = (const S *)p.b_val;
    I bs[N], be[N];
    sfor<N>([&](auto Q) {
        bs[Q] = 0;
        be[Q] = 0;
        if (k[Q] < p.b_nrows) {
            if (g1) {
                const I r = p.wsplit_abs ? (I)0 : (I)p.b_rp[k[Q]];
                const uint32_t *sp = p.wsplit + (uint64_t)k[Q] * p.wnch1;
                bs[Q] = r + (I)sp[g0];
                be[Q] = r + (I)sp[g1];
            } else {
                bs[Q] = (I)p.b_rp[k[Q]];
                be[Q] = (I)p.b_rp[k[Q] + 1];
            }
        }
    });
    sfor<N>([&](auto Q) {
        if ((uint64_t)(be[Q] - bs[Q]) <= kLongB)
            for (I jdx = bs[Q]; jdx < be[Q]; ++jdx)
                grp(make_uint4(p.b_col[jdx], kSent, kSent, kSent), quad1<S>(VALS ? Sem::prod(a[Q], bv_[jdx]) : S(0)));
    });
    sfor<N>([&](auto Q) {
        for (unsigned long long m = __ballot((uint64_t)(be[Q] - bs[Q]) > kLongB); m; m &= m - 1) {
            const int l = (int)__builtin_ctzll(m);
            const I s = (I)readlane_u64((uint64_t)bs[Q], l), e = (I)readlane_u64((uint64_t)be[Q], l);
            const S av = readlane_val(a[Q], l);
            if constexpr (SLAT_LONG_UNROLL >= 4) {
                // several 64-entry stretches per step: their loads in flight together, a group call
                // per four
                constexpr int kLU = SLAT_LONG_UNROLL >= 4 ? SLAT_LONG_UNROLL : 4;
                for (I j0 = s + (I)lane; j0 < e; j0 += (I)(kLU * kWave)) {
                    uint32_t cc[kLU];
                    Quad<S> pr[kLU / 4] = {};
                    sfor<kLU>([&](auto U) {
                        const I j = j0 + (I)(U * kWave);
                        cc[U] = kSent;
                        if (j < e) {
                            cc[U] = p.b_col[j];
                            if constexpr (VALS) pr[U / 4].v[U % 4] = bv_[j];
                        }
                    });
                    sfor<kLU / 4>([&](auto Gi) {
                        if constexpr (VALS) sfor<4>([&](auto U) { pr[Gi].v[U] = Sem::prod(av, pr[Gi].v[U]); });
                        grp(make_uint4(cc[4 * Gi], cc[4 * Gi + 1], cc[4 * Gi + 2], cc[4 * Gi + 3]), pr[Gi]);
                    });
                }
            } else {
                for (I jdx = s + (I)lane; jdx < e; jdx += (I)kWave)
                    grp(make_uint4(p.b_col[jdx], kSent, kSent, kSent), quad1<S>(VALS ? Sem::prod(av, bv_[jdx]) : S(0)));
            }
        }
    });
}

// Lane-per-A-entry walk of a row: lane l owns entries base + l and base + 64 + l.
template <typename Sem, bool ELL, bool VALS, typename I, typename G>
__device__ __forceinline__ void walk_row(const Args &p, I a0, I a1, G &&grp, uint32_t g0 = 0, uint32_t g1 = 0) {
    using S = typename Sem::S;
    const int lane = lane_id();
    const S *av_ = (const S *)p.a_val;
    for (I base = a0; base < a1; base += (I)(2 * kWave)) {
        const I i0 = base + (I)lane, i1 = i0 + (I)kWave;
        uint32_t kk[2] = {kSent, kSent};
        S av[2] = {S(0), S(0)};
        if (i0 < a1) {
            kk[0] = p.a_col[i0];
            if constexpr (VALS) av[0] = av_[i0];
        }
        if (i1 < a1) {
            kk[1] = p.a_col[i1];
            if constexpr (VALS) av[1] = av_[i1];
        }
        if constexpr (ELL) {
            if (kk[0] < p.b_nrows) walk_brow<Sem, ELL, VALS, I>(p, kk[0], av[0], 0, grp);
            if (kk[1] < p.b_nrows) walk_brow<Sem, ELL, VALS, I>(p, kk[1], av[1], 0, grp);
        } else {
            walk_csr<Sem, VALS, I, 2>(p, kk, av, grp, g0, g1);
        }
    }
}

// window offset of column c: valid iff c is a real column inside [wlo, wlo + WIN). The padding
// sentinel never lands in a window: the host rejects n_cols > 2^32 - 2^17 (WIN < 2^16).
__device__ __forceinline__ bool win_off(uint32_t c, uint32_t wlo, uint32_t WIN, uint32_t &off) {
    off = c - wlo;
    return off < WIN;  // kSent - wlo >= WIN because the host keeps n_cols <= 2^32 - 2^17
}



// ------------------------------------------------------------------------------------------------
// Short rows of wide launches (MAGNUS's accumulation of rows whose outputs fit a small table): an
// LDS hash table per wave, keys = column ids (kSent = empty, never a column), linear probing.
// Symbolic counts the inserted keys; numeric accumulates values in the slots, then every lane
// ranks the keys it holds by counting the smaller ones among all of the row's keys (broadcast
// reads of a staged key list) and writes (col, value) at out + rank: sorted output, no sort pass.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kHashT = 512;      // numeric slots per wave (rows with <= kHashT / 2 outputs)
constexpr uint32_t kSymHashT = 1024;  // symbolic keys per wave (rows with <= 0.7 * kSymHashT products)
constexpr uint32_t kHashHeld = kHashT / kWave;

// u32 short rows (k_numeric_short): u32 slots plus one wrap bit per slot after them instead of u64
// slots; all terms are non-negative, so a wrap happens iff the exact sum reaches 2^32 and the
// Saturating<u32> sum is then u32::MAX (src/graph_csr.rs:29-37). 2 KB less LDS per wave.
struct SemU32W {
    using S = uint32_t;
    using P = uint32_t;
    using V = uint32_t;
    static constexpr int kSlots = 1;
    static constexpr bool kOrdered = false;
    static constexpr bool kNarrowable = true;
    static constexpr uint32_t kExtraWords = kHashT / 32;  // the wrap bits
    __device__ static __forceinline__ P prod(S a, S b) { return SemU32::prod(a, b); }
    __device__ static __forceinline__ void acc(V *vals, uint32_t r, P p) {
        const uint32_t old = atomicAdd(&vals[r], p);
        if (old + p < old) atomicOr(&vals[kHashT + (r >> 5)], 1u << (r & 31));
    }
    __device__ static __forceinline__ S finish(const V *vals, uint32_t t) {
        return (vals[kHashT + (t >> 5)] >> (t & 31)) & 1u ? 0xFFFFFFFFu : vals[t];
    }
    __device__ static __forceinline__ bool is_zero(S v) { return v == 0; }
};
// SemU32W for a batch whose sums cannot reach 2^32 (max A x max B x groups < 2^32): plain adds, no
// returned value to test for a wrap, so the atomics pipeline freely (the same slots and wrap words)
struct SemU32WN : SemU32W {
    __device__ static __forceinline__ void acc(V *vals, uint32_t r, P p) { atomicAdd(&vals[r], p); }
};
template <typename Sem, typename = void>
struct ExtraWords : std::integral_constant<uint32_t, 0> {};
template <typename Sem>
struct ExtraWords<Sem, std::void_t<decltype(Sem::kExtraWords)>> : std::integral_constant<uint32_t, Sem::kExtraWords> {};
// the semiring k_numeric_short accumulates in
template <typename Sem>
using ShortSem = std::conditional_t<std::is_same_v<Sem, SemU32>, SemU32W, Sem>;

__device__ __forceinline__ uint32_t hash_slot(uint32_t c, uint32_t logt) { return (c * 0x9E3779B1u) >> (32 - logt); }

// slots of N columns at once (kSent = no column): every probe round issues all pending CAS
// before it looks at any result, so the LDS latency is paid once per round, not once per column.
// fresh[i]: this call inserted column i.
// NB: the first round branch-free (below); the numeric tables take it, symbolic's do not (C4: numeric
// 0.825 -> 0.806 ms, symbolic 0.411 -> 0.432 ms with it, profiles/r03_ab_nb2_ballot.txt)
template <int N, bool NB = false>
__device__ __forceinline__ void hash_batch(uint32_t *keys, uint32_t logt, const uint32_t (&c)[N], uint32_t (&sl)[N],
                                           bool (&fresh)[N]) {
    const uint32_t mask = (1u << logt) - 1;
    uint32_t pend = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        sl[i] = hash_slot(c[i], logt);
        fresh[i] = false;
        if (c[i] != kSent) pend |= 1u << i;
    }
    if constexpr (NB) {
        // The first round branch-free: every key issues its CAS, a padding key on the lane's own
        // dummy word (zero, never kSent: the CAS fails and writes nothing; one word per lane, so no
        // two lanes of an instruction share an address), so the round's CASes issue back to back.
        // With a branch per key the compiler cannot prove a skipped key's last CAS result has landed
        // and waits for all LDS traffic (lgkmcnt(0)) before every CAS. Later rounds, with few keys
        // left, keep the branches (a key no lane needs issues nothing).
        __shared__ uint32_t s_dummy[kWave];
        const uint32_t lane = (uint32_t)lane_id();
        s_dummy[lane] = 0;
        uint32_t prev[N];
#pragma unroll
        for (int i = 0; i < N; ++i) prev[i] = atomicCAS((pend >> i) & 1u ? &keys[sl[i]] : &s_dummy[lane], kSent, c[i]);
#pragma unroll
        for (int i = 0; i < N; ++i)
            if ((pend >> i) & 1u) {
                if (prev[i] == kSent || prev[i] == c[i]) {
                    fresh[i] = prev[i] == kSent;
                    pend &= ~(1u << i);
                } else {
                    sl[i] = (sl[i] + 1) & mask;
                }
            }
    }
    while (__builtin_amdgcn_readfirstlane(__ballot(pend != 0) != 0)) {
        uint32_t prev[N];
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (pend & (1u << i)) prev[i] = atomicCAS(&keys[sl[i]], kSent, c[i]);
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (pend & (1u << i)) {
                if (prev[i] == kSent || prev[i] == c[i]) {
                    fresh[i] = prev[i] == kSent;
                    pend &= ~(1u << i);
                } else {
                    sl[i] = (sl[i] + 1) & mask;
                }
            }
    }
}

// symbolic: distinct columns of the row = keys this wave inserted
struct HashCount {
    uint32_t *keys;
    uint32_t cnt = 0, nprod = 0;
    template <int Q>
    __device__ __forceinline__ void run(const uint4 *c) {
        uint32_t cc[4 * Q], sl[4 * Q];
        bool fresh[4 * Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            cc[4 * q] = c[q].x;
            cc[4 * q + 1] = c[q].y;
            cc[4 * q + 2] = c[q].z;
            cc[4 * q + 3] = c[q].w;
        }
        hash_batch<4 * Q>(keys, 10, cc, sl, fresh);  // kSymHashT = 2^10
#pragma unroll
        for (int i = 0; i < 4 * Q; ++i) {
            cnt += fresh[i] ? 1u : 0u;
            nprod += cc[i] != kSent ? 1u : 0u;
        }
    }
    __device__ __forceinline__ void operator()(uint4 c, const Quad<uint32_t> &) { run<1>(&c); }
    // one quad (4 columns) per probe batch: wider batches cost more registers than they save
    __device__ __forceinline__ void multi(const uint4 *c, const Quad<uint32_t> *) {
        sfor<kRegQ>([&](auto Q) { run<1>(c + Q); });
    }
};

// numeric: products into the slots of their columns (Sem::acc: atomics for the integer
// semirings, a plain add for f64, whose ordered walk never has two lanes on one column)
template <typename Sem>
struct HashAcc {
    using S = typename Sem::S;
    uint32_t *keys;
    typename Sem::V *vals;
    template <int Q>
    __device__ __forceinline__ void run(const uint4 *c, const Quad<S> *pr) {
        uint32_t cc[4 * Q], sl[4 * Q];
        bool fresh[4 * Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            cc[4 * q] = c[q].x;
            cc[4 * q + 1] = c[q].y;
            cc[4 * q + 2] = c[q].z;
            cc[4 * q + 3] = c[q].w;
        }
        hash_batch<4 * Q, true>(keys, 9, cc, sl, fresh);  // kHashT = 2^9
#pragma unroll
        for (int i = 0; i < 4 * Q; ++i)
            if (cc[i] != kSent) Sem::acc(vals, sl[i], pr[i / 4].v[i % 4]);
    }
    __device__ __forceinline__ void put(uint32_t c, S pr) {
        uint32_t cc[1] = {c}, sl[1];
        bool fresh[1];
        hash_batch<1, true>(keys, 9, cc, sl, fresh);
        if (c != kSent) Sem::acc(vals, sl[0], pr);
    }
    __device__ __forceinline__ void operator()(uint4 c, const Quad<S> &pr) { run<1>(&c, &pr); }
    __device__ __forceinline__ void multi(const uint4 *c, const Quad<S> *pr) {
        sfor<kRegQ>([&](auto Q) { run<1>(c + Q, pr + Q); });
    }
};

// Per-wave LDS of the numeric hash path: keys u32[kHashT] | vals V[kHashT * kSlots] | stage
// u32[kHashT / 2 + 4] (the row's keys, compacted, padded with kSent for 16-byte reads)
template <typename Sem>
__host__ __device__ constexpr uint32_t hash_bytes() {
    return kHashT * 4 + kHashT * (uint32_t)sizeof(typename Sem::V) * Sem::kSlots + ExtraWords<Sem>::value * 4 +
           (kHashT / 2 + 4) * 4;
}

// ------------------------------------------------------------------------------------------------
// numeric: one wavefront per row
// ------------------------------------------------------------------------------------------------
struct NumLayout {
    uint32_t off_slots, bytes;
};

// Per-wave LDS region: W (ww+1)*8 (uint2 per bitmap word: .x column bits, .y rank of the word's
// first column, so a rank lookup is ONE ds_read_b64; W[ww] = {0, 2^31} catches every column outside
// the window, whose rank then fails the chunk test) | rank slots `area` bytes: values, then u16
// column offsets within the window
__host__ __device__ inline NumLayout num_layout(uint32_t ww, uint32_t area) {
    auto up = [](uint32_t x, uint32_t a) { return (x + a - 1) / a * a; };
    NumLayout L;
    L.off_slots = up((ww + 1) * 8, 16);  // + W[ww]: the dummy word of out-of-window columns
    L.bytes = up(L.off_slots + area, 16);
    return L;
}

// rank (within chunk [r0, r0 + nch)) of column c, or kSent. The word index is clamped to the dummy
// word W[ww] (no bits, base 2^31) instead of tested: out-of-window and padding columns read it and
// fail the chunk test. The LDS read happens for every lane, so a batch issues all its lookups
// before it waits on any.
__device__ __forceinline__ uint2 rank_word(const uint2 *W, uint32_t ww, uint32_t c, uint32_t wlo, uint32_t &off) {
    off = c - wlo;
    return W[min(off >> 5, ww)];
}
__device__ __forceinline__ uint32_t rank_in(uint2 w, uint32_t off, uint32_t r0, uint32_t nch) {
    // popc of the word's bits below the column (v_bfe masks the width to 5 bits) plus the word's rank
    const uint32_t rk = __builtin_popcount(__builtin_amdgcn_ubfe(w.x, 0u, off)) + (w.y - r0);
    return rk < nch ? rk : kSent;
}


template <typename S>
__device__ __forceinline__ S permute_val(int dst, S v) {
    if constexpr (sizeof(S) == 4) {
        return __builtin_bit_cast(S, __builtin_amdgcn_ds_permute(dst, __builtin_bit_cast(int, v)));
    } else {
        const uint64_t u = __builtin_bit_cast(uint64_t, v);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(uint32_t)u);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(uint32_t)(u >> 32));
        return __builtin_bit_cast(S, ((uint64_t)hi << 32) | lo);
    }
}

// materialise v in VGPRs here (an empty asm consuming it): stops the compiler from sinking the
// load that produces v into a later conditional block
template <typename T>
__device__ __forceinline__ void pin(T &v) {
    if constexpr (sizeof(T) == 4) {
        asm volatile("" : "+v"(v));
    } else {
        uint64_t u = __builtin_bit_cast(uint64_t, v);
        uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
        asm volatile("" : "+v"(lo), "+v"(hi));
        v = __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
    }
}

// Compaction of per-lane work items (k, a) into full 64-lane batches with ds_permute: the lanes
// that hold an item send it to consecutive lanes of the batch; a full batch is handed to `run`
// (every lane one item, kSent = none). Masked-off lanes cost an LDS instruction nearly as much as
// active ones, so ragged tails are processed dense.
template <typename S>
struct TailBatch {
    uint32_t filled = 0, bk = kSent;
    S ba = S(0);
    template <typename F>
    __device__ __forceinline__ void add(bool has, uint32_t k, S a, F &&run) {
        const int lane = lane_id();
        unsigned long long m = __ballot(has);
        while (m) {
            const uint32_t n = __popcll(m);
            const uint32_t taken = min(n, (uint32_t)kWave - filled);
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const uint32_t pos = filled + below;
            const bool go = has && pos < filled + taken;
            // senders write to consecutive receiving lanes; the rest to a lane outside the
            // receiving range (there is one whenever any lane is not sending)
            const int dst = (int)((go ? pos : ((filled + taken) & (kWave - 1))) * 4);
            const uint32_t rk = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)k);
            const S ra = permute_val(dst, a);
            if ((uint32_t)lane >= filled && (uint32_t)lane < filled + taken) {
                bk = rk;
                ba = ra;
            }
            filled += taken;
            has = has && !go;
            m = __ballot(has);
            if (filled == kWave) {
                run(bk, ba);
                filled = 0;
                bk = kSent;
            }
        }
    }
    template <typename F>
    __device__ __forceinline__ void flush(F &&run) {
        if (filled) run(bk, ba);
        filled = 0;
        bk = kSent;
    }
};

// Every compacted tail batch (ELL groups t >= 1 of the A entries the lanes hold), in a fixed order:
// fn(bi, c4, pr4) for the batches bi with want(bi); returns the number of batches.
template <typename Sem, bool VALS, typename Wt, typename F>
__device__ __forceinline__ uint32_t for_tails(const Args &p, const uint32_t *kq, const typename Sem::S *aq,
                                              const uint32_t *ngq, uint32_t mx, Wt &&want, F &&fn) {
    using S = typename Sem::S;
    uint32_t bi = 0;
    for (uint32_t t = 1; t < mx; ++t) {
        TailBatch<S> tb;
        auto run = [&](uint32_t k, S a) {
            if (want(bi)) {
                uint4 c = make_uint4(kSent, kSent, kSent, kSent);
                Quad<S> pr{};
                if (k != kSent) {
                    c = ell_cols(p, k, t);
                    if constexpr (VALS) pr = prods<Sem>(a, ell_vals<S>(p, k, t));
                }
                fn(bi, c, pr);
            }
            ++bi;
        };
#pragma unroll
        for (int q = 0; q < kRegQ; ++q) tb.add(ngq[q] > t, kq[q], aq[q], run);
        tb.flush(run);
    }
    return bi;
}

// ------------------------------------------------------------------------------------------------
// RowWalker: every group (4 B entries as columns + products) of one row of A·B, for one wave.
// A entries are taken in segments of 64*kRegQ held by the lanes (kq/aq). With the ELL copy of B,
// a segment's later groups (entry, t >= 1) of ALL rounds are compacted with ds_permute into at
// most kNB dense 64-lane batches of (B row, group, a) kept in registers, so a pass issues all of a
// segment's group loads at once (one L2 round trip) and masked-off lanes do not burn LDS
// instructions. One-segment rows keep their segment across passes; longer rows rebuild it per pass.
// Loads sit bare inside their branches and all arithmetic on them comes after: a use inside the
// branch would make the wave wait there and serialise the loads.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kNB = 2;  // compacted tail batches per segment (bk0/bk1)

template <typename Sem, typename I, bool ELL, bool AVALS>
struct RowWalker {
    using S = typename Sem::S;
    static constexpr uint32_t kSeg = kWave * kRegQ;
    static constexpr uint32_t kOvf = 0xFFFFFFFFu;  // segment with more tail items than kNB batches
    const Args &p;
    I a0, a1;
    uint64_t len;
    uint32_t nseg;
    bool single;
    uint32_t kq[kRegQ], ngq[kRegQ];
    S aq[kRegQ];
    uint32_t bk0 = kSent, bk1 = kSent, bt0 = 0, bt1 = 0, nb = 0;
    S ba0 = S(0), ba1 = S(0);
    uint32_t amax = 0;  // lane max of the A values seen (narrow-slot bound, u32)
    uint32_t sg0 = 0, sg1 = 0;  // CSR B: walk only column chunks [sg0, sg1) of each B row (p.wsplit)

    __device__ __forceinline__ RowWalker(const Args &p_, I a0_, I a1_) : p(p_), a0(a0_), a1(a1_) {
        len = (uint64_t)(a1 - a0);
        nseg = (uint32_t)((len + kSeg - 1) / kSeg);
        single = nseg == 1;
        if (single) load_seg(a0);
    }
    // the A entries [sb, min(a1, sb + kSeg)) of a row, kRegQ per lane (kSent / 0 past the end)
    __device__ static __forceinline__ void seg_loads(const Args &p, I sb, I a1, uint32_t *k, S *a) {
        const int lane = lane_id();
        const S *av_ = (const S *)p.a_val;
        // wave-uniform segment base + a 32-bit lane offset (SGPR-base addressing, no 64-bit math)
        const uint32_t *seg_c = p.a_col + sb;
        const S *seg_v = av_ + sb;
        const uint32_t seg_n = (uint32_t)min<uint64_t>((uint64_t)(a1 - sb), kSeg);
        sfor<kRegQ>([&](auto Q) {
            constexpr int q = Q;
            const uint32_t j = (uint32_t)(q * kWave + lane);
            k[q] = kSent;
            a[q] = S(0);
            if (j < seg_n) {
                k[q] = seg_c[j];
                if constexpr (AVALS) a[q] = seg_v[j];
            }
        });
    }

    __device__ __forceinline__ void load_seg(I sb) {
        seg_loads(p, sb, a1, kq, aq);
        finish_seg();
    }

    // group counts and the compacted tail batches of the segment in kq / aq
    __device__ __forceinline__ void finish_seg() {
        const int lane = lane_id();
        sfor<kRegQ>([&](auto Q) {
            if (kq[Q] >= p.b_nrows) kq[Q] = kSent;  // malformed input: ignore the entry
            if constexpr (Sem::kNarrowable) amax = max(amax, sat32(aq[Q]));
        });
        if constexpr (!ELL) return;
        uint32_t mx = 0;
        sfor<kRegQ>([&](auto Q) {
            constexpr int q = Q;
            ngq[q] = kq[q] != kSent ? p.ell_ng[kq[q]] : 0u;
            mx = max(mx, ngq[q]);
        });
        mx = wave_max_u32(mx);
        bk0 = bk1 = kSent;
        uint32_t off = 0;  // items placed so far (uniform)
        for (uint32_t t = 1; t < mx; ++t) {
            sfor<kRegQ>([&](auto Q) {
                constexpr int q = Q;
                const bool has = ngq[q] > t;
                const unsigned long long m = __ballot(has);
                const uint32_t cnt = __popcll(m);
                if (cnt == 0) return;
                const uint32_t below =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                // senders go to lanes (off + rank) mod 64; the rest to a lane outside that range
                // (one exists unless all 64 lanes send)
                const int dst = (int)(((has ? off + below : off + cnt) & (kWave - 1)) * 4);
                const uint32_t rk = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)kq[q]);
                const S ra = AVALS ? permute_val(dst, aq[q]) : S(0);
                const uint32_t i = ((uint32_t)lane - off) & (kWave - 1);  // receive slot
                const uint32_t g = off + i;                              // item index -> batch g / 64
                // value selects, not conditional stores: keeps the batch registers in VGPRs
                const bool in0 = (i < cnt) & (g < (uint32_t)kWave);
                const bool in1 = (i < cnt) & (g >= (uint32_t)kWave) & (g < 2u * kWave);
                bk0 = in0 ? rk : bk0;
                ba0 = in0 ? ra : ba0;
                bt0 = in0 ? t : bt0;
                bk1 = in1 ? rk : bk1;
                ba1 = in1 ? ra : ba1;
                bt1 = in1 ? t : bt1;
                off += cnt;
            });
        }
        nb = (off + kWave - 1) / kWave;
        if (nb > kNB) nb = kOvf;
    }

    // grp(c4, pr4) / grp.multi(c4[kRegQ], pr4[kRegQ]) for every group; products (PSem) when VV.
    // UNI: every B value equals v0 (a pattern B), so no B values are loaded and an entry's four
    // products are the one value prod(a, v0)
    template <bool VV, typename PSem = Sem, bool UNI = false, typename G>
    __device__ __forceinline__ void each_group(G &grp, S v0 = S(0)) {
        if constexpr (ELL) {
            for (uint32_t sg = 0; sg < nseg; ++sg) {
                if (!single) load_seg(a0 + (I)((uint64_t)sg * kSeg));
                if (nb == kOvf) {  // rare: too many tail items for the register batches
                    sfor<kRegQ>([&](auto Q) {
                        if (kq[Q] != kSent) walk_brow<Sem, true, VV, I>(p, kq[Q], aq[Q], 0, grp);
                    });
                    continue;
                }
                uint4 cq[kRegQ], ct0 = make_uint4(kSent, kSent, kSent, kSent), ct1 = ct0;
                Quad<S> pq[kRegQ], pt0{}, pt1{};
                sfor<kRegQ>([&](auto Q) {
                    constexpr int q = Q;
                    cq[q] = make_uint4(kSent, kSent, kSent, kSent);
                    pq[q] = Quad<S>{};
                    if (kq[q] != kSent) {
                        cq[q] = ell_cols(p, kq[q], 0);
                        if constexpr (VV && !UNI) pq[q] = ell_vals<S>(p, kq[q], 0);
                    }
                });
                if (bk0 != kSent) {
                    ct0 = ell_cols(p, bk0, bt0);
                    if constexpr (VV && !UNI) pt0 = ell_vals<S>(p, bk0, bt0);
                }
                if (bk1 != kSent) {
                    ct1 = ell_cols(p, bk1, bt1);
                    if constexpr (VV && !UNI) pt1 = ell_vals<S>(p, bk1, bt1);
                }
                if constexpr (VV && UNI) {
                    sfor<kRegQ>([&](auto Q) { pq[Q] = splat4(PSem::prod(aq[Q], v0)); });
                    pt0 = splat4(PSem::prod(ba0, v0));
                    pt1 = splat4(PSem::prod(ba1, v0));
                } else if constexpr (VV) {
                    sfor<kRegQ>([&](auto Q) { pq[Q] = prods<PSem>(aq[Q], pq[Q]); });
                    pt0 = prods<PSem>(ba0, pt0);
                    pt1 = prods<PSem>(ba1, pt1);
                }
                grp.multi(cq, pq);
                if (nb > 0) grp(ct0, pt0);
                if (nb > 1) grp(ct1, pt1);
            }
        } else if (single) {
            walk_csr<Sem, VV, I, kRegQ>(p, kq, aq, grp, sg0, sg1);
        } else {
            walk_row<Sem, false, VV, I>(p, a0, a1, grp, sg0, sg1);
        }
    }
};

__device__ __forceinline__ void pin_u64(unsigned long long v) { pin(v); }

// log2 of the chunk width of SpanPass: 32 chunks cover every column
__device__ __forceinline__ uint32_t chunk_shift(uint64_t ncols) {
    uint32_t b = 0;
    while (b < 58 && (ncols - 1) >> (b + 5)) ++b;
    return max(b, 5u);
}

// the windows [wlo, wlo + WIN) of a row spanning [lo, hi]: each next window starts at the first
// touched chunk at or after the previous window's end
template <typename F>
__device__ __forceinline__ void for_windows(uint64_t lo, uint64_t hi, uint32_t WIN, uint32_t cm, uint32_t csh, F &&win) {
    uint64_t wlo = lo & ~31ull;
    while (wlo <= hi) {
        win((uint32_t)wlo);
        const uint64_t e = wlo + WIN;
        if (e > hi) break;
        const uint64_t ce = e >> csh;
        const uint32_t rest = ce >= 32 ? 0u : (cm >> ce);
        if (!rest) break;
        wlo = (rest & 1u) ? e : (ce + (uint64_t)__builtin_ctz(rest)) << csh;
    }
}

// numeric pass 1: column span of the row (rows wider than one window)
// plus the mask of touched column chunks (32 chunks of 2^csh columns), so the windows skip the
// empty stretches of a row whose columns wrap around (a torus row near the boundary)
template <typename S, bool CHUNKS = false>
struct SpanPass {
    uint32_t csh;
    uint32_t l = 0xFFFFFFFFu, h = 0, cm = 0;
    __device__ __forceinline__ void operator()(uint4 c, const Quad<S> &) {
        const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (cc[e] != kSent) {
                l = min(l, cc[e]);
                h = max(h, cc[e]);
                if constexpr (CHUNKS) cm |= 1u << ((cc[e] >> csh) & 31);
            }
    }
    __device__ __forceinline__ void multi(const uint4 *c, const Quad<S> *pr) {
        sfor<kRegQ>([&](auto Q) { (*this)(c[Q], pr[Q]); });
    }
};

// the window's column bitmap: word w at L0[w * STRIDE] (numeric: W[w].x, STRIDE 2; symbolic: 1),
// fire-and-forget LDS atomics. Z: the window starts at column 0 (one window covers every column).
template <typename S, int STRIDE = 2, bool Z = false>
struct BitmapPass {
    uint32_t *L0;
    uint32_t wlo, WIN;
    uint32_t blk = 0;  // lane's mask of touched 64-word blocks (2048 columns each)
    __device__ __forceinline__ void operator()(uint4 c, const Quad<S> &) {
        const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            uint32_t off;
            if (win_off(cc[e], Z ? 0u : wlo, WIN, off)) {
                atomicOr(&L0[(off >> 5) * STRIDE], 1u << (off & 31));
                blk |= 1u << (off >> 11);
            }
        }
    }
    __device__ __forceinline__ void multi(const uint4 *c, const Quad<S> *pr) {
        sfor<kRegQ>([&](auto Q) { (*this)(c[Q], pr[Q]); });
    }
};

// numeric pass 3: accumulate products into rank slots; all rank lookups of a batch first.
// NARROW: u32 value slots (the row provably cannot reach 2^32), else the semiring's V slots.
// Z: the window starts at column 0; R0: the chunk starts at rank 0 (the window's ranks fit one
// chunk); UNI: a group's four products are one value (pattern B). Each drops per-slot VALU work.
template <typename Sem, bool NARROW, bool Z = false, bool R0 = false, bool UNI = false>
struct AccPass {
    using S = typename Sem::S;
    const uint2 *W;
    void *vals;
    uint16_t *cols;  // column offset within the window
    uint32_t ww, wlo, r0, nch;
    PhaseClock *pc;
    template <int Q>
    __device__ __forceinline__ void run(const uint4 *c, const Quad<S> *pr_in) {
        uint2 w[Q][4];
        uint32_t off[Q][4];
        S pr[Q][4];
        // products pinned in VGPRs up front: keeps B-value loads out of the per-slot branches
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            S u = pr_in[q].v[0];
            if constexpr (UNI) pin(u);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                pr[q][e] = UNI ? u : pr_in[q].v[e];
                if constexpr (!UNI) pin(pr[q][e]);
            }
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t cc[4] = {c[q].x, c[q].y, c[q].z, c[q].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) w[q][e] = rank_word(W, ww, cc[e], Z ? 0u : wlo, off[q][e]);
        }
        if constexpr (SLAT_PHASES) {
            pin(w[0][0].x);
            pc->mark(10);  // rank reads
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t r = rank_in(w[q][e], off[q][e], R0 ? 0u : r0, nch);
                if (r != kSent) {
                    if constexpr (NARROW)
                        atomicAdd((uint32_t *)vals + r, (uint32_t)pr[q][e]);
                    else
                        Sem::acc((typename Sem::V *)vals, r, pr[q][e]);
                    cols[r] = (uint16_t)off[q][e];
                }
            }
        }
        if constexpr (SLAT_PHASES) pc->mark(11);  // atomics issued
    }
    __device__ __forceinline__ void operator()(uint4 c, const Quad<S> &pr) { run<1>(&c, &pr); }
    // several groups' rank lookups issued before any is used: one LDS round trip per kAccQ groups
    // instead of per group. 4 for 32-bit values (headline numeric 89.7 -> 87.6 us), 2 for 64-bit ones
    // (4 took the Sat64 instance 103 -> 141 us), profiles/r03_ab_eu_sp8_aq.txt
    static constexpr int kAccQ = sizeof(S) == 4 ? SLAT_ACC_Q : 2;
    __device__ __forceinline__ void multi(const uint4 *c, const Quad<S> *pr) {
        static_assert(kRegQ % kAccQ == 0, "kAccQ divides kRegQ");
        sfor<kRegQ / kAccQ>([&](auto Q) { run<kAccQ>(c + Q * kAccQ, pr + Q * kAccQ); });
    }
};

// accumulate straight into the row's C slice (kGlobalOverflow semirings, rows beyond the LDS
// slots): global atomic add at out + rank, the column stored alongside (duplicates store the same)
template <typename Sem>
struct GlobalAcc {
    using S = typename Sem::S;
    const uint2 *W;
    uint32_t ww, wlo, nrank;
    uint32_t *oc;
    S *ov;
    __device__ __forceinline__ void operator()(uint4 c, const Quad<S> &pr) {
        const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            uint32_t off;
            const uint2 w = rank_word(W, ww, cc[e], wlo, off);
            const uint32_t r = rank_in(w, off, 0u, nrank);
            if (r != kSent) {
                atomicAdd(&ov[r], pr.v[e]);
                oc[r] = wlo + off;
            }
        }
    }
    __device__ __forceinline__ void multi(const uint4 *c, const Quad<S> *pr) {
        sfor<kRegQ>([&](auto Q) { (*this)(c[Q], pr[Q]); });
    }
};

// ------------------------------------------------------------------------------------------------
// symbolic: structural nnz per output row, one wavefront per row (the RowWalker traversal, column
// bitmap only; counts = popcounts of the lane-owned words, which the same lanes then clear)
// ------------------------------------------------------------------------------------------------
template <int STRIDE, bool Z = false>
struct SymPass {
    BitmapPass<uint32_t, STRIDE, Z> bm;
    bool count;
    uint32_t nprod = 0;
    __device__ __forceinline__ void operator()(uint4 c, const Quad<uint32_t> &pr) {
        bm(c, pr);
        if (count) nprod += (c.x != kSent) + (c.y != kSent) + (c.z != kSent) + (c.w != kSent);
    }
    __device__ __forceinline__ void multi(const uint4 *c, const Quad<uint32_t> *pr) {
        sfor<kRegQ>([&](auto Q) { (*this)(c[Q], pr[Q]); });
    }
};

// MODE 0: every row by bitmap windows. Wide launches split the rows in two launches by the
// MAGNUS-style category (a uniform test on the row: len(A row) * max row of B <= 0.7 kSymHashT):
// MODE 1 counts the short rows in the LDS hash table and skips the rest, MODE 2 the converse.
__host__ __device__ constexpr bool sym_short_row(uint64_t len, uint32_t b_maxrow) {
    return len * b_maxrow <= kSymHashT * 7 / 10;
}

// The structural nnz of one output row (symbolic, one wavefront; MODE as in k_symbolic), or kNoRow
// when the row belongs to the other launch of its category. L0: the wave's LDS words (zero / kSent).
constexpr uint64_t kNoRow = ~0ull;
template <typename I, bool ELL, int MODE>
__device__ __forceinline__ uint64_t sym_row(const Args &p, uint64_t row, bool listed, uint32_t *L0,
                                            unsigned long long &flops, bool have = false, uint64_t pa0 = 0,
                                            uint64_t pa1 = 0) {
    const int lane = lane_id();
    const uint32_t WIN = p.ww * 32;
    const I a0 = have ? (I)pa0 : (I)p.a_rp[row], a1 = have ? (I)pa1 : (I)p.a_rp[row + 1];
    if constexpr (MODE != 0) {
        if (!listed && sym_short_row((uint64_t)(a1 - a0), p.b_maxrow) != (MODE == 1)) return kNoRow;  // the other launch's row
    }
    uint64_t cnt = 0;
    if constexpr (MODE == 1) {
        if (a1 > a0) {
            // short row: distinct columns = keys inserted into the wave's hash table
            RowWalker<SemNone, I, ELL, false> rw(p, a0, a1);
            HashCount hc{L0};
            rw.template each_group<false>(hc);
            wave_sync();
            cnt = wave_sum_u32(hc.cnt);
            if (p.stats) flops += wave_sum_u32(hc.nprod);
            uint4 *k4 = (uint4 *)L0;
            for (uint32_t w = lane; w < kSymHashT / 4; w += kWave) k4[w] = make_uint4(kSent, kSent, kSent, kSent);
            wave_sync();
        }
    } else if (a1 > a0) {
        RowWalker<SemNone, I, ELL, false> rw(p, a0, a1);
        uint64_t lo = 0, hi = p.ncols - 1;
        uint32_t cmask = 0xFFFFFFFFu;  // touched column chunks (MODE 2 only; else all)
        const uint32_t csh = MODE == 2 ? chunk_shift(p.ncols) : 0u;
        if (p.wide) {
            SpanPass<uint32_t, MODE == 2> mm{csh};
            rw.template each_group<false>(mm);
            const uint32_t l = wave_min_u32(mm.l), h = wave_max_u32(mm.h);
            if constexpr (MODE == 2) cmask = wave_or_u32(mm.cm);
            lo = l;
            hi = h;
            if (l > h) {
                lo = 1;
                hi = 0;
            }
        }
        bool first = true;
        // one window; Z (std::true_type) when it starts at column 0 and covers every column
        auto window = [&](auto ztag, uint32_t wlo) {
            constexpr bool Z = decltype(ztag)::value;
            SymPass<1, Z> sp{BitmapPass<uint32_t, 1, Z>{L0, wlo, WIN}, p.stats != 0 && first};
            if (!(p.ablate & 1u)) rw.template each_group<false>(sp);
            wave_sync();
            // count = popcount of the touched 64-word blocks only (word b*64 + lane per lane),
            // which the same lanes then clear
            uint32_t lc = 0;
            uint32_t *keep = nullptr;  // the stored bitmap of this row (Z launches with p.sbm)
            const uint32_t bmask = wave_or_u32(sp.bm.blk);
            if constexpr (Z)
                if (p.sbm) {
                    keep = p.sbm + row * ((uint64_t)p.nblk * kWave);
                    if (lane == 0) p.smask[row] = bmask;
                }
            for (uint32_t m = bmask; m; m &= m - 1) {
                const uint32_t w = (uint32_t)__builtin_ctz(m) * kWave + lane;
                const uint32_t x = L0[w];
                lc += __popc(x);
                L0[w] = 0;
                if (keep) keep[w] = x;
            }
            cnt += wave_sum_u32(lc);
            if (first && p.stats) flops += wave_sum_u32(sp.nprod);
            first = false;
            wave_sync();
        };
        if (!p.wide) {
            window(std::true_type{}, 0u);
        } else if constexpr (MODE == 2) {
            for_windows(lo, hi, WIN, cmask, csh, [&](uint32_t wlo) {
                // CSR B bucketed by chunk: the window walks only its chunks' part of each B row
                if (!ELL && p.wsplit) {
                    rw.sg0 = wlo >> csh;
                    rw.sg1 = (uint32_t)min<uint64_t>(p.wnch1 - 1, (((uint64_t)wlo + WIN - 1) >> csh) + 1);
                }
                window(std::false_type{}, wlo);
            });
        } else {
            for (uint64_t wlo = lo & ~31ull; wlo <= hi; wlo += WIN) window(std::false_type{}, (uint32_t)wlo);
        }
    }
    return cnt;
}

}  // namespace slat
#include "spgemm_stored.hpp"
namespace slat {

// variant builds: -DSLAT_SYM_WPE=w caps k_symbolic's registers for w waves per SIMD (0: no cap)
#ifndef SLAT_SYM_WPE
#define SLAT_SYM_WPE 0
#endif
template <typename I, bool ELL, int MODE = 0>
__global__ __launch_bounds__(kBlock)
#if SLAT_SYM_WPE
__attribute__((amdgpu_waves_per_eu(SLAT_SYM_WPE)))
#endif
void k_symbolic(Args p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    constexpr int kWpb = kBlock / kWave;
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);  // wave-uniform: row math in SGPRs
    // per-wave words: the window bitmap, or (MODE 1) the hash keys
    // (MODE 4 lays its regions out itself: sym_stored_words)
    const uint32_t region_w = MODE == 1 ? kSymHashT : MODE == 4 ? 0u : p.ww;
    uint32_t *L0 = smem + (size_t)wv * region_w;
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) p.c_rp[0] = 0;
        if (threadIdx.x < kShards) {  // fields read by k_numeric; [3] (flops) is zeroed by the host
            p.shards[threadIdx.x * kShardStride + 1] = 0;
            p.shards[threadIdx.x * kShardStride + 2] = 0;
        }
    }
    // the block's max row count (p.bmax): LDS max of the waves' maxima; the last wave to finish
    // stores it (no block barrier at the end, no global atomics on one word)
    __shared__ uint32_t s_bmax, s_bdone;
    if (p.bmax) {
        if (threadIdx.x == 0) s_bmax = s_bdone = 0;
        __syncthreads();
    }
    const bool listed = MODE == 2 && p.list != nullptr;  // rows of this category, listed by k_symbolic_short
    const uint64_t nit = listed ? list_len(p) : p.nrows;
    // a wave with no listed row leaves before touching LDS (C4 lists none: the launch is then
    // only its dispatch)
    if (listed && !p.bmax && (uint64_t)blockIdx.x * kWpb + wv >= nit) return;
    for (uint32_t w = lane; w < region_w; w += kWave) L0[w] = MODE == 1 ? kSent : 0u;
    wave_sync();
    unsigned long long flops = 0;
    uint64_t mx = 0;  // max row count (p.bmax)
    const uint64_t stride = (uint64_t)gridDim.x * kWpb;
    // tickets only in the wide launches' passes (MODE 1 / 2): the code costs the single-window
    // instance 18 VGPRs even unused
    const bool dyn = MODE != 0 && p.tq != nullptr;  // launch-uniform
    const TicketQueue tq(p.tq, nit, stride);
    unsigned long long pend = 0;
    // (SLAT_SYM_PREFETCH, single-window passes) the next row's bounds loaded by lanes 0-1 ahead
    constexpr bool kPre = SLAT_SYM_PREFETCH && MODE == 0;
    uint64_t pre = 0;
    auto prefetch = [&](uint64_t r) {
        if constexpr (kPre)
            if (r < nit && lane < 2) pre = p.a_rp[r + lane];
    };
    if constexpr (MODE == 4) {
        symbolic_rows_stored<I>(p, smem, wv, (uint64_t)blockIdx.x * kWpb + wv, stride, mx, flops);
    } else {
    prefetch((uint64_t)blockIdx.x * kWpb + wv);
    for (uint64_t it = (uint64_t)blockIdx.x * kWpb + wv; it < nit; it = dyn ? tq.resolve(pend) : it + stride) {
        if (dyn) pend = tq.issue();
        const uint64_t row = listed ? (uint64_t)__builtin_amdgcn_readfirstlane(p.list[it]) : it;
        uint64_t pa0 = 0, pa1 = 0;
        if constexpr (kPre) {
            pa0 = readlane_u64(pre, 0);
            pa1 = readlane_u64(pre, 1);
            prefetch(it + stride);
        }
        if (fat_row(p, row)) continue;  // the fat-row kernels' row
        const uint64_t cnt = sym_row<I, ELL, MODE>(p, row, listed, L0, flops, kPre, pa0, pa1);
        if (cnt == kNoRow) continue;
        if (lane == 0) p.counts[row] = cnt;
        mx = max(mx, cnt);
    }
    }
    if (p.stats && lane == 0 && flops)
        atomicAdd(&p.shards[((blockIdx.x * kWpb + wv) % kShards) * kShardStride + 3], flops);
    if (p.bmax && lane == 0) {
        atomicMax(&s_bmax, (uint32_t)(mx < 0xFFFFFFFFull ? mx : 0xFFFFFFFFull));
        if (atomicAdd(&s_bdone, 1u) == (uint32_t)kWpb - 1) p.bmax[blockIdx.x] = atomicMax(&s_bmax, 0u);
    }
}

// k_numeric's register cap: 3 waves per SIMD (<= 168 VGPRs). The wide-slot (Sat64 / f64) and
// narrow instances spill nothing at that cap and gain the third wave: Sat64 A^6*A numeric
// 146 -> 117 us, u32 unchanged (profiles/r03_ab_sat64_narrow.txt, variant "w3"). At 4 waves (128
// VGPRs) round 2 saw a memory fault; it came from that build's uncommitted compacted-bitmap code,
// not from the cap. Variant builds: -DSLAT_NUM_WPE=w.
#ifndef SLAT_NUM_WPE
#define SLAT_NUM_WPE 3
#endif
#define SLAT_NUM_ATTR __attribute__((amdgpu_waves_per_eu(SLAT_NUM_WPE)))

// MODE 0: every row by bitmap windows. Wide launches split the rows by output count (known from
// symbolic): MODE 1 accumulates the rows with <= kHashT / 2 outputs in the LDS hash table and
// skips the rest, MODE 2 takes the rest by row-span windows.
// The numeric pass of one wavefront over rows first, first + stride, ... (k_numeric: the grid's
// waves; p.tq: from a ticket queue instead). smem8: the workgroup's LDS, wave wv's region at wv * its
// size.
template <typename Sem, typename I, bool ELL, int MODE>
__device__ __forceinline__ void numeric_rows(const Args &p, uint8_t *smem8, int wv, uint64_t first, uint64_t stride) {
    using S = typename Sem::S;
    using V = typename Sem::V;
    constexpr int kWpb = kBlock / kWave;
    constexpr bool kVals = !Sem::kOrdered;  // f64 accumulates from an ordered CSR walk

    const int lane = lane_id();
    const bool listed = MODE == 2 && p.list != nullptr;  // rows of this category, listed by k_numeric_short
    const uint64_t nit = listed ? list_len(p) : p.nrows;
    // a wave with no listed row leaves before touching LDS (C4 lists none)
    if (listed && first >= nit) return;
    const NumLayout lay = num_layout(p.ww, p.area);
    // per-wave region: the bitmap window + rank slots, or (wide launches) the hash table in the
    // same place
    const uint32_t region_b = MODE == 1 ? hash_bytes<Sem>() : lay.bytes;
    uint8_t *region = smem8 + (size_t)wv * region_b;
    uint2 *W = (uint2 *)region;
    uint32_t *L0 = (uint32_t *)region;  // L0[2w] aliases W[w].x
    uint8_t *slots = region + lay.off_slots;
    // rank-chunk capacities: narrow = u32 value + u16 column, wide = V*kSlots + u16 column
    const uint32_t cap_n = p.area / 6, cap_w = p.area / (uint32_t)(sizeof(V) * Sem::kSlots + 2);
    uint32_t bvmax = 0xFFFFFFFFu;  // max B value of this call (u32 semiring with the ELL copy)
    bool buni = false;             // every B value equals bvmax (a pattern B)
    if constexpr (Sem::kNarrowable)
        if (p.b_vmax) {
            const unsigned long long v = ((volatile unsigned long long *)p.b_vmax)[kVMaxWord];
            const unsigned long long vi = ((volatile unsigned long long *)p.b_vmax)[kVMinInvWord];
            if ((uint32_t)(v >> 32) == p.epoch) {
                bvmax = (uint32_t)v;
                // (a wider value type clamps to u32 in the summary: all-equal clamped values are
                // not a pattern unless below the clamp)
                buni = SLAT_NUM_UNI && (uint32_t)(vi >> 32) == p.epoch && ~(uint32_t)vi == bvmax &&
                       (sizeof(S) == 4 || bvmax != 0xFFFFFFFFu);
            }
        }
    const S bv0 = (S)bvmax;
    S *cval = (S *)p.c_val;

    // hash table of the short-row path: keys | values | staged keys
    uint32_t *hkeys = (uint32_t *)region;
    V *hvals = (V *)(region + kHashT * 4);
    uint32_t *hstage = (uint32_t *)(region + kHashT * 4 + kHashT * sizeof(V) * Sem::kSlots);
    if constexpr (MODE == 1) {
        for (uint32_t w = lane; w < kHashT; w += kWave) hkeys[w] = kSent;
        for (uint32_t w = lane; w < kHashT * Sem::kSlots; w += kWave) hvals[w] = V(0);
    } else {
        for (uint32_t w = lane; w < p.ww; w += kWave) W[w] = make_uint2(0u, 0u);
        if (lane == 0) W[p.ww] = make_uint2(0u, 0x80000000u);  // dummy word: never set, never cleared
        for (uint32_t w = lane; w < p.area / 4; w += kWave) ((uint32_t *)slots)[w] = 0;  // emit keeps it zero
    }
    wave_sync();

    const uint32_t WIN = p.ww * 32;
    uint32_t zrows = 0;
    PhaseClock pc{};
    if constexpr (SLAT_PHASES) pc.t = __builtin_amdgcn_s_memtime();
    auto mark = [&](int i) { pc.mark(i); };
    uint64_t *ph = pc.ph;
    using RW = RowWalker<Sem, I, ELL, kVals>;
    const bool dyn = MODE != 0 && p.tq != nullptr;  // launch-uniform (single-window passes: a fixed stride)
    const TicketQueue tq(p.tq, nit, stride);
    unsigned long long pend = 0;
    for (uint64_t it = first; it < nit; it = dyn ? tq.resolve(pend) : it + stride) {
        if (dyn) pend = tq.issue();
        const uint64_t row = listed ? (uint64_t)__builtin_amdgcn_readfirstlane(p.list[it]) : it;
        if (fat_row(p, row)) continue;  // the fat-row kernels' row
        const I a0 = (I)p.a_rp[row], a1 = (I)p.a_rp[row + 1];
        const uint64_t out_begin = p.c_rp[row], out_end = p.c_rp[row + 1];
        uint64_t out_pos = out_begin;
        uint32_t zeros = 0;
        ph[kPhaseSlots - 1] += 1;
        if constexpr (MODE != 0) {
            // the other launch's row (listed rows are this launch's by construction: the sorted
            // short-row category also lists rows with few outputs but > 256 entries or > 64 groups)
            if (!listed && (out_end - out_begin <= kHashT / 2) != (MODE == 1)) continue;
        }
        if constexpr (MODE == 1) {
            // short row (its output count, known from symbolic, fits half the table)
            if (a1 > a0) {
            HashAcc<Sem> ha{hkeys, hvals};
            if constexpr (Sem::kOrdered) {
                traverse_ordered<I, S>(p, a0, a1, [&](uint32_t j, S a, S b) { ha.put(j, Sem::prod(a, b)); });
            } else {
                RowWalker<Sem, I, ELL, kVals> rw(p, a0, a1);
                rw.template each_group<true>(ha);
            }
            wave_sync();
            // the keys each lane holds (slots lane, lane + 64, ...), staged compacted for all lanes
            uint32_t hk[kHashHeld], nh = 0;
            sfor<kHashHeld>([&](auto I_) {
                hk[I_] = hkeys[I_ * kWave + lane];
                nh += hk[I_] != kSent ? 1u : 0u;
            });
            const uint32_t incl = wave_incl_scan(nh, 0u, [](uint32_t x, uint32_t y) { return x + y; });
            const uint32_t tot = readlane_u32(incl, kWave - 1);
            uint32_t at = incl - nh;
            sfor<kHashHeld>([&](auto I_) {
                if (hk[I_] != kSent) hstage[at++] = hk[I_];
            });
            if (lane < 4) hstage[tot + lane] = kSent;  // pad for the 16-byte reads
            wave_sync();
            // rank = number of the row's keys below the held key (all keys distinct)
            uint32_t rk[kHashHeld];
            sfor<kHashHeld>([&](auto I_) { rk[I_] = 0; });
            const uint4 *st4 = (const uint4 *)hstage;
            for (uint32_t b = 0; b < tot; b += 4) {
                const uint4 q = st4[b >> 2];
                sfor<kHashHeld>([&](auto I_) {
                    const uint32_t k = hk[I_];
                    rk[I_] += (q.x < k) + (q.y < k) + (q.z < k) + (q.w < k);
                });
            }
            uint32_t *oc = p.c_col + out_begin;
            S *ov = cval + out_begin;
            const uint64_t lim = out_end - out_begin;
            sfor<kHashHeld>([&](auto I_) {
                if (hk[I_] != kSent) {
                    const uint32_t sl = I_ * kWave + lane;
                    const S v = Sem::finish(hvals, sl);
                    zeros += Sem::is_zero(v) ? 1u : 0u;
                    if (rk[I_] < lim) {  // never write past the row's slice
                        oc[rk[I_]] = hk[I_];
                        ov[rk[I_]] = v;
                    }
                    hkeys[sl] = kSent;  // leave the table clean
#pragma unroll
                    for (int w = 0; w < Sem::kSlots; ++w) hvals[sl * Sem::kSlots + w] = V(0);
                }
            });
            out_pos += tot;
            wave_sync();
            }
        } else if (a1 > a0) {
            RW rw(p, a0, a1);
            const uint64_t len = rw.len;
            if constexpr (SLAT_PHASES) pin(rw.kq[0]);  // wait for the A entries inside phase 0
            mark(0);  // row bounds + A entries, group counts, tail compaction
            auto each_group = [&](auto &&grp, auto vals_tag) { rw.template each_group<decltype(vals_tag)::value>(grp); };
            uint64_t lo = 0, hi = p.ncols - 1;
            uint32_t cmask = 0xFFFFFFFFu;  // touched column chunks (MODE 2 only; else all)
            const uint32_t csh = MODE == 2 ? chunk_shift(p.ncols) : 0u;
            if (p.wide) {
                SpanPass<S, MODE == 2> mm{csh};
                each_group(mm, std::false_type{});
                const uint32_t l = wave_min_u32(mm.l), h = wave_max_u32(mm.h);
                if constexpr (MODE == 2) cmask = wave_or_u32(mm.cm);
                lo = l;
                hi = h;
                if (l > h) {
                    lo = 1;
                    hi = 0;
                }
            }
            // one window: Z (std::true_type) when it starts at column 0 and covers every column
            auto window = [&](auto ztag, uint32_t wlo) {
                constexpr bool Z = decltype(ztag)::value;
                const bool stored = Z && p.sbm != nullptr;  // launch-uniform
                uint32_t bmask, wcnt = 0;
                // a multi-segment row's first 512 A values for the narrow bound below, loaded
                // ahead of its stored bitmap so both loads wait out one memory latency together
                // (nothing has walked the row's later segments yet)
                const bool aearly = SLAT_AEARLY && Sem::kNarrowable && stored && !rw.single && bvmax != 0xFFFFFFFFu;
                S aq8[8];
                if constexpr (Sem::kNarrowable)
                    if (aearly) {
                        const S *av = (const S *)p.a_val;
                        sfor<8>([&](auto I_) {
                            const I j = a0 + (I)lane + (I)(I_ * kWave);
                            aq8[I_] = j < a1 ? av[j] : S(0);
                        });
                    }
                if (stored) {
                    // 1'. the row's bitmap as symbolic left it: touched blocks only, loaded 8 blocks
                    //     at a time, ranked from registers and written whole ({bits, rank} per word),
                    //     so untouched blocks may hold stale words (no valid column reads them) and
                    //     nothing is cleared afterwards
                    bmask = __builtin_amdgcn_readfirstlane(p.smask[row]);
                    const uint32_t *src = p.sbm + row * ((uint64_t)p.nblk * kWave) + lane;
                    uint32_t m = bmask;
                    while (m) {
                        uint32_t bs[8], xs[8];
                        sfor<8>([&](auto I_) {
                            bs[I_] = m ? (uint32_t)__builtin_ctz(m) : 32u;
                            m &= m - 1;
                        });
                        sfor<8>([&](auto I_) {
                            xs[I_] = 0;
                            if (bs[I_] < 32u) xs[I_] = src[bs[I_] * kWave];
                        });
                        sfor<8>([&](auto I_) {
                            if (bs[I_] < 32u) {
                                const uint32_t c = __popc(xs[I_]);
                                const uint32_t incl = wave_incl_scan(c, 0u, [](uint32_t x, uint32_t y) { return x + y; });
                                W[bs[I_] * kWave + lane] = make_uint2(xs[I_], wcnt + incl - c);
                                wcnt += readlane_u32(incl, kWave - 1);
                            }
                        });
                    }
                    wave_sync();
                    mark(1);
                    if (wcnt == 0) return;
                } else {
                    // 1. column bitmap of the window (into W[w].x)
                    BitmapPass<S, 2, Z> bm{L0, wlo, WIN};
                    if (!(p.ablate & 32u)) each_group(bm, std::false_type{});
                    wave_sync();
                    (void)__builtin_amdgcn_readfirstlane(L0[0]);
                    mark(1);  // bitmap pass
                    // 2. word ranks into W[w].y, over the touched 64-word blocks only: block b's words
                    //    are b*64 + lane, a wave scan per block carried across blocks
                    bmask = wave_or_u32(bm.blk);
                    for (uint32_t m = bmask; m; m &= m - 1) {
                        const uint32_t w = (uint32_t)__builtin_ctz(m) * kWave + lane;
                        const uint32_t c = __popc(W[w].x);
                        const uint32_t incl = wave_incl_scan(c, 0u, [](uint32_t x, uint32_t y) { return x + y; });
                        W[w].y = wcnt + incl - c;
                        wcnt += readlane_u32(incl, kWave - 1);
                    }
                    if (wcnt == 0) return;  // bitmap empty: nothing to clear
                }
                mark(2);  // word ranks
                // narrow u32 slots when the row's sums provably stay below 2^32:
                // max(A row) * max(B) * len(A row) < 2^32 (each output sums <= len products)
                bool narrow = false;
                if constexpr (Sem::kNarrowable) {
                    // (rw.amax covers a one-segment row; a longer row reads its A values once more:
                    // with a stored bitmap nothing walked its later segments yet, so its amax would
                    // hold nothing)
                    if (bvmax != 0xFFFFFFFFu) {
                        uint32_t am = rw.amax;
                        if (!rw.single) {
                            I j0 = a0;
                            if (aearly) {
                                sfor<8>([&](auto I_) { am = max(am, sat32(aq8[I_])); });
                                j0 += (I)(8 * kWave);
                            }
                            const S *av = (const S *)p.a_val;
                            for (I j = j0 + (I)lane; j < a1; j += (I)kWave) am = max(am, sat32(av[j]));
                        }
                        const uint32_t wam = wave_max_u32(am);
                        const uint64_t x = (uint64_t)wam * bvmax;
                        // a 64-bit A value of 2^32 or more clamps to 0xFFFFFFFF in sat32: its true
                        // size is unknown, so such a row never narrows (as for B's clamped max)
                        narrow = (sizeof(S) == 4 || wam != 0xFFFFFFFFu) && (x == 0 || len <= 0xFFFFFFFFull / x);
                    }
                }
                // one rank chunk [r0, r0 + nch): zero its slots, accumulate, emit. R0: r0 == 0.
                auto chunk = [&](auto narrow_tag, auto uni_tag, auto r0tag, uint32_t r0, uint32_t cap) {
                    constexpr bool NW = decltype(narrow_tag)::value;
                    constexpr bool UNI = decltype(uni_tag)::value;
                    constexpr bool R0 = decltype(r0tag)::value;
                    using VS = std::conditional_t<NW, uint32_t, V>;  // value slot word
                    constexpr uint32_t kVW = NW ? 1 : Sem::kSlots;   // words per slot
                    VS *vals = (VS *)slots;
                    uint16_t *cols = (uint16_t *)(slots + ((cap * kVW * sizeof(VS) + 3) & ~3u));
                    const uint32_t nch = min(cap, wcnt - r0);
                    // (the slots are zero: the previous chunk's emit cleared what it used)
                    mark(8);
                    // 3. values and the column offset of every rank (duplicates store the same)
                    if constexpr (Sem::kOrdered) {
                        if (!(p.ablate & 8u))
                            traverse_ordered<I, S>(p, a0, a1, [&](uint32_t j, S a, S b) {
                                uint32_t off;
                                const uint2 w = rank_word(W, p.ww, j, wlo, off);
                                const uint32_t r = rank_in(w, off, r0, nch);
                                if (r != kSent) {
                                    Sem::acc((V *)vals, r, Sem::prod(a, b));
                                    cols[r] = (uint16_t)off;
                                }
                            });
                    } else if (!(p.ablate & 8u)) {
                        AccPass<Sem, NW, Z && R0, Z && R0, UNI> acc{W, vals, cols, p.ww, wlo, r0, nch, &pc};
                        using PS = std::conditional_t<NW, SemNarrowT<S>, Sem>;
                        rw.template each_group<true, PS, UNI>(acc, bv0);
                    }
                    wave_sync();
                    if constexpr (SLAT_PHASES) (void)__builtin_amdgcn_readfirstlane((uint32_t)vals[0]);
                    mark(12);  // accumulate pass drain
                    // 4. emit at the row's slice, coalesced
                    // wave-uniform output base + 32-bit lane offsets
                    uint32_t *oc = p.c_col + out_pos;
                    S *ov = cval + out_pos;
                    const uint32_t lim = (uint32_t)min<uint64_t>(out_end - min(out_pos, out_end), nch);
                    for (uint32_t t = lane; t < nch; t += kWave) {
                        S v;
                        if constexpr (NW)
                            v = (S)vals[t];
                        else
                            v = Sem::finish((const V *)vals, t);
                        const uint32_t col = cols[t];
                        // leave the slot area zero for the next chunk (values and column offsets):
                        // no separate zeroing pass before the accumulate
#pragma unroll
                        for (uint32_t w = 0; w < kVW; ++w) vals[t * kVW + w] = VS(0);
                        cols[t] = 0;
                        zeros += Sem::is_zero(v) ? 1u : 0u;
                        if (t < lim && !(p.ablate & 16u)) {  // never write past the row's slice
                            oc[t] = wlo + col;
                            ov[t] = v;
                        }
                    }
                    out_pos += nch;
                    wave_sync();
                    mark(4);  // emit
                };
                auto run_chunks = [&](auto narrow_tag, auto uni_tag) {
                    constexpr bool NW = decltype(narrow_tag)::value;
                    const uint32_t cap = NW ? cap_n : cap_w;
                    // u32 rows under the narrow bound cannot overflow a u32 sum, so their atomics
                    // in C are exact too: no re-traversal per rank chunk for hub rows (B walked in
                    // CSR form; the ELL instances keep their registers: +3 us on the 30^3 bench)
                    constexpr bool kGO = GlobalOverflow<Sem>::value || (Sem::kNarrowable && NW && !ELL);
                    if constexpr (kGO) {
                        if (wcnt > cap) {
                            // one pass into the C slice: zero it, then global atomics at out + rank
                            uint32_t *oc = p.c_col + out_pos;
                            S *ov = cval + out_pos;
                            const uint32_t lim = (uint32_t)min<uint64_t>(out_end - min(out_pos, out_end), wcnt);
                            for (uint32_t t = lane; t < lim; t += kWave) ov[t] = S(0);
                            __builtin_amdgcn_s_waitcnt(0);  // the zeros reach L2 before the atomics
                            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                            GlobalAcc<Sem> ga{W, p.ww, Z ? 0u : wlo, lim, oc, ov};
                            if constexpr (NW)
                                rw.template each_group<true, SemNarrowT<S>, decltype(uni_tag)::value>(ga, bv0);
                            else
                                rw.template each_group<true>(ga);
                            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
                            // zero sums (cancellation) are counted by the compaction test below
                            for (uint32_t t = lane; t < lim; t += kWave) {
                                const S v = __hip_atomic_load(&ov[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                zeros += Sem::is_zero(v) ? 1u : 0u;
                            }
                            out_pos += wcnt;
                            wave_sync();
                            return;
                        }
                    }
                    if (Z && wcnt <= cap) {  // the common case: one chunk from rank 0
                        chunk(narrow_tag, uni_tag, std::true_type{}, 0u, cap);
                    } else {
                        for (uint32_t r0 = 0; r0 < wcnt; r0 += cap) chunk(narrow_tag, uni_tag, std::false_type{}, r0, cap);
                    }
                };
                if constexpr (Sem::kNarrowable && ELL) {
                    if (narrow && buni)
                        run_chunks(std::true_type{}, std::true_type{});
                    else if (narrow)
                        run_chunks(std::true_type{}, std::false_type{});
                    else
                        run_chunks(std::false_type{}, std::false_type{});
                } else if constexpr (Sem::kNarrowable) {  // B in CSR form: values always loaded
                    if (narrow)
                        run_chunks(std::true_type{}, std::false_type{});
                    else
                        run_chunks(std::false_type{}, std::false_type{});
                } else {
                    run_chunks(std::false_type{}, std::false_type{});
                }
                if (!stored) {
                    for (uint32_t m = bmask; m; m &= m - 1) W[(uint32_t)__builtin_ctz(m) * kWave + lane].x = 0;
                    wave_sync();
                }
            };
            if (!p.wide) {
                window(std::true_type{}, 0u);
            } else if constexpr (MODE == 2) {
                for_windows(lo, hi, WIN, cmask, csh, [&](uint32_t wlo) {
                // CSR B bucketed by chunk: the window walks only its chunks' part of each B row
                if (!ELL && p.wsplit) {
                    rw.sg0 = wlo >> csh;
                    rw.sg1 = (uint32_t)min<uint64_t>(p.wnch1 - 1, (((uint64_t)wlo + WIN - 1) >> csh) + 1);
                }
                window(std::false_type{}, wlo);
            });
            } else {
                for (uint64_t wlo64 = lo & ~31ull; wlo64 <= hi; wlo64 += WIN) window(std::false_type{}, (uint32_t)wlo64);
            }
        }
        mark(5);  // window clears, empty rows
        const uint32_t rz = p.ablate ? 0u : wave_sum_u32(zeros);  // ablation runs: no compaction
        const uint64_t got = out_pos - out_begin - rz;
        if (lane == 0) p.counts[row] = got;
        zrows += rz ? 1u : 0u;
    }
    mark(6);  // row tail (counts)
    if constexpr (SLAT_PHASES) {
        if (lane == 0) {
            unsigned long long *dst = p.shards + 512 + ((blockIdx.x * kWpb + wv) % 64) * kPhaseSlots;
            for (int i = 0; i < kPhaseSlots; ++i) atomicAdd(&dst[i], (unsigned long long)ph[i]);
        }
    }
    add_zero_rows(&p.host_out[2], zrows, p.seq != 0);
}

// MODE 4: single-window launches with stored bitmaps and B's ELL image (spgemm_stored.hpp)
template <typename Sem, typename I, bool ELL, int MODE = 0>
__global__ __launch_bounds__(kBlock) SLAT_NUM_ATTR void k_numeric(Args p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    constexpr int kWpb = kBlock / kWave;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);  // wave-uniform: row math in SGPRs
    if constexpr (MODE == 4)
        numeric_rows_stored<Sem, I>(p, smem8, wv, (uint64_t)blockIdx.x * kWpb + wv, (uint64_t)gridDim.x * kWpb);
    else
        numeric_rows<Sem, I, ELL, MODE>(p, smem8, wv, (uint64_t)blockIdx.x * kWpb + wv, (uint64_t)gridDim.x * kWpb);
    signal_done(p);
}

// ------------------------------------------------------------------------------------------------
// Short rows of wide launches, batched (MAGNUS's small-row category, integer semirings, ELL B).
// A wave takes a tile of 64 consecutive rows and packs runs of consecutive short rows into batches
// of <= kHashT / 2 outputs and <= 256 A entries: one hash table holds the whole batch under
// composite keys (local row << cbits | column), so one dependent load chain and one rank pass
// serve several rows, and every lane has work. Rank-by-count over composite keys is the order of
// (row, column), i.e. the offset from the batch's first output: rows are contiguous in C.
// Rows with more outputs belong to the window launch (MODE 2) and are skipped here.
// ------------------------------------------------------------------------------------------------
// append row r of the lanes with `take` to p.list (one atomic per wave)
__device__ __forceinline__ void list_rows(const Args &p, bool take, uint64_t r) {
    if (!p.list) return;
    const unsigned long long m = __ballot(take);
    if (!m) return;
    unsigned int base = 0;
    if (lane_id() == 0) base = atomicAdd(p.list_cnt, (unsigned int)__popcll(m));
    base = __builtin_amdgcn_readfirstlane(base);
    if (take) p.list[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = (uint32_t)r;
    if (p.spec_flag && lane_id() == 0) __hip_atomic_store(p.spec_flag, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}


// Positions of the batch's (A entry, ELL group) pairs in group order: exclusive prefix of the group
// counts over the entries (kRegQ rounds of the wave). Returns the number of groups.
__device__ __forceinline__ uint32_t group_positions(const uint32_t (&ng)[kRegQ], uint32_t (&pos)[kRegQ]) {
    uint32_t tot = 0;
    sfor<kRegQ>([&](auto Q) {
        const uint32_t incl = wave_incl_scan(ng[Q], 0u, [](uint32_t x, uint32_t y) { return x + y; });
        pos[Q] = tot + incl - ng[Q];
        tot += readlane_u32(incl, kWave - 1);
    });
    return tot;
}

// The pairs of group positions [base, base + kStageG) staged one per slot, so the accumulation
// runs one group per lane (every lane busy) instead of one A entry per lane and group index (C4:
// a quarter of the lanes): gk = B row | group << 24 (B rows < 2^24 with the ELL copy), gl = local
// row, ga = A value.
constexpr uint32_t kStageG = 256;
// (CSR: kq = the B row's first entry offset, cnt = its length; ELL: kq = the B row, cnt = its groups)
template <bool VALS, bool CSR, typename S>
__device__ __forceinline__ void stage_groups(uint32_t base, uint32_t mxg, const uint32_t (&kq)[kRegQ],
                                             const uint32_t (&lq)[kRegQ], const uint32_t (&cnt)[kRegQ],
                                             const uint32_t (&pos)[kRegQ], const S (&aq)[kRegQ], uint32_t *gk,
                                             uint8_t *gl, S *ga) {
    for (uint32_t t = 0; t < mxg; ++t)
        sfor<kRegQ>([&](auto Q) {
            const uint32_t g = pos[Q] + t - base;  // wraps past kStageG below base
            if (t < short_groups<CSR>(cnt[Q]) && g < kStageG) {
                if constexpr (CSR) {
                    gk[g] = kq[Q] + 4 * t;
                    gl[g] = (uint8_t)(lq[Q] | ((min(4u, cnt[Q] - 4 * t) - 1) << 6));
                } else {
                    gk[g] = kq[Q] | (t << 24);
                    gl[g] = (uint8_t)lq[Q];
                }
                if constexpr (VALS) ga[g] = aq[Q];
            }
        });
    wave_sync();
}
// a staged group's columns (kSent past its entries) and its local row
template <bool CSR>
__device__ __forceinline__ uint4 staged_cols(const Args &p, uint32_t w, uint32_t glb) {
    if constexpr (CSR)
        return csr_cols(p, w, (glb >> 6) + 1);
    else
        return ell_cols(p, w & 0xFFFFFFu, w >> 24);
}
template <bool CSR, typename S>
__device__ __forceinline__ Quad<S> staged_vals(const Args &p, uint32_t w, uint32_t glb) {
    if constexpr (CSR)
        return csr_vals<S>(p, w, (glb >> 6) + 1);
    else
        return ell_vals<S>(p, w & 0xFFFFFFu, w >> 24);
}

// MAGNUS row categorisation input: the ELL groups of each row of a 64-row tile (lane j: row r0 + j),
// i.e. a product bound of 4 per group, from the tile's entries with coalesced loads: the exclusive
// prefix of the entries' group counts, read at each row's first and end entry (mod 2^32: only rows
// of <= 256 entries use the difference, and the entries of longer rows are skipped, not read).
// pf: u32[256] of LDS, left dirty.
// Rows of more than `jump` entries are jumped over (their bound is never needed: they are long).
template <bool CSR>
__device__ __forceinline__ uint32_t tile_groups(const Args &p, uint64_t A0j, uint64_t A1j, uint32_t nt, uint32_t *pf,
                                                uint64_t jump = 256) {
    const uint32_t lane = (uint32_t)lane_id();
    const uint64_t T0 = readlane_u64(A0j, 0), T1 = readlane_u64(A1j, (int)nt - 1);
    const bool longj = lane < nt && A1j - A0j > jump;
    uint32_t gs = 0, ge = 0, run = 0;
    for (uint64_t c0 = T0; c0 < T1;) {
        const unsigned long long in = __ballot(longj && A0j <= c0 && c0 < A1j);
        if (in) {  // inside a long row: jump to its end
            if (A0j == c0) gs = run;
            if (A1j == c0) ge = run;
            c0 = readlane_u64(A1j, (int)__builtin_ctzll(in));
            continue;
        }
        uint32_t kk[4], g[4];
        sfor<4>([&](auto Q) {
            const uint64_t idx = c0 + Q * kWave + lane;
            kk[Q] = idx < T1 ? p.a_col[idx] : kSent;
        });
        sfor<4>([&](auto Q) { g[Q] = short_groups<CSR>(short_brow<CSR>(p, kk[Q])); });
        sfor<4>([&](auto Q) {
            const uint32_t incl = wave_incl_scan(g[Q], 0u, [](uint32_t x, uint32_t y) { return x + y; });
            pf[Q * kWave + lane] = run + incl - g[Q];
            run += readlane_u32(incl, kWave - 1);
        });
        wave_sync();
        if (A0j >= c0 && A0j < T1 && A0j - c0 < 256) gs = pf[A0j - c0];
        if (A1j >= c0 && A1j < T1 && A1j - c0 < 256) ge = pf[A1j - c0];
        wave_sync();
        c0 += 256;
    }
    if (A0j >= T1) gs = run;
    if (A1j >= T1) ge = run;
    return lane < nt ? ge - gs : 0u;
}

// Symbolic of the short rows of a wide launch, batched like k_numeric_short: tiles of 64 rows,
// runs of consecutive rows with product bound <= 0.7 kSymHashT and <= 256 entries share one
// table of composite keys; a fresh insert counts for its row. Other rows go to p.list.
// LDS per wave: keys u32[kSymHashT] | entry markers u32[256] | row counts u32[64] | staged groups:
// gk u32[kStageG], gl u8[kStageG]
__host__ __device__ constexpr uint32_t sym_short_bytes() { return kSymHashT * 4 + 256 * 4 + kWave * 4 + kStageG * 5; }

template <typename I, bool CSR = false>
__global__ __launch_bounds__(kBlock) void k_symbolic_short(Args p) {
    constexpr int kWpb = kBlock / kWave;
    const uint32_t kCap = p.sym_cap ? p.sym_cap : kSymHashT * SLAT_SYM_CAP_PCT / 100;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    uint32_t *keys = smem + (size_t)wv * (sym_short_bytes() / 4);
    uint32_t *marks = keys + kSymHashT, *rcnt = marks + 256, *gk = rcnt + kWave;
    uint8_t *gl = (uint8_t *)(gk + kStageG);
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            p.c_rp[0] = 0;
            if (p.list_reset) *p.list_reset = 0;  // the numeric list's length (appended to after this kernel)
        }
        if (threadIdx.x < kShards) {
            p.shards[threadIdx.x * kShardStride + 1] = 0;
            p.shards[threadIdx.x * kShardStride + 2] = 0;
        }
    }
    for (uint32_t w = lane; w < kSymHashT; w += kWave) keys[w] = kSent;
    for (uint32_t w = lane; w < 256; w += kWave) marks[w] = 0;
    rcnt[lane] = 0;
    wave_sync();
    const uint32_t cb = p.cbits;
    unsigned long long flops = 0;
    const uint32_t T = p.tile_rows ? p.tile_rows : (uint32_t)kWave;
    const uint64_t ntiles = (p.nrows + T - 1) / T;
    const XcdStride xs(ntiles, kWpb, wv);
    for (uint64_t tile = xs.first; tile < xs.end; tile += xs.stride) {
        const uint64_t r0 = tile * T, r = r0 + lane;
        const uint32_t nt = (uint32_t)min<uint64_t>(T, p.nrows - r0);
        uint64_t A0j = 0, A1j = 0;
        if ((uint32_t)lane < nt) {
            A0j = p.a_rp[r];
            A1j = p.a_rp[r + 1];
        }
        const uint64_t lj = A1j - A0j;
        // product bound: 4 per ELL group (the markers serve as the prefix window, then are cleared).
        // With a small cap (single-window launches) a row of more than cap / 4 entries is taken as
        // long without reading its entries (bound >= 4 per entry with a non-empty B row; a row sent
        // long with empty B rows among its entries is still correct, only another category)
        const uint64_t jump = p.sym_cap ? (uint64_t)kCap / 4 : 256;
        const uint32_t gj = tile_groups<CSR>(p, A0j, A1j, nt, marks, jump);
        const uint32_t bj = gj > 0x3FFFFFFFu ? 0xFFFFFFFFu : 4 * gj;
        ((uint4 *)marks)[lane] = make_uint4(0, 0, 0, 0);
        wave_sync();
        const bool fatj = (uint32_t)lane < nt && fat_row(p, r);
        const bool shortj = (uint32_t)lane < nt && bj <= kCap && lj <= jump && !fatj;
        const unsigned long long shortm = __ballot(shortj);
        list_rows(p, (uint32_t)lane < nt && !shortj && !fatj, r);
        if (p.spec_flag && (uint32_t)lane < nt && !shortj && !fatj) p.counts[r] = 0;  // (the call is void)
        uint32_t b = 0;
        for (;;) {
            const unsigned long long m = b < (uint32_t)kWave ? (shortm >> b) << b : 0ull;
            if (!m) break;
            b = (uint32_t)__builtin_ctzll(m);
            const bool inb = (uint32_t)lane >= b;
            const uint32_t pb = wave_incl_scan(inb ? bj : 0u, 0u, [](uint32_t x, uint32_t y) { return x + y; });
            const uint32_t pl = wave_incl_scan(inb ? (uint32_t)lj : 0u, 0u, [](uint32_t x, uint32_t y) { return x + y; });
            const unsigned long long stop =
                __ballot(inb && (!shortj || pb > kCap || pl > 256 || (cb == 0 && (uint32_t)lane > b)));
            const uint32_t e = stop ? (uint32_t)__builtin_ctzll(stop) : nt;  // > b: row b is short
            const uint64_t A0 = readlane_u64(A0j, (int)b), A1 = readlane_u64(A1j, (int)(e - 1));
            const uint32_t nent = (uint32_t)(A1 - A0);
            if (inb && (uint32_t)lane < e && lj > 0) atomicMax(&marks[(uint32_t)(A0j - A0)], (uint32_t)lane - b + 1);
            wave_sync();
            uint32_t kq[kRegQ], lq[kRegQ], ng[kRegQ], carry = 0, mxg = 0;
            // (SLAT_MK_HOIST: every round's marker read issued before the first scan)
            uint32_t mks[kRegQ];
            if constexpr (SLAT_MK_HOIST)
                sfor<kRegQ>([&](auto Q) {
                    const uint32_t i = Q * kWave + lane;
                    mks[Q] = i < nent ? marks[i] : 0u;
                });
            sfor<kRegQ>([&](auto Q) {
                const uint32_t i = Q * kWave + lane;
                const uint32_t mk = SLAT_MK_HOIST ? mks[Q] : (i < nent ? marks[i] : 0u);
                const uint32_t run = max(wave_incl_scan(mk, 0u, [](uint32_t x, uint32_t y) { return max(x, y); }), carry);
                carry = readlane_u32(run, kWave - 1);
                lq[Q] = run - 1;
                kq[Q] = kSent;
                if (i < nent) {
                    kq[Q] = p.a_col[A0 + i];
                    marks[i] = 0;
                }
            });
            // (ng: ELL, the B row's groups; CSR, its length, and kq its first entry)
            uint32_t gq[kRegQ];
            sfor<kRegQ>([&](auto Q) {
                ng[Q] = short_brow<CSR>(p, kq[Q]);
                gq[Q] = short_groups<CSR>(ng[Q]);
                mxg = max(mxg, gq[Q]);
            });
            mxg = wave_max_u32(mxg);
            uint32_t nprod = 0, pos[kRegQ];
            const uint32_t G = group_positions(gq, pos);
            const uint32_t noval[kRegQ] = {};
            for (uint32_t base = 0; base < G; base += kStageG) {
                stage_groups<false, CSR, uint32_t>(base, mxg, kq, lq, ng, pos, noval, gk, gl, nullptr);
                const uint32_t n = min(G - base, kStageG);
                for (uint32_t g0 = 0; g0 < n; g0 += kWave) {
                    const uint32_t g = g0 + lane;
                    uint32_t cc[4] = {kSent, kSent, kSent, kSent}, sl[4], lr = 0;
                    if (g < n) {
                        const uint32_t w = gk[g], glb = gl[g];
                        const uint4 c = staged_cols<CSR>(p, w, glb);
                        lr = glb & 63u;
                        const uint32_t hi = lr << cb;
                        cc[0] = c.x != kSent ? (hi | c.x) : kSent;
                        cc[1] = c.y != kSent ? (hi | c.y) : kSent;
                        cc[2] = c.z != kSent ? (hi | c.z) : kSent;
                        cc[3] = c.w != kSent ? (hi | c.w) : kSent;
                    }
                    bool fresh[4];
                    if (p.stats)  // launch-uniform: no VALU for the product count otherwise
#pragma unroll
                        for (int x = 0; x < 4; ++x) nprod += cc[x] != kSent ? 1u : 0u;
                    hash_batch<4>(keys, 10, cc, sl, fresh);
                    const uint32_t f = (uint32_t)fresh[0] + fresh[1] + fresh[2] + fresh[3];
                    if (f) atomicAdd(&rcnt[lr], f);
                }
                wave_sync();
            }
            if (p.stats) flops += wave_sum_u32(nprod);
            if (inb && (uint32_t)lane < e) {
                p.counts[r] = rcnt[lane - b];
                rcnt[lane - b] = 0;
            }
            uint4 *k4 = (uint4 *)keys;
            for (uint32_t w = lane; w < kSymHashT / 4; w += kWave) k4[w] = make_uint4(kSent, kSent, kSent, kSent);
            wave_sync();
            b = e;
        }
    }
    if (p.stats && lane == 0 && flops)
        atomicAdd(&p.shards[((blockIdx.x * kWpb + wv) % kShards) * kShardStride + 3], flops);
}

// ------------------------------------------------------------------------------------------------
// Wave-wide bitonic sort of 256 (key, payload) pairs, 4 per lane (element i = lane * 4 + e): the
// emit order of the hash categories' keys.
// ------------------------------------------------------------------------------------------------
// value of lane (lane ^ M): DPP quad permutes for 1 and 2 (bound_ctrl: no old value to set up, every
// lane reads a valid source), ds_swizzle (bit-mask mode, within 32 lanes) up to 16, ds_bpermute for
// 32. (DPP row_ror / half-mirror pairs for 4 and 8 and gfx950's permlane16/32 swaps for 16 and 32
// measured no faster on C4's sorts: profiles/r03_ab_dyn_xlane.txt.)
template <int M>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x) {
    if constexpr (M == 1)
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, true);  // quad_perm [1,0,3,2]
    else if constexpr (M == 2)
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xf, 0xf, true);  // quad_perm [2,3,0,1]
    else if constexpr (M < 32)
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (M << 10) | 0x1F);
    else
        return (uint32_t)__shfl_xor((int)x, 32);
}
template <int M, typename T>
__device__ __forceinline__ T lane_xor_t(T v) {
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, lane_xor<M>(__builtin_bit_cast(uint32_t, v)));
    } else {
        const uint64_t u = __builtin_bit_cast(uint64_t, v);
        return __builtin_bit_cast(T, ((uint64_t)lane_xor<M>((uint32_t)(u >> 32)) << 32) | lane_xor<M>((uint32_t)u));
    }
}

// One compare-exchange step (K, J) of the bitonic network over 256 elements, element i = lane * 4 + e.
// U (unique keys, or ties whose payloads do not matter: the emit's kSent padding): a swap is one
// compare xor'ed with the lane's direction mask. Otherwise ties keep their own payload, so a pair
// never duplicates or loses one.
template <int K, int J, bool HV, bool U, typename T>
__device__ __forceinline__ void bitonic_step(uint32_t (&k)[4], T (&v)[4], uint32_t lane) {
    if constexpr (J >= 4) {
        constexpr int M = J / 4;
        const bool asc = (lane & (K / 4)) == 0;
        const bool tmin = ((lane & M) == 0) == asc;
        uint32_t pk[4];
        T pv[4];
        sfor<4>([&](auto E) {
            pk[E] = lane_xor<M>(k[E]);
            if constexpr (HV) pv[E] = lane_xor_t<M>(v[E]);
        });
        sfor<4>([&](auto E) {
            const bool sw = U ? ((pk[E] < k[E]) == tmin) : (tmin ? pk[E] < k[E] : pk[E] > k[E]);
            if constexpr (HV) v[E] = sw ? pv[E] : v[E];
            k[E] = sw ? pk[E] : k[E];
        });
    } else {
        sfor<4>([&](auto E) {
            constexpr int e = decltype(E)::value;
            if constexpr ((e & J) == 0) {
                constexpr int f = e | J;
                const bool asc = (((lane << 2) | (uint32_t)e) & (uint32_t)K) == 0;
                const bool sw = U ? ((k[f] < k[e]) == asc) : (asc ? k[e] > k[f] : k[e] < k[f]);
                const uint32_t t = k[e];
                k[e] = sw ? k[f] : t;
                k[f] = sw ? t : k[f];
                if constexpr (HV) {
                    const T tv = v[e];
                    v[e] = sw ? v[f] : tv;
                    v[f] = sw ? tv : v[f];
                }
            }
        });
    }
}
template <int K, int J, bool HV, bool U, typename T>
__device__ __forceinline__ void bitonic_merge(uint32_t (&k)[4], T (&v)[4], uint32_t lane) {
    bitonic_step<K, J, HV, U, T>(k, v, lane);
    if constexpr (J > 1) bitonic_merge<K, J / 2, HV, U, T>(k, v, lane);
}
// ascending sort of the wave's 256 keys (kSent last), payloads travel with their keys
template <bool HV, typename T, bool U = false>
__device__ __forceinline__ void wave_sort256(uint32_t (&k)[4], T (&v)[4]) {
    const uint32_t lane = (uint32_t)lane_id();
    bitonic_merge<2, 1, HV, U, T>(k, v, lane);
    bitonic_merge<4, 2, HV, U, T>(k, v, lane);
    bitonic_merge<8, 4, HV, U, T>(k, v, lane);
    bitonic_merge<16, 8, HV, U, T>(k, v, lane);
    bitonic_merge<32, 16, HV, U, T>(k, v, lane);
    bitonic_merge<64, 32, HV, U, T>(k, v, lane);
    bitonic_merge<128, 64, HV, U, T>(k, v, lane);
    bitonic_merge<256, 128, HV, U, T>(k, v, lane);
}

// LDS of k_numeric_short per wave: the hash table of ShortSem<Sem> (hash_bytes: keys | values |
// staged keys u32[260], which also stage the groups' B rows gk) | scratch of short_mx bytes, in turn
// the entry -> row markers u32[256], the staged A values ga S[256] and the emit's slots u32[256]
// (cleared after each batch) | per-row zero counts u32[64] | staged local rows gl u8[kStageG]
template <typename Sem>
__host__ __device__ constexpr uint32_t short_mx() {
    return 256 * (uint32_t)sizeof(typename Sem::S) > 1024 ? 256 * (uint32_t)sizeof(typename Sem::S) : 1024;
}
template <typename Sem>
__host__ __device__ constexpr uint32_t short_bytes() {
    return hash_bytes<ShortSem<Sem>>() + short_mx<Sem>() + kWave * 4 + kStageG;
}

// Emit of a batch of rows held in the hash table (<= 256 keys, all distinct): the keys and their
// slots are compacted into hstage / hslot, loaded 4 per lane and sorted across the wave
// (wave_sort256); a key's sorted position IS its output index in the batch, since keys are
// composite (lr << cb | column, cb > 0) and the batch's rows are contiguous in C. The table is left
// clean; zero values go to zero(local row).
// PACK: the batch's keys fit 23 bits (<= 8 local rows, cb <= 20), so key << 9 | slot is one u32 and the
// sort moves no payload (half the lane exchanges and selects)
template <typename Sem, bool PACK, typename Z>
__device__ __forceinline__ void batch_emit(uint32_t *hkeys, typename Sem::V *hvals, uint32_t *hstage, uint32_t *hslot,
                                           uint32_t cb, uint32_t tot, uint32_t *oc, typename Sem::S *ov, Z &&zero) {
    using S = typename Sem::S;
    using V = typename Sem::V;
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t hk[kHashHeld], nh = 0;
    sfor<kHashHeld>([&](auto I_) {
        hk[I_] = hkeys[I_ * kWave + lane];
        nh += hk[I_] != kSent ? 1u : 0u;
    });
    const uint32_t incl = wave_incl_scan(nh, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    const uint32_t nk = min(readlane_u32(incl, kWave - 1), kHashT / 2);
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
    const uint4 k4 = ((const uint4 *)hstage)[lane], s4 = ((const uint4 *)hslot)[lane];
    uint32_t k[4] = {k4.x, k4.y, k4.z, k4.w}, sl[4] = {s4.x, s4.y, s4.z, s4.w};
    sfor<4>([&](auto E) {
        if (lane * 4 + E >= nk) k[E] = kSent;
    });
    if constexpr (PACK) {
        sfor<4>([&](auto E) {
            if (k[E] != kSent) k[E] = (k[E] << 9) | sl[E];
        });
        wave_sort256<false, uint32_t, true>(k, sl);
        sfor<4>([&](auto E) {
            sl[E] = k[E] & (kHashT - 1);
            if (k[E] != kSent) k[E] >>= 9;
        });
    } else {
        wave_sort256<true, uint32_t, true>(k, sl);  // distinct keys (kSent padding aside)
    }
    const uint32_t cmask = cb ? (1u << cb) - 1 : 0xFFFFFFFFu;
    sfor<4>([&](auto E) {
        const uint32_t i = lane * 4 + E;
        if (k[E] != kSent) {
            const S v = Sem::finish(hvals, sl[E]);
            if (Sem::is_zero(v)) zero(cb ? k[E] >> cb : 0u);
            if (i < tot) {  // never write past the batch's slice
                oc[i] = k[E] & cmask;
                ov[i] = v;
            }
#pragma unroll
            for (int w = 0; w < Sem::kSlots; ++w) hvals[sl[E] * Sem::kSlots + w] = V(0);
        }
    });
    if (lane < ExtraWords<Sem>::value) hvals[kHashT * Sem::kSlots + lane] = V(0);
    wave_sync();
}

template <typename Sem0, typename I, bool CSR>
__device__ __forceinline__ void numeric_short_body(Args p) {
    using Sem = ShortSem<Sem0>;
    using S = typename Sem::S;
    using V = typename Sem::V;
    static_assert(!Sem::kOrdered, "f64 keeps the ordered single-row path");
    constexpr int kWpb = kBlock / kWave;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    constexpr uint32_t kMx = short_mx<Sem0>();
    uint8_t *region = smem8 + (size_t)wv * short_bytes<Sem0>();
    uint32_t *hkeys = (uint32_t *)region;
    V *hvals = (V *)(region + kHashT * 4);
    uint32_t *hstage = (uint32_t *)(region + kHashT * 4 + kHashT * sizeof(V) * Sem::kSlots + ExtraWords<Sem>::value * 4);
    uint32_t *marks = (uint32_t *)(region + hash_bytes<Sem>());
    uint32_t *hslot = marks;                // the emit's slots
    S *ga = (S *)marks;                     // the accumulation's A values
    uint32_t *zc = marks + kMx / 4;
    uint32_t *gk = hstage;
    uint8_t *gl = (uint8_t *)(zc + kWave);
    static_assert(kStageG * sizeof(S) <= kMx && kMx >= 1024, "scratch too small");
    for (uint32_t w = lane; w < kHashT; w += kWave) hkeys[w] = kSent;
    for (uint32_t w = lane; w < kHashT * Sem::kSlots + ExtraWords<Sem>::value; w += kWave) hvals[w] = V(0);
    for (uint32_t w = lane; w < kMx / 16; w += kWave) ((uint4 *)marks)[w] = make_uint4(0, 0, 0, 0);
    zc[lane] = 0;
    wave_sync();
    // pattern B (every B value equal): no B-value loads (u32 with the ELL copy, as k_numeric)
    uint32_t bvmax = 0;
    bool buni = false;
    if constexpr (Sem::kNarrowable)
        if (p.b_vmax) {
            const unsigned long long v = ((volatile unsigned long long *)p.b_vmax)[kVMaxWord];
            const unsigned long long vi = ((volatile unsigned long long *)p.b_vmax)[kVMinInvWord];
            if ((uint32_t)(v >> 32) == p.epoch) {
                bvmax = (uint32_t)v;
                // (a wider value type clamps to u32 in the summary: all-equal clamped values are
                // not a pattern unless below the clamp)
                buni = SLAT_NUM_UNI && (uint32_t)(vi >> 32) == p.epoch && ~(uint32_t)vi == bvmax &&
                       (sizeof(S) == 4 || bvmax != 0xFFFFFFFFu);
            }
        }
    const S bv0 = (S)bvmax;
    const S *av_ = (const S *)p.a_val;
    S *cval = (S *)p.c_val;
    uint32_t zrows = 0;
    const uint32_t cb = p.cbits;
    // packed emit keys (batch_emit PACK): batches of <= 8 rows whose composite keys, shifted past a
    // 9-bit slot, stay below kSent
    const bool pack = SLAT_SHORT_PACK && cb > 0 && cb <= 20 && ((((7ull << cb) | (p.ncols - 1)) << 9) | 511ull) < 0xFFFFFFFFull;
    const uint32_t T = p.tile_rows ? p.tile_rows : (uint32_t)kWave;
    const uint64_t ntiles = (p.nrows + T - 1) / T;
    PhaseClock pc{};  // diagnostic builds (SLAT_PHASES): where the waves' time goes
    if constexpr (SLAT_PHASES) pc.t = __builtin_amdgcn_s_memtime();
    const XcdStride xs(ntiles, kWpb, wv);
    for (uint64_t tile = xs.first; tile < xs.end; tile += xs.stride) {
        const uint64_t r0 = tile * T, r = r0 + lane;
        const uint32_t nt = (uint32_t)min<uint64_t>(T, p.nrows - r0);
        uint64_t A0j = 0, A1j = 0, obj = 0, oej = 0;
        if ((uint32_t)lane < nt) {
            A0j = p.a_rp[r];
            A1j = p.a_rp[r + 1];
            obj = p.c_rp[r];
            oej = p.c_rp[r + 1];
        }
        const uint64_t uj = oej - obj, lj = A1j - A0j;
        const bool fatj = (uint32_t)lane < nt && fat_row(p, r);
        // rows of <= 256 outputs and <= 256 A entries (rows with more entries go to the window launch).
        // A row of no outputs has no products: skipped (a speculative launch's rows that symbolic
        // listed have 0 here, whatever their products: in a batch they could overfill the table)
        const bool emptyj = uj == 0;
        const bool shortj = (uint32_t)lane < nt && uj <= kHashT / 2 && lj <= 256 && !fatj && !emptyj;
        const unsigned long long shortm = __ballot(shortj);
        list_rows(p, (uint32_t)lane < nt && !shortj && !fatj && !emptyj, r);  // the window launch's rows
        uint32_t b = 0;
        for (;;) {
            const unsigned long long m = b < (uint32_t)kWave ? (shortm >> b) << b : 0ull;
            if (!m) break;
            b = (uint32_t)__builtin_ctzll(m);
            // the batch: short rows b, b+1, ... while outputs <= kHashT / 2 and entries <= 256
            const bool inb = (uint32_t)lane >= b;
            const uint32_t uu = inb ? (uint32_t)min<uint64_t>(uj, 1u << 20) : 0u;
            const uint32_t ll = inb ? (uint32_t)min<uint64_t>(lj, 1u << 20) : 0u;
            const uint32_t pu = wave_incl_scan(uu, 0u, [](uint32_t x, uint32_t y) { return x + y; });
            const uint32_t pl = wave_incl_scan(ll, 0u, [](uint32_t x, uint32_t y) { return x + y; });
            const unsigned long long stop = __ballot(inb && (!shortj || pu > kHashT / 2 || pl > 256 ||
                                                             (cb == 0 && (uint32_t)lane > b) ||
                                                             (pack && (uint32_t)lane - b >= 8u)));
            const uint32_t e = stop ? (uint32_t)__builtin_ctzll(stop) : nt;
            pc.mark(0);  // tile header, batch formation
            pc.ph[kPhaseSlots - 1] += 1;
            const uint64_t A0 = readlane_u64(A0j, (int)b);
            const uint64_t OB = readlane_u64(obj, (int)b);
            HashAcc<Sem> ha{hkeys, hvals};
            const uint64_t A1 = readlane_u64(A1j, (int)(e - 1));
            const uint32_t nent = (uint32_t)(A1 - A0);
            const uint32_t lim = readlane_u32(pu, (int)(e - 1));
            // entry -> local row: mark each row's first entry (a later, non-empty row wins a tie
            // with empty rows before it), then a running max over the entries
            if (inb && (uint32_t)lane < e && lj > 0) atomicMax(&marks[(uint32_t)(A0j - A0)], (uint32_t)lane - b + 1);
            wave_sync();
            uint32_t kq[kRegQ], lq[kRegQ], ng[kRegQ];
            S aq[kRegQ];
            uint32_t carry = 0, mxg = 0;
            // (SLAT_MK_HOIST: every round's marker read issued before the first scan)
            uint32_t mks[kRegQ];
            if constexpr (SLAT_MK_HOIST)
                sfor<kRegQ>([&](auto Q) {
                    const uint32_t i = Q * kWave + lane;
                    mks[Q] = i < nent ? marks[i] : 0u;
                });
            sfor<kRegQ>([&](auto Q) {
                const uint32_t i = Q * kWave + lane;
                const uint32_t mk = SLAT_MK_HOIST ? mks[Q] : (i < nent ? marks[i] : 0u);
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
            // (ng: ELL, the B row's groups; CSR, its length, and kq its first entry; malformed
            // entries: 0)
            sfor<kRegQ>([&](auto Q) {
                ng[Q] = short_brow<CSR>(p, kq[Q]);
                mxg = max(mxg, short_groups<CSR>(ng[Q]));
            });
            mxg = wave_max_u32(mxg);
            pc.mark(1);  // A entries, local rows, group counts
            uint32_t pos[kRegQ];
            uint32_t G;
            {
                uint32_t gq[kRegQ];
                sfor<kRegQ>([&](auto Q) { gq[Q] = short_groups<CSR>(ng[Q]); });
                G = group_positions(gq, pos);
            }
            bool narrow = false;  // u32: no sum of this batch can wrap (each key takes <= G products)
            if constexpr (std::is_same_v<Sem, SemU32W>) {
                if (bvmax) {
                    uint32_t am = 0;
                    sfor<kRegQ>([&](auto Q) { am = max(am, (uint32_t)aq[Q]); });
                    const unsigned long long ab = (unsigned long long)wave_max_u32(am) * bvmax;
                    narrow = ab < (1ull << 32) && ab * G < (1ull << 32);
                }
            }
            for (uint32_t base = 0; base < G; base += kStageG) {
                stage_groups<true, CSR, S>(base, mxg, kq, lq, ng, pos, aq, gk, gl, ga);
                const uint32_t n = min(G - base, kStageG);
                for (uint32_t g0 = 0; g0 < n; g0 += kWave) {
                    const uint32_t g = g0 + lane;
                    uint4 ck = make_uint4(kSent, kSent, kSent, kSent);
                    Quad<S> pr{};
                    if (g < n) {
                        const uint32_t w = gk[g], glb = gl[g];
                        const uint4 c = staged_cols<CSR>(p, w, glb);
                        const S a = ga[g];
                        pr = buni ? splat4(Sem::prod(a, bv0)) : prods<Sem>(a, staged_vals<CSR, S>(p, w, glb));
                        const uint32_t hi = (glb & 63u) << cb;
                        ck.x = c.x != kSent ? (hi | c.x) : kSent;
                        ck.y = c.y != kSent ? (hi | c.y) : kSent;
                        ck.z = c.z != kSent ? (hi | c.z) : kSent;
                        ck.w = c.w != kSent ? (hi | c.w) : kSent;
                    }
                    if constexpr (std::is_same_v<Sem, SemU32W>) {
                        if (narrow) {
                            HashAcc<SemU32WN>{hkeys, hvals}(ck, pr);
                        } else {
                            ha(ck, pr);
                        }
                    } else {
                        ha(ck, pr);
                    }
                }
                wave_sync();
            }
            wave_sync();
            pc.mark(2);  // ELL loads, hash accumulation
            auto zero = [&](uint32_t lr) { atomicAdd(&zc[lr], 1u); };
            if (pack)
                batch_emit<Sem, true>(hkeys, hvals, hstage, hslot, cb, lim, p.c_col + OB, cval + OB, zero);
            else
                batch_emit<Sem, false>(hkeys, hvals, hstage, hslot, cb, lim, p.c_col + OB, cval + OB, zero);
            pc.mark(3);  // emit
            if (inb && (uint32_t)lane < e) {
                const uint32_t z = zc[lane - b];
                p.counts[r] = uj - z;
                zrows += z ? 1u : 0u;
            }
            wave_sync();
            if (inb && (uint32_t)lane < e) zc[lane - b] = 0;
            for (uint32_t w = lane; w < kMx / 16; w += kWave) ((uint4 *)marks)[w] = make_uint4(0, 0, 0, 0);  // markers
            wave_sync();
            pc.mark(4);  // counts
            b = e;
        }
    }
    if constexpr (SLAT_PHASES) {
        if (lane == 0) {
            unsigned long long *dst = p.shards + 512 + ((blockIdx.x * kWpb + wv) % 64) * kPhaseSlots;
            for (int i = 0; i < kPhaseSlots; ++i) atomicAdd(&dst[i], (unsigned long long)pc.ph[i]);
        }
    }
    add_zero_rows(&p.host_out[2], wave_sum_u32(zrows), p.seq != 0);
}

template <typename Sem0, typename I, bool CSR = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_numeric_short(Args p) {
    numeric_short_body<Sem0, I, CSR>(p);
    signal_done(p);
}
// u32: 5 waves per SIMD (6.6 KB of LDS per wave, <= 96 VGPRs; the wider semirings are held to 4
// waves by their LDS anyway). At 6 waves (<= 80 VGPRs) 28 VGPRs spilled to scratch and C4's numeric
// pass took 1.235 ms against 0.942 ms here, 4 waves 1.053 ms (profiles/r03_ab_prefetch_short_wpe.txt).
// Variant builds: -DSLAT_SHORT_WPE=w (0: no cap).
#ifndef SLAT_SHORT_WPE
#define SLAT_SHORT_WPE 5
#endif
template <typename I, bool CSR = false>
__global__ __launch_bounds__(kBlock)
#if SLAT_SHORT_WPE
__attribute__((amdgpu_waves_per_eu(SLAT_SHORT_WPE)))
#endif
void k_numeric_short_u32(Args p) {
    numeric_short_body<SemU32, I, CSR>(p);
    signal_done(p);
}

// ------------------------------------------------------------------------------------------------
// row_ptr = inclusive scan of the row counts: ONE single-pass kernel (decoupled look-back). Tiles of
// 2048 rows, each publishes its aggregate then its inclusive prefix in an epoch-tagged status word
// (no init kernel). The last
// tile writes the total nnz and the max row nnz into mapped host memory (no copy in the stream).
// ------------------------------------------------------------------------------------------------
#ifndef SLAT_SCAN_THREADS
#define SLAT_SCAN_THREADS 256  // variant builds: tile geometry of k_scan_rows
#endif
#ifndef SLAT_SCAN_ITEMS
#define SLAT_SCAN_ITEMS 8
#endif
constexpr int kScanThreads = SLAT_SCAN_THREADS, kScanItems = SLAT_SCAN_ITEMS;
constexpr uint64_t kScanTile = (uint64_t)kScanThreads * kScanItems;
constexpr unsigned long long kStAgg = 1ull << 40, kStInc = 2ull << 40, kStVal = (1ull << 40) - 1;


// Decoupled look-back by a whole wave: publish tile `tile`'s aggregate, then walk back over the
// earlier tiles' epoch-tagged status words (an aggregate, or an inclusive prefix that ends the walk)
// and publish the tile's own inclusive prefix; returns its exclusive prefix. Tiles are taken in
// ticket (or resident block) order, so every earlier tile belongs to a block that is running or
// done and never waits on a later one. A round reads kLookR predecessors per lane (the nearest
// inclusive prefix by ballot, the aggregates before it by a wave sum) instead of one dependent load
// per predecessor: many small tiles arriving together (k_lane: ~400 one-wave blocks) made a lane-0
// walk a chain of hundreds of loads. Called by every lane of the wave; returns the tile's exclusive
// prefix in every lane.
// (split in two: lookback_publish stores the tile's aggregate (tile 0: its inclusive prefix), and
// lookback_walk reads the predecessors, so a caller can do work that does not need the offset in
// between)
__device__ __forceinline__ void lookback_publish(unsigned long long *status, uint64_t tile, uint32_t epoch,
                                                 unsigned long long agg) {
    const unsigned long long tag = (unsigned long long)epoch << 42;
    if (lane_id() == 0)
        __hip_atomic_store(&status[tile], tag | (tile == 0 ? kStInc : kStAgg) | agg, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int kLookR = 4;  // predecessors per lane per round of the walk
__device__ __forceinline__ unsigned long long lookback_walk(unsigned long long *status, uint64_t tile, uint32_t epoch,
                                                            unsigned long long agg) {
    auto ld = [](unsigned long long *x) { return __hip_atomic_load(x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    auto st = [](unsigned long long *x, unsigned long long v) {
        __hip_atomic_store(x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    const int lane = lane_id();
    const unsigned long long tag = (unsigned long long)epoch << 42;
    if (tile == 0) return 0;
    unsigned long long excl = 0;
    // round: lane l reads predecessors tile - 1 - (l * kLookR + i), i < kLookR, so one round covers
    // 256 (a grid whose blocks arrive together walks back to block 0: k_lane's 422 blocks took 7
    // rounds of 64, each a device-scope load latency, ~7 us; now 2)
    for (int64_t j0 = (int64_t)tile - 1;; j0 -= kWave * kLookR) {
        unsigned long long x[kLookR];
        int first = kLookR, last = kWave;
        unsigned long long inc = 0;
        while (true) {
            sfor<kLookR>([&](auto I) {
                const int64_t j = j0 - (lane * kLookR + I);
                x[I] = 0;
                if (j >= 0) x[I] = ld(&status[j]);
            });
            // the lane's nearest published inclusive prefix (kLookR: none), the wave's nearest by
            // ballot; only the statuses between this tile and that one must be published (a later
            // tile's walk need not wait for tiles before the nearest inclusive prefix)
            uint32_t valid = 0;
            first = kLookR;
            sfor<kLookR>([&](auto I) {
                const int64_t j = j0 - (lane * kLookR + I);
                const bool v = j < 0 || ((x[I] >> 42) == epoch && (x[I] & (kStAgg | kStInc)) != 0);
                valid |= (v ? 1u : 0u) << I;
                if (first == kLookR && j >= 0 && v && (x[I] & kStInc)) first = I;
            });
            inc = __ballot(first < kLookR);
            last = inc ? (int)__builtin_ctzll(inc) : kWave;  // the lane holding it (kWave: none)
            const uint32_t need = lane < last ? (1u << kLookR) - 1 : lane == last ? (1u << first) - 1 : 0u;
            if (__ballot((valid & need) != need) == 0) break;
            __builtin_amdgcn_s_sleep(1);
        }
        unsigned long long v = 0;
        sfor<kLookR>([&](auto I) {
            const int64_t j = j0 - (lane * kLookR + I);
            if (j >= 0 && (lane < last || (lane == last && (int)I <= first))) v += x[I] & kStVal;
        });
        v = wave_incl_scan_u64(v);
        excl += readlane_u64(v, kWave - 1);
        if (inc || j0 - (int64_t)(kWave * kLookR) < 0) break;
    }
    if (lane == 0) st(&status[tile], tag | kStInc | (excl + agg));
    return excl;
}
__device__ __forceinline__ unsigned long long lookback_prefix_wave(unsigned long long *status, uint64_t tile,
                                                                   uint32_t epoch, unsigned long long agg) {
    lookback_publish(status, tile, epoch, agg);
    return lookback_walk(status, tile, epoch, agg);
}


// bpart (optional): k_build_ell's nbpart per-block B-value partials ((~min << 32) | max), reduced by
// one wave of tile 0 into vmax[kVMaxWord] = (vepoch << 32) | max, vmax[kVMinInvWord] =
// (vepoch << 32) | ~min for the numeric pass (which runs after this kernel)
// Tiles in increasing order per block: block b takes tiles b, b + G, b + 2G, ... (G = the grid,
// at most one block per CU, all resident), so every tile's predecessors belong to blocks that are
// running or done, and the walk back from tile t finds tile t - G's inclusive prefix within one round
// of 256 predecessors. (Ticket order, used before for grids past the CU count, took one atomic on a
// single address per tile: C4's 489 tiles took 23 us for an 8 MB scan.)
static __global__ __launch_bounds__(kScanThreads) void k_scan_rows(const uint64_t *counts, uint64_t n, uint64_t *rp,
                                                            unsigned long long *status, uint32_t epoch,
                                                            unsigned long long *maxw, unsigned long long *host_out,
                                                            const unsigned long long *bpart, uint32_t nbpart,
                                                            unsigned long long *vmax, uint32_t vepoch,
                                                            const uint32_t *bmax, uint32_t nbmax,
                                                            unsigned int *zero_word) {
    __shared__ unsigned long long wsum[kScanThreads / kWave];
    if (zero_word && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0;  // (the next call's list length)
    __shared__ unsigned long long s_bcast[2];
    __shared__ uint32_t wmax[kScanThreads / kWave];
    const int t = threadIdx.x, lane = lane_id(), w = t / kWave;
    const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
    // (tile 0's last wave) k_build_ell's B-value partials, the first 8 per lane loaded now, so they
    // land under the tile's scan instead of after it (a chain of dependent loads at the end of the
    // kernel: 211 partials on the headline)
    constexpr int kBP = 8;
    unsigned long long bq[kBP];
    const bool bred = blockIdx.x == 0 && nbpart && w == kScanThreads / kWave - 1;
    if (bred)
#pragma unroll
        for (int k = 0; k < kBP; ++k) {
            const uint32_t i = (uint32_t)lane + (uint32_t)k * kWave;
            bq[k] = i < nbpart ? bpart[i] : 0ull;
        }
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        // bmax (<= 16 * kScanThreads entries): the counts' producer left per-block max counts; the
        // last tile reduces them, its loads issued now so they land during the look-back
        uint32_t bm = 0;
        if (bmax && tile == ntiles - 1) {
            uint32_t q[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint32_t i = (uint32_t)t + (uint32_t)k * kScanThreads;
                q[k] = i < nbmax ? bmax[i] : 0u;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) bm = max(bm, q[k]);
        }
        const uint64_t i0 = tile * kScanTile + (uint64_t)t * kScanItems;
        unsigned long long v[kScanItems], run = 0;
        uint32_t mx = 0;
#pragma unroll
        for (int e = 0; e < kScanItems; ++e) v[e] = i0 + e < n ? counts[i0 + e] : 0ull;
#pragma unroll
        for (int e = 0; e < kScanItems; ++e) {
            mx = max(mx, (uint32_t)min<unsigned long long>(v[e], 0xFFFFFFFFull));
            run += v[e];
            v[e] = run;
        }
        const unsigned long long wi = wave_incl_scan_u64(run);
        mx = wave_max_u32(bmax ? bm : mx);
        if (lane == kWave - 1) wsum[w] = wi;
        if (lane == 0) wmax[w] = mx;
        __syncthreads();
        unsigned long long wpre = 0, agg = 0;
        for (int k = 0; k < kScanThreads / kWave; ++k) {
            const unsigned long long x = wsum[k];
            wpre += k < w ? x : 0ull;
            agg += x;
        }
        if (w == 0) {
            uint32_t m = 0;
            for (int k = 0; k < kScanThreads / kWave; ++k) m = max(m, wmax[k]);
            // max row first (its result waited for), then the status: the max is in place once any
            // later tile sees this tile's status (bmax: the last tile has it from the producer's maxima)
            if (!bmax && lane == 0) maxw_raise(maxw, epoch, m);
            // the walk by the whole wave, 256 predecessors per round: a lane-0 walk was one dependent
            // load per predecessor still holding only its aggregate (one rank's eighth of C4, 62
            // tiles: 18.8 us for a 1 MB scan)
            const unsigned long long excl = lookback_prefix_wave(status, tile, epoch, agg);
            if (lane == 0) s_bcast[1] = excl;
            const uint32_t mr = tile == ntiles - 1 ? (bmax ? m : maxw_read(maxw, epoch)) : 0u;
            if (lane == 0 && tile == ntiles - 1) {
                if (n > 0) rp[0] = 0;
                const unsigned long long out[2] = {excl + agg, (unsigned long long)mr};
                for (int k = 0; k < 2; ++k)
                    __hip_atomic_store(&host_out[k], out[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        __syncthreads();
        const unsigned long long pre = s_bcast[1] + wpre + (wi - run);
#pragma unroll
        for (int e = 0; e < kScanItems; ++e)
            if (i0 + e < n) rp[1 + i0 + e] = pre + v[e];
        if (tile == 0 && bred) {
            uint32_t bx = 0, bn = 0;  // max, max of ~min
#pragma unroll
            for (int k = 0; k < kBP; ++k) {
                bx = max(bx, (uint32_t)bq[k]);
                bn = max(bn, (uint32_t)(bq[k] >> 32));
            }
            for (uint32_t i = lane + kBP * kWave; i < nbpart; i += kWave) {
                const unsigned long long q = bpart[i];
                bx = max(bx, (uint32_t)q);
                bn = max(bn, (uint32_t)(q >> 32));
            }
            bx = wave_max_u32(bx);
            bn = wave_max_u32(bn);
            if (lane == 0) {
                vmax[kVMaxWord] = ((unsigned long long)vepoch << 32) | bx;
                vmax[kVMinInvWord] = ((unsigned long long)vepoch << 32) | bn;
            }
        }
        __syncthreads();  // (the LDS words are reused by the block's next tile)
    }
}

// ------------------------------------------------------------------------------------------------
// compaction (rare): drop exact-zero values, moving row slices into exact-size arrays
// ------------------------------------------------------------------------------------------------
template <typename Sem>
__global__ __launch_bounds__(kBlock) void k_compact(const uint64_t *old_rp, const uint64_t *new_rp, uint64_t nrows,
                                                    const uint32_t *old_col, const typename Sem::S *old_val,
                                                    uint32_t *new_col, typename Sem::S *new_val) {
    const int lane = lane_id();
    constexpr int kWpb = kBlock / kWave;
    const uint64_t stride = (uint64_t)gridDim.x * kWpb;
    for (uint64_t row = (uint64_t)blockIdx.x * kWpb + threadIdx.x / kWave; row < nrows; row += stride) {
        const uint64_t s = old_rp[row], e = old_rp[row + 1];
        uint64_t d = new_rp[row];
        for (uint64_t t0 = s; t0 < e; t0 += kWave) {
            const uint64_t t = t0 + lane;
            typename Sem::S v{};
            bool keep = false;
            if (t < e) {
                v = old_val[t];
                keep = !Sem::is_zero(v);
            }
            const unsigned long long m = __ballot(keep);
            const uint32_t off = __popcll(m & ((1ull << lane) - 1ull));
            if (keep) {
                new_col[d + off] = old_col[t];
                new_val[d + off] = v;
            }
            d += __popcll(m);
        }
    }
}

// max over rows of row_ptr[i+1] - row_ptr[i]
static __global__ __launch_bounds__(kBlock) void k_max_row(const uint64_t *rp, uint64_t nrows, unsigned long long *shards) {
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
