// slat_internal.hpp — the context and host helpers shared by the library's translation units
// (slat_api.hip: SpGEMM; slat_graph.hip: the reference's SpGEMM consumers). Not installed.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "slat.h"

// A/B experiment knobs (environment variables) exist only in builds made with -DSLAT_AB_KNOBS
// (tools/build_variant.sh adds it): the shipped libslat.so ignores the environment, so a stray
// variable cannot change its kernel choices. (SLAT_MATMUL_PROGRESS, the reference's
// MATMUL_PROGRESS switch, is a feature and is read by every build.)
inline const char *slat_ab_knob(const char *name) {
#ifdef SLAT_AB_KNOBS
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

struct slat_hostio;  // the page-locked staging ring and its copy threads (slat_hostio.hip)

// internal call flag (above the public SLAT_FLAG_* bits): the rerun of a void speculative wide
// launch, which queues the listed-row launches
constexpr uint32_t kFlagNoSpec = 0x80000000u;

struct slat_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    int cu_count = 256;
    size_t lds_per_block_max = 65536;
    // workspace (grown on demand)
    void *ws = nullptr;
    size_t ws_bytes = 0;
    unsigned long long *h_shards = nullptr;  // pinned (stats / max-row read-backs)
    unsigned long long *h_out = nullptr;     // mapped pinned: [0] nnz, [1] max row nnz, [2] rows with zeros
    unsigned long long *h_out_dev = nullptr; // its device alias (written by k_scan_rows / k_numeric); [7]: the
                                             // end-of-call sequence word (k_signal)
    unsigned long long done_seq = 0;         // last sequence number queued to [7]
    unsigned long long *d_words = nullptr;   // [0] max-B word, [1] unused, [2] max-row word, [3] ~min-B word,
                                             // [4] check flags, [5] work tickets (zeroed by each launch's last taker),
                                             // [6] unused, [8] / [10] the symbolic list length (alternating
                                             // by call), [12] the numeric list length,
    unsigned long long *d_done = nullptr;    // the call's last kernel's two-level done count (signal_done)
    unsigned long long *d_maxw = nullptr;    // = d_done + kDoneBytes / 8: the one-kernel paths' max-row words
    unsigned long long *d_vmax = nullptr;    // = d_words + 0: (epoch << 32) | max B value (k_build_ell)
    uint32_t epoch = 0;                      // per-call tag of d_vmax (no reset between calls)
    uint32_t list_parity = 0;                // which of d_words[8] / [10] the next batched call's symbolic list uses
    bool lists_dirty = false;                // a call stopped before its scan zeroed the other list word
    // (A, B, row block) triples whose lane-kernel attempt overflowed (a row past slat_lane_cap()
    // products): the next call on the same triple goes to the pipeline directly instead of running
    // both. Keyed by both operands' arrays, sizes and the row range; an entry whose array the context
    // frees is dropped (slat_dev_free), so a new matrix at a recycled address starts clean
    struct LaneMiss {
        const void *a_rp, *a_col, *b_rp, *b_col;
        uint64_t a_nnz, b_nnz, a_rows, row_begin, row_end;
    } lane_miss[8] = {};
    uint32_t lane_miss_next = 0;
    // (A, B, row block) triples whose speculative wide launch (the listed-row launches skipped, as if
    // every row were short) found a row of the window category: the next call on the same triple
    // queues the listed-row launches directly instead of running twice
    LaneMiss list_miss[8] = {};
    uint32_t list_miss_next = 0;
    unsigned long long *d_status = nullptr;  // scan tile status words (epoch-tagged)
    uint64_t status_cap = 0;                 // tiles d_status holds
    uint32_t scan_epoch = 0;                 // tag of the status / max-row words (22 bits)
    size_t free_b = 0;                       // cached hipMemGetInfo free bytes
    uint32_t free_age = 0;
    bool mem_changed = true;                 // the pool took or returned a chunk since free_b was read
    hipEvent_t ev[6] = {};
    // device memory: hipMalloc'd chunks carved into pieces. A freed piece is cached and handed out
    // again in stream order (slat_dev_alloc); adjacent free pieces of a chunk merge; a chunk goes
    // back to the driver only when it is one free piece again.
    struct Block {
        void *p;
        size_t bytes;
        hipStream_t s;
        void *chunk;  // the hipMalloc'd base this piece belongs to
    };
    std::vector<Block> cache;                  // free pieces, oldest first
    size_t cache_bytes = 0;
    std::unordered_map<void *, Block> live;    // allocated piece -> its extent
    std::unordered_map<void *, size_t> chunks; // hipMalloc'd base -> its size
    slat_stats stats = {};
    slat_hostio *hio = nullptr;  // created by the first pageable host copy
};

// A prepared right operand (slat_bprep_create): the borrowed view, its max row, and (ell) the padded
// ELL image with the clamped B-value summary words vmax[kVMaxWord] / [kVMinInvWord] tagged `epoch`
struct slat_bprep {
    slat_csr_view b;
    uint64_t maxrow_b = 0;
    uint32_t wq = 0;
    bool ell = false;
    uint32_t *ecol = nullptr;
    void *eval = nullptr;
    uint8_t *eng = nullptr;
    unsigned long long *vmax = nullptr;
    uint32_t epoch = 0;
    int device = 0;
    const slat_ctx *owner = nullptr;  // the context whose pool and stream hold the image
};

#define SLAT_HIP(ctx, expr)                                                                        \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(e_);                        \
            return SLAT_EHIP;                                                                      \
        }                                                                                          \
    } while (0)

static inline slat_status fail(slat_ctx *ctx, slat_status s, const std::string &msg) {
    if (ctx) ctx->err = msg;
    return s;
}

static inline size_t vsize(int32_t dtype) { return dtype == SLAT_U32 ? 4 : 8; }

// C arrays in one device block (one allocation, one free per matrix):
// row_ptr | col_idx | values, each 256-byte aligned. alloc = 1 marks the layout for slat_csr_free.
enum { kAllocSeparate = 0, kAllocJoint = 1 };
static inline size_t joint_bytes(uint64_t nrows, uint64_t cap, size_t vs) {
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    return up((nrows + 1) * 8) + up(std::max<uint64_t>(cap, 1) * 4) + std::max<uint64_t>(cap, 1) * vs;
}
// Device memory of the library (C arrays, scan status, constructor scratch): blocks from hipMalloc,
// kept by the context after slat_dev_free and handed out again on the same stream (stream order
// makes the reuse safe without a sync). Not hipMallocAsync: on this image its pool lost kernel
// writes to part of a freshly grown block ("Device memory").
hipError_t slat_dev_alloc(slat_ctx *ctx, void **p, size_t bytes, hipStream_t s);
void slat_dev_free(slat_ctx *ctx, void *p, hipStream_t s);
// keep the first `bytes` of live piece p and cache the rest (a bound-sized C trimmed to its nnz)
void slat_dev_shrink(slat_ctx *ctx, void *p, size_t bytes);
void slat_dev_trim(slat_ctx *ctx);  // device sync, then every cached block back to the driver

// One block of the layout above.
static inline hipError_t alloc_joint(slat_ctx *ctx, slat_csr *m, uint64_t nrows, uint64_t cap, size_t vs, hipStream_t s) {
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t rp_b = up((nrows + 1) * 8), col_b = up(std::max<uint64_t>(cap, 1) * 4);
    uint8_t *base = nullptr;
    const hipError_t e = slat_dev_alloc(ctx, (void **)&base, joint_bytes(nrows, cap, vs), s);
    if (e != hipSuccess) return e;
    m->row_ptr = (uint64_t *)base;
    m->col_idx = (uint32_t *)(base + rp_b);
    m->values = base + rp_b + col_b;
    m->alloc = kAllocJoint;
    return hipSuccess;
}

// Host <-> device copies of host arrays on the context's stream, synchronous (slat_hostio.hip):
// pageable segments through the page-locked staging ring with a parallel memcpy, page-locked ones by
// one DMA each
struct slat_hostseg {
    void *host;
    void *dev;
    size_t bytes;
};
slat_status slat_copy_h2d(slat_ctx *ctx, const slat_hostseg *segs, int n);
slat_status slat_copy_d2h(slat_ctx *ctx, const slat_hostseg *segs, int n);
void slat_hostio_destroy(slat_ctx *ctx);

// workspace of at least `bytes` in ctx->ws (grown with a stream sync; contents not kept)
slat_status slat_ensure_ws(slat_ctx *ctx, size_t bytes);
// structural checks of a view (dtype, null arrays, u32 ids)
slat_status slat_check_view(slat_ctx *ctx, const slat_csr_view *v, const char *name);
// rp[0..n] = exclusive prefix of counts[0..n) (rp[n] = total) by k_scan_rows on stream s; the total
// and the max count land in ctx->h_out[0], [1] once the stream reaches that point
// bpart / nbpart / vepoch: k_build_ell's u32 B-value partials, reduced into ctx->d_vmax (else none)
// bmax / nbmax (<= 4096): per-block max counts left by the counts' producer; the scan then reduces
// those instead of its tiles' (slat_next_scan_epoch: the epoch the next scan tags its words with; it
// clears them on wrap)
slat_status slat_launch_scan(slat_ctx *ctx, const uint64_t *counts, uint64_t n, uint64_t *rp, hipStream_t s,
                             const unsigned long long *bpart = nullptr, uint32_t nbpart = 0, uint32_t vepoch = 0,
                             const uint32_t *bmax = nullptr, uint32_t nbmax = 0, unsigned int *zero_word = nullptr);
uint32_t slat_next_scan_epoch(slat_ctx *ctx, hipStream_t s);

// StdRng stream position (host_gen.cpp): key words and the index of the next keystream word; and
// the host state after `draws` more u64 draws (device generators draw by position)
extern "C" void slat_rng_position(const slat_rng *rng, uint32_t key[8], uint64_t *word);
extern "C" void slat_rng_advance(slat_rng *rng, uint64_t draws);
