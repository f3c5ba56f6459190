// spgemm_stored.hpp — k_numeric MODE 4: the numeric pass of single-window launches whose symbolic
// pass stored each row's bitmap blocks and whose B has its padded ELL image (the 30^3 chain's
// A^(k-1) * A, BASELINE configs C2 / C3), for the semirings that add in any order (u32, Sat64, f64
// any order). Included by spgemm_kernels.hpp after the generic passes it shares helpers with.
//
// The generic pass (MODE 0) takes six memory latencies per row one after another: the row's bounds,
// its A segment, the ELL group counts of its entries, the stored-block mask, the stored bitmap
// blocks, the ELL groups. Here a row waits out four:
//   1. bounds, C slice, stored-block mask and fat mark, loaded by lanes 0-5 one row AHEAD (issued
//      after the previous row's last loads, so they arrive under its accumulate and emit);
//   2. the A entries (up to 512, eight per lane) and the stored bitmap blocks, issued together;
//   3. the group counts of the entries;
//   4. the ELL groups, issued before the word ranks are built from the bitmap blocks, so the rank
//      scan (LDS writes, DPP scans) runs under their latency.
// Entries whose B row has more than one group (t >= 1) are appended to a queue in LDS with one
// ds_write each (the generic walker compacts them through registers with two ds_permutes and six
// selects per round), and read back as full 64-lane batches. Word ranks of two bitmap blocks share one DPP scan (16-bit halves).
// The preloaded groups serve a pattern B under the narrow bound (every step of the 30^3 chain, u32
// and Sat64); a row's later segments, later rank chunks and the other value cases walk from memory
// with the generic RowWalker.
#pragma once

namespace slat {

// A entries per lane in a segment: 8 (512 entries) for 4-byte values, 4 for 8-byte ones (registers)
#ifndef SLAT_ST_Q4
#define SLAT_ST_Q4 8
#endif
template <typename S>
constexpr int kStQ = sizeof(S) == 4 ? SLAT_ST_Q4 : 4;
constexpr uint32_t kStBlk = 8;                    // stored bitmap blocks loaded with the A entries
constexpr uint32_t kStTail = 4;                   // tail batches (64 items) held in registers
constexpr uint32_t kStQueue = kStTail * kWave;    // tail items per segment (more: per-entry walk)

// the tail queue's entries in the slot area: (B row << 3 | group, A value)
template <typename S>
struct StItem {
    uint32_t kt;
    uint32_t pad;
    S a;
};

// one rank chunk's accumulate: a group of four columns and their products, rank lookups first, then
// the adds. A column outside [r0, r0 + nch) (another chunk's, or padding) adds into its lane's own
// sink slot (slot sink + lane, past the chunk's slots) instead of taking a branch: the branch cost an
// exec save, a skip and a restore per product (one sink slot for every lane would serialise the
// instruction on its address). FIRST (rank chunk 0, r0 = 0): a rank past the chunk is either past the
// row (padding: 2^31 and up) or, when the row has more chunks, at least cap, so min(rank, sink + lane)
// takes the place of the compare and select: such a rank lands in its own lane's sink slot or in
// another lane's (all of them cleared at the row's end)
template <typename Sem, bool NW, bool FIRST = false>
struct StAcc {
    using S = typename Sem::S;
    using V = typename Sem::V;
    const uint2 *W;
    uint32_t ww;
    void *vals;
    uint16_t *cols;
    uint32_t r0, nch, sink;
    __device__ __forceinline__ void operator()(const uint4 &c, const Quad<S> &pr) const {
        const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
        uint2 w[4];
        sfor<4>([&](auto E) { w[E] = W[min(cc[E] >> 5, ww)]; });
        const uint32_t ls = sink + (uint32_t)lane_id();
        sfor<4>([&](auto E) {
            const uint32_t r = __builtin_popcount(__builtin_amdgcn_ubfe(w[E].x, 0u, cc[E])) + (w[E].y - r0);
            const uint32_t rr = FIRST ? min(r, ls) : r < nch ? r : ls;
            if constexpr (NW)
                atomicAdd((uint32_t *)vals + rr, (uint32_t)pr.v[E]);
            else
                Sem::acc((V *)vals, rr, pr.v[E]);
            cols[rr] = (uint16_t)cc[E];
        });
    }
    __device__ __forceinline__ void multi(const uint4 *c, const Quad<S> *pr) const {
        sfor<kRegQ>([&](auto Q) { (*this)(c[Q], pr[Q]); });
    }
};

template <typename Sem, typename I>
__device__ __forceinline__ void numeric_rows_stored(const Args &p, uint8_t *smem8, int wv, uint64_t first,
                                                    uint64_t stride) {
    using S = typename Sem::S;
    using V = typename Sem::V;
    using Item = std::conditional_t<sizeof(S) == 4, uint2, StItem<S>>;
    constexpr int kQ = kStQ<S>;
    constexpr uint32_t kSeg = kWave * kQ;
    const int lane = lane_id();
    const uint64_t nit = p.nrows;
    const NumLayout lay = num_layout(p.ww, p.area);
    uint8_t *region = smem8 + (size_t)wv * lay.bytes;
    uint2 *W = (uint2 *)region;
    uint8_t *slots = region + lay.off_slots;
    // rank slots per chunk, after kWave sink slots (StAcc) are set aside
    const uint32_t cap_n = p.area / 6 - kWave, cap_w = p.area / (uint32_t)(sizeof(V) * Sem::kSlots + 2) - kWave;
    Item *queue = (Item *)slots;  // kStQueue items + a sink entry, zero again before any slot is used

    uint32_t bvmax = 0xFFFFFFFFu;
    bool buni = false;
    if constexpr (Sem::kNarrowable)
        if (p.b_vmax) {
            const unsigned long long v = ((volatile unsigned long long *)p.b_vmax)[kVMaxWord];
            const unsigned long long vi = ((volatile unsigned long long *)p.b_vmax)[kVMinInvWord];
            if ((uint32_t)(v >> 32) == p.epoch) {
                bvmax = (uint32_t)v;
                buni = SLAT_NUM_UNI && (uint32_t)(vi >> 32) == p.epoch && ~(uint32_t)vi == bvmax &&
                       (sizeof(S) == 4 || bvmax != 0xFFFFFFFFu);
            }
        }
    const S bv0 = (S)bvmax;
    S *cval = (S *)p.c_val;

    for (uint32_t w = lane; w < p.ww; w += kWave) W[w] = make_uint2(0u, 0u);
    if (lane == 0) W[p.ww] = make_uint2(0u, 0x80000000u);  // out-of-window / padding columns: no rank
    for (uint32_t w = lane; w < p.area / 4; w += kWave) ((uint32_t *)slots)[w] = 0;
    wave_sync();

    // the row after this one: lanes 0-1 its A bounds, 2-3 its C slice (bd), lane 4 its stored-block
    // mask (bm), lane 5 its fat mark (fm). Each load sits bare in its branch, into a variable of its
    // own type: a conversion inside the branch made the wave wait for the load there (vmcnt(0), so
    // for every load in flight, the groups included)
    struct Ahead {
        uint64_t bd;
        uint32_t bm;
        uint32_t fm;
    };
    auto ahead = [&](uint64_t r, Ahead &h) {
        h.bd = 0;
        h.bm = 0;
        h.fm = 0;
        if (r < nit) {
            if (lane < 4) h.bd = (lane < 2 ? p.a_rp : (const uint64_t *)p.c_rp)[r + (uint64_t)(lane & 1)];
            if (lane == 4) h.bm = p.smask[r];
            if (lane == 5 && p.fr_mark) h.fm = p.fr_mark[r];
        }
    };

    uint32_t zrows = 0;
    Ahead nxt;
    ahead(first, nxt);
    for (uint64_t row = first; row < nit; row += stride) {
        const I a0 = (I)readlane_u64(nxt.bd, 0), a1 = (I)readlane_u64(nxt.bd, 1);
        const uint64_t ob = readlane_u64(nxt.bd, 2), oe = readlane_u64(nxt.bd, 3);
        const uint32_t bmask = readlane_u32(nxt.bm, 4);
        if (readlane_u32(nxt.fm, 5) != 0) {  // the fat-row kernels' row
            ahead(row + stride, nxt);
            continue;
        }
        uint64_t out_pos = ob;
        uint32_t zeros = 0;
        bool issued = false;  // the next row's bounds are in flight
        if (a1 > a0 && bmask != 0) {
            const uint64_t len = (uint64_t)(a1 - a0);
            const uint32_t seg_n = len < kSeg ? (uint32_t)len : kSeg;
            const S *av_ = (const S *)p.a_val;
            // 2. the first segment's entries and the stored bitmap blocks
            uint32_t kq[kQ], ngq[kQ];
            S aq[kQ];
            {
                const uint32_t *sc = p.a_col + a0;
                const S *sv = av_ + a0;
                sfor<kQ>([&](auto Q) {
                    const uint32_t j = (uint32_t)(Q * kWave + lane);
                    kq[Q] = kSent;
                    aq[Q] = S(0);
                    if (j < seg_n) {
                        kq[Q] = sc[j];
                        aq[Q] = sv[j];
                    }
                });
            }
            uint32_t bs[kStBlk], xs[kStBlk];
            {
                const uint32_t *src = p.sbm + row * ((uint64_t)p.nblk * kWave) + lane;
                uint32_t m = bmask;
                sfor<kStBlk>([&](auto I_) {
                    bs[I_] = m ? (uint32_t)__builtin_ctz(m) : 32u;
                    m &= m - 1;
                    xs[I_] = src[(bs[I_] < 32u ? bs[I_] : 0u) * kWave];  // unconditional: precise waits
                });
            }
            // 3. group counts (malformed ids past B's rows are ignored, as in the generic walker)
            uint32_t amax = 0, mx = 0;
            sfor<kQ>([&](auto Q) {
                if (kq[Q] >= p.b_nrows) kq[Q] = kSent;
                ngq[Q] = kq[Q] != kSent ? p.ell_ng[kq[Q]] : 0u;
            });
            sfor<kQ>([&](auto Q) {
                if constexpr (Sem::kNarrowable) amax = max(amax, sat32(aq[Q]));
                mx = max(mx, ngq[Q]);
            });
            mx = wave_max_u32(mx);
            // the tail items (entry, group t >= 1) into the LDS queue, in (t, q, lane) order
            uint32_t off = 0;
            for (uint32_t t = 1; t < mx; ++t) {
                sfor<kQ>([&](auto Q) {
                    const bool has = ngq[Q] > t;
                    const unsigned long long m = __ballot(has);
                    if (m) {
                        const uint32_t below =
                            __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        // (only the lanes with an item write: lanes writing one sink address would
                        // serialise the instruction)
                        if (has) {
                            Item it;
                            if constexpr (sizeof(S) == 4) {
                                it = make_uint2((kq[Q] << 3) | t, __builtin_bit_cast(uint32_t, aq[Q]));
                            } else {
                                it.kt = (kq[Q] << 3) | t;
                                it.pad = 0;
                                it.a = aq[Q];
                            }
                            queue[min(off + below, kStQueue)] = it;
                        }
                        off += (uint32_t)__popcll(m);
                    }
                });
            }
            const bool ovf = off > kStQueue;  // too many tail items: every entry walks its own groups
            uint32_t tk[kStTail];
            S ta[kStTail];
            if (off) {
                wave_sync();
                sfor<kStTail>([&](auto T) {
                    tk[T] = kSent;
                    ta[T] = S(0);
                    const uint32_t i = (uint32_t)(T * kWave + lane);
                    if (!ovf && i < off) {
                        const Item it = queue[i];
                        if constexpr (sizeof(S) == 4) {
                            tk[T] = it.x;
                            ta[T] = __builtin_bit_cast(S, it.y);
                        } else {
                            tk[T] = it.kt;
                            ta[T] = it.a;
                        }
                    }
                });
                wave_sync();
                const uint32_t used = min(off, kStQueue);
                Item z{};
                for (uint32_t i = lane; i < used; i += kWave) queue[i] = z;
                if (lane == 0) queue[kStQueue] = z;
                wave_sync();
            } else {
                sfor<kStTail>([&](auto T) {
                    tk[T] = kSent;
                    ta[T] = S(0);
                });
            }
            // 4. the segment's ELL column groups (a B that is not a pattern has its values loaded at
            //    the accumulate: registers for both would cost the kernel its third wave per SIMD)
            uint4 cq[kQ], ct[kStTail];
            sfor<kQ>([&](auto Q) {
                cq[Q] = make_uint4(kSent, kSent, kSent, kSent);
                if (kq[Q] != kSent) cq[Q] = ell_cols(p, kq[Q], 0);
            });
            sfor<kStTail>([&](auto T) {
                ct[T] = make_uint4(kSent, kSent, kSent, kSent);
                if (!ovf && tk[T] != kSent) ct[T] = ell_cols(p, tk[T] >> 3, tk[T] & 7u);
            });
            // (the next row's bounds: behind every load of this row's first segment)
            ahead(row + stride, nxt);
            issued = true;
            // word ranks of the stored blocks, two blocks per scan (16-bit halves: a block sums to
            // at most 2048), while the groups are in flight
            uint32_t wcnt = 0;
            const auto plus = [](uint32_t x, uint32_t y) { return x + y; };
            sfor<kStBlk / 2>([&](auto J) {
                constexpr int j0 = 2 * J, j1 = 2 * J + 1;
                if (bs[j0] < 32u) {
                    const uint32_t c0 = __popc(xs[j0]), c1 = bs[j1] < 32u ? __popc(xs[j1]) : 0u;
                    const uint32_t incl = wave_incl_scan(c0 | (c1 << 16), 0u, plus);
                    const uint32_t tot = readlane_u32(incl, kWave - 1);
                    W[bs[j0] * kWave + lane] = make_uint2(xs[j0], wcnt + (incl & 0xFFFFu) - c0);
                    wcnt += tot & 0xFFFFu;
                    if (bs[j1] < 32u) {
                        W[bs[j1] * kWave + lane] = make_uint2(xs[j1], wcnt + (incl >> 16) - c1);
                        wcnt += tot >> 16;
                    }
                }
            });
            {  // blocks past the first kStBlk (rows touching more of the window)
                uint32_t m = bmask;
                sfor<kStBlk>([&](auto) { m &= m - 1; });
                const uint32_t *src = p.sbm + row * ((uint64_t)p.nblk * kWave) + lane;
                for (; m; m &= m - 1) {
                    const uint32_t b = (uint32_t)__builtin_ctz(m);
                    const uint32_t x = src[b * kWave];
                    const uint32_t c = __popc(x);
                    const uint32_t incl = wave_incl_scan(c, 0u, plus);
                    W[b * kWave + lane] = make_uint2(x, wcnt + incl - c);
                    wcnt += readlane_u32(incl, kWave - 1);
                }
            }
            wave_sync();
            // narrow u32 slots when no sum can reach 2^32: max(A row) * max(B) * len(A row) < 2^32
            bool narrow = false;
            if constexpr (Sem::kNarrowable) {
                if (bvmax != 0xFFFFFFFFu) {
                    for (I j = a0 + (I)kSeg + (I)lane; j < a1; j += (I)kWave) amax = max(amax, sat32(av_[j]));
                    const uint32_t wam = wave_max_u32(amax);
                    const uint64_t x = (uint64_t)wam * bvmax;
                    narrow = (sizeof(S) == 4 || wam != 0xFFFFFFFFu) && (x == 0 || len <= 0xFFFFFFFFull / x);
                }
            }

            // Pattern B under the narrow bound (every step of the 30^3 chain, u32 and Sat64): the first
            // segment's groups come from the registers loaded above. Everything else (a B with other
            // values, rows that may reach 2^32, a row's later segments, rank chunks after the first)
            // walks from memory with the generic walker: registers for both would spill.
            auto run = [&](auto narrow_tag, auto uni_tag) {
                constexpr bool NW = decltype(narrow_tag)::value;
                constexpr bool UNI = decltype(uni_tag)::value;
                constexpr bool PRE = NW && UNI;
                using VS = std::conditional_t<NW, uint32_t, V>;
                constexpr uint32_t kVW = NW ? 1 : Sem::kSlots;
                using PS = std::conditional_t<NW, SemNarrowT<S>, Sem>;
                const uint32_t cap = NW ? cap_n : cap_w;
                VS *vals = (VS *)slots;  // cap slots, then the kWave sink slots
                uint16_t *cols = (uint16_t *)(slots + (size_t)(cap + kWave) * kVW * sizeof(VS));
                // emit of one chunk at the row's slice, coalesced, already sorted; the slots are left zero
                auto emit = [&](uint32_t nch) {
                    wave_sync();
                    uint32_t *oc = p.c_col + out_pos;
                    S *ov = cval + out_pos;
                    const uint32_t lim = (uint32_t)min<uint64_t>(oe - min(out_pos, oe), nch);
                    for (uint32_t t = lane; t < nch; t += kWave) {
                        S v;
                        if constexpr (NW)
                            v = (S)vals[t];
                        else
                            v = Sem::finish((const V *)vals, t);
                        const uint32_t col = cols[t];
#pragma unroll
                        for (uint32_t w = 0; w < kVW; ++w) vals[t * kVW + w] = VS(0);
                        cols[t] = 0;
                        zeros += Sem::is_zero(v) ? 1u : 0u;
                        if (t < lim) {  // never write past the row's slice
                            oc[t] = col;
                            ov[t] = v;
                        }
                    }
                    out_pos += nch;
                    wave_sync();
                };
                // the entries [from, a1) walked from memory into rank chunk [r0, r0 + nch)
                auto walk = [&](const auto &acc, I from) {
                    if (from < a1) {
                        RowWalker<Sem, I, true, true> rw(p, from, a1);
                        rw.template each_group<true, PS, UNI>(acc, bv0);
                    }
                };
                uint32_t r0 = 0;
                if constexpr (PRE) {
                    // chunk 0 (peeled: in a loop the compiler hoists all 48 groups' rank addresses out of
                    // it and spills them)
                    const uint32_t nch = min(cap, wcnt);
                    const StAcc<Sem, NW, true> acc{W, p.ww, vals, cols, 0u, nch, cap};
                    sfor<kQ>([&](auto Q) {
                        if (Q * kWave < seg_n) acc(cq[Q], splat4(PS::prod(aq[Q], bv0)));
                    });
                    if (!ovf) {
                        sfor<kStTail>([&](auto T) {
                            if (T * kWave < off) acc(ct[T], splat4(PS::prod(ta[T], bv0)));
                        });
                    } else {
                        // (a full first group: the B row may have more; an empty next group ends the walk)
                        sfor<kQ>([&](auto Q) {
                            if (cq[Q].w != kSent)
                                walk_brow<PS, true, false, I>(p, kq[Q], aq[Q], 1, [&](uint4 c, const Quad<S> &) {
                                    acc(c, splat4(PS::prod(aq[Q], bv0)));
                                });
                        });
                    }
                    walk(acc, a0 + (I)seg_n);
                    emit(nch);
                    r0 = cap;
                }
                for (; r0 < wcnt; r0 += cap) {
                    const uint32_t nch = min(cap, wcnt - r0);
                    walk(StAcc<Sem, NW>{W, p.ww, vals, cols, r0, nch, cap}, a0);
                    emit(nch);
                }
                // the lane's sink slot back to zero: the next row may take the other slot layout (narrow
                // or wide), whose value slots overlap these bytes
#pragma unroll
                for (uint32_t w = 0; w < kVW; ++w) vals[(cap + (uint32_t)lane) * kVW + w] = VS(0);
                cols[cap + (uint32_t)lane] = 0;
                wave_sync();
            };
#ifdef SLAT_ST_ONLY
            if constexpr (Sem::kNarrowable) run(std::bool_constant<SLAT_ST_ONLY / 2>{}, std::bool_constant<SLAT_ST_ONLY % 2>{}); else
#endif
            if constexpr (Sem::kNarrowable) {
                if (narrow && buni)
                    run(std::true_type{}, std::true_type{});
                else if (narrow)
                    run(std::true_type{}, std::false_type{});
                else if (buni)
                    run(std::false_type{}, std::true_type{});
                else
                    run(std::false_type{}, std::false_type{});
            } else {
                run(std::false_type{}, std::false_type{});
            }
        }
        if (!issued) ahead(row + stride, nxt);
        const uint32_t rz = wave_sum_u32(zeros);
        if (lane == 0) p.counts[row] = out_pos - ob - rz;
        zrows += rz ? 1u : 0u;
    }
    add_zero_rows(&p.host_out[2], zrows, p.seq != 0);
}

// ------------------------------------------------------------------------------------------------
// k_symbolic MODE 4: the symbolic pass of the same launches (single window, stored bitmaps, B's ELL
// image). Per segment of up to 64 * kSymQ A entries: the entries, their group counts, the tail
// groups appended to an LDS queue (one ds_write each, instead of the register compaction's two
// ds_permutes and six selects per round), every group's columns loaded at once, then one ds_or per
// column with no branch (the padding ORs into its lane's sink word past the window). The row's count is the
// popcount of its touched 64-word blocks, which are stored for the numeric pass with their mask.
// LDS per wave: the window's words, 64 sink words, then the queue (sym_stored_words).
// ------------------------------------------------------------------------------------------------
constexpr int kSymQ = 4;                        // A entries per lane in a segment (256 per segment)
constexpr uint32_t kSymTail = 2;                // tail batches per segment held in registers
constexpr uint32_t kSymQueue = kSymTail * kWave;

// the window's words, 64 sink words (a padding column ORs into its lane's own: one shared sink word
// serialised every instruction with padding), the queue and its sink entry
__host__ __device__ constexpr uint32_t sym_stored_words(uint32_t ww) { return ((ww + kWave + 3) & ~3u) + kSymQueue + 4; }

template <typename I>
__device__ __forceinline__ void symbolic_rows_stored(const Args &p, uint32_t *smem, int wv, uint64_t first,
                                                     uint64_t stride, uint64_t &mx, unsigned long long &flops) {
    constexpr uint32_t kSeg = kWave * kSymQ;
    const int lane = lane_id();
    const uint64_t nit = p.nrows;
    const uint32_t ww = p.ww;
    uint32_t *L0 = smem + (size_t)wv * sym_stored_words(ww);
    uint32_t *queue = L0 + ((ww + kWave + 3) & ~3u);  // kSymQueue items + a sink entry
    const uint32_t blk_ok = p.nblk >= 32 ? 0xFFFFFFFFu : (1u << p.nblk) - 1;  // (the padding's bit 31)
    for (uint32_t w = lane; w < ww + kWave; w += kWave) L0[w] = 0;
    wave_sync();
    // the next row's A bounds (lanes 0-1) and fat mark (lane 2), each load bare in its branch
    uint64_t nb = 0;
    uint32_t nf = 0;
    auto ahead = [&](uint64_t r) {
        nb = 0;
        nf = 0;
        if (r < nit) {
            if (lane < 2) nb = p.a_rp[r + (uint64_t)lane];
            if (lane == 2 && p.fr_mark) nf = p.fr_mark[r];
        }
    };
    ahead(first);
    for (uint64_t row = first; row < nit; row += stride) {
        const I a0 = (I)readlane_u64(nb, 0), a1 = (I)readlane_u64(nb, 1);
        const bool fat = readlane_u32(nf, 2) != 0;
        ahead(row + stride);
        if (fat) continue;  // the fat-row kernels' row
        uint32_t blk = 0, nprod = 0;
        for (I sb = a0; sb < a1; sb += (I)kSeg) {
            const uint64_t rest = (uint64_t)(a1 - sb);
            const uint32_t sn = rest < kSeg ? (uint32_t)rest : kSeg;
            uint32_t kq[kSymQ], ngq[kSymQ];
            const uint32_t *sc = p.a_col + sb;
            sfor<kSymQ>([&](auto Q) {
                const uint32_t j = (uint32_t)(Q * kWave + lane);
                kq[Q] = j < sn ? sc[j] : kSent;
            });
            uint32_t mxg = 0;
            sfor<kSymQ>([&](auto Q) {
                if (kq[Q] >= p.b_nrows) kq[Q] = kSent;  // malformed input: ignore the entry
                ngq[Q] = kq[Q] != kSent ? p.ell_ng[kq[Q]] : 0u;
            });
            sfor<kSymQ>([&](auto Q) { mxg = max(mxg, ngq[Q]); });
            mxg = wave_max_u32(mxg);
            uint32_t off = 0;
            for (uint32_t t = 1; t < mxg; ++t) {
                sfor<kSymQ>([&](auto Q) {
                    const bool has = ngq[Q] > t;
                    const unsigned long long m = __ballot(has);
                    if (m) {
                        const uint32_t below =
                            __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        if (has) queue[min(off + below, kSymQueue)] = (kq[Q] << 3) | t;
                        off += (uint32_t)__popcll(m);
                    }
                });
            }
            const bool ovf = off > kSymQueue;
            uint32_t tk[kSymTail];
            if (off) wave_sync();
            sfor<kSymTail>([&](auto T) {
                const uint32_t i = (uint32_t)(T * kWave + lane);
                tk[T] = !ovf && i < off ? queue[i] : kSent;
            });
            uint4 cq[kSymQ], ct[kSymTail];
            sfor<kSymQ>([&](auto Q) {
                cq[Q] = make_uint4(kSent, kSent, kSent, kSent);
                if (kq[Q] != kSent) cq[Q] = ell_cols(p, kq[Q], 0);
            });
            sfor<kSymTail>([&](auto T) {
                ct[T] = make_uint4(kSent, kSent, kSent, kSent);
                if (tk[T] != kSent) ct[T] = ell_cols(p, tk[T] >> 3, tk[T] & 7u);
            });
            auto bits = [&](const uint4 &c) {
                const uint32_t cc[4] = {c.x, c.y, c.z, c.w};
                sfor<4>([&](auto E) {
                    const uint32_t wd = cc[E] >> 5;
                    // (a padding column's word is past ww + 63: min sends it to the lane's sink word)
                    atomicOr(&L0[min(wd, ww + (uint32_t)lane)], 1u << (cc[E] & 31));
                    blk |= 1u << ((cc[E] >> 11) & 31);
                });
            };
            // the product count for the stats, outside the bit loop: a predicated count inside it
            // costs three VALU per slot even when no stats are asked for
            auto live = [](const uint4 &c) {
                return (uint32_t)(c.x != kSent) + (c.y != kSent) + (c.z != kSent) + (c.w != kSent);
            };
            sfor<kSymQ>([&](auto Q) {
                if (Q * kWave < sn) bits(cq[Q]);
            });
            sfor<kSymTail>([&](auto T) {
                if (T * kWave < off) bits(ct[T]);
            });
            if (p.stats) {  // launch-uniform branch
                sfor<kSymQ>([&](auto Q) { nprod += live(cq[Q]); });
                sfor<kSymTail>([&](auto T) { nprod += live(ct[T]); });
            }
            if (ovf)  // more tail groups than the queue: each entry walks its own
                sfor<kSymQ>([&](auto Q) {
                    if (cq[Q].w != kSent)
                        walk_brow<SemNone, true, false, I>(p, kq[Q], 0u, 1, [&](uint4 c, const Quad<uint32_t> &) {
                            bits(c);
                            if (p.stats) nprod += live(c);
                        });
                });
        }
        wave_sync();
        // the row's count: popcount of its touched blocks (word b * 64 + lane per lane), stored for
        // the numeric pass and cleared
        const uint32_t bmask = wave_or_u32(blk) & blk_ok;
        uint32_t *keep = p.sbm + row * ((uint64_t)p.nblk * kWave);
        if (lane == 0) p.smask[row] = bmask;
        uint32_t lc = 0;
        for (uint32_t m = bmask; m; m &= m - 1) {
            const uint32_t w = (uint32_t)__builtin_ctz(m) * kWave + lane;
            const uint32_t x = L0[w];
            lc += __popc(x);
            L0[w] = 0;
            keep[w] = x;
        }
        const uint64_t cnt = wave_sum_u32(lc);
        if (p.stats) flops += wave_sum_u32(nprod);
        if (lane == 0) p.counts[row] = cnt;
        mx = max(mx, cnt);
        wave_sync();
    }
}

}  // namespace slat
