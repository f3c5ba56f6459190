// graph_kernels.hpp — gfx950 device code for the reference's SpGEMM consumers (SURVEY.md §8(f)
// rank 1): element-wise C = A + B (CsrMatrix::add, src/graph_csr.rs:487-542), the pattern
// equality test of power_until_stable (:567-569) and the component labels of
// connected_components (:580-603). All of them are one wavefront per row, HBM/L2-latency bound
// (binary searches in the other operand's row), no LDS.
#pragma once
#include "spgemm_kernels.hpp"

namespace slat {

// first position p in col[s, e) with col[p] >= c (e if none)
__device__ __forceinline__ uint64_t lower_bound_col(const uint32_t *col, uint64_t s, uint64_t e, uint32_t c) {
    while (s < e) {
        const uint64_t mid = s + ((e - s) >> 1);
        if (col[mid] < c)
            s = mid + 1;
        else
            e = mid;
    }
    return s;
}

// `sadd` of the reference per value type: Saturating<u32> (src/graph_csr.rs:29-32), Sat64
// (src/graph_sprs.rs:29-36), plain f64 `+` (linalg/src/csr.rs:81-85; no FMA involved)
__device__ __forceinline__ uint32_t sat_add(uint32_t a, uint32_t b) {
    const unsigned long long t = (unsigned long long)a + b;
    return t > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)t;
}
__device__ __forceinline__ unsigned long long sat_add(unsigned long long a, unsigned long long b) {
    const unsigned long long t = a + b;
    return t < a ? ~0ull : t;
}
__device__ __forceinline__ double sat_add(double a, double b) { return __dadd_rn(a, b); }

// C = A + B, one wavefront per row, as a sorted union without a serial merge: every entry finds
// its partner (or insertion point) in the other row by binary search, and its output position is
//   A entry i:  (A entries before i that survive) + (B-only entries with a smaller column)
//   B entry j:  (B-only entries before j)        + (A entries with a smaller column that survive)
// from wave scans of the `matched` and `matched with a zero sum` flags. Equal columns combine with
// sat_add and are dropped when the sum is exactly zero (the reference's `if v != 0`); unmatched
// entries are copied as they are. COUNT: exact row lengths into counts[]; else fill C's rows.
template <typename S, bool COUNT>
__global__ __launch_bounds__(kBlock) void k_add(const uint64_t *arp, const uint32_t *acol, const S *aval,
                                                const uint64_t *brp, const uint32_t *bcol, const S *bval,
                                                uint64_t n, uint64_t *counts, const uint64_t *crp, uint32_t *ccol,
                                                S *cval) {
    constexpr int kWpb = kBlock / kWave;
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    for (uint64_t r = (uint64_t)blockIdx.x * kWpb + wv; r < n; r += (uint64_t)gridDim.x * kWpb) {
        const uint64_t as = arp[r], ae = arp[r + 1], bs = brp[r], be = brp[r + 1];
        const uint64_t out = COUNT ? 0 : crp[r];
        uint64_t mc = 0, zc = 0;  // matches / zero sums among the entries of earlier chunks
        for (uint64_t base = as; base < ae; base += kWave) {
            const uint64_t i = base + lane;
            uint32_t m = 0, z = 0, c = 0;
            uint64_t lb = bs;
            S v = S(0);
            if (i < ae) {
                c = acol[i];
                v = aval[i];
                lb = lower_bound_col(bcol, bs, be, c);
                if (lb < be && bcol[lb] == c) {
                    m = 1;
                    v = sat_add(v, bval[lb]);
                    z = v == S(0);
                }
            }
            const uint32_t mx = wave_excl_scan_u32(m), zx = wave_excl_scan_u32(z);
            if (!COUNT && i < ae && !z) {
                const uint64_t pos = (i - as) - (zc + zx) + (lb - bs) - (mc + mx);
                ccol[out + pos] = c;
                cval[out + pos] = v;
            }
            mc += wave_sum_u32(m);
            zc += wave_sum_u32(z);
        }
        if constexpr (COUNT) {
            if (lane == 0) counts[r] = (ae - as) + (be - bs) - mc - zc;
        } else {
            mc = zc = 0;
            for (uint64_t base = bs; base < be; base += kWave) {
                const uint64_t j = base + lane;
                uint32_t m = 0, z = 0, c = 0;
                uint64_t la = as;
                if (j < be) {
                    c = bcol[j];
                    la = lower_bound_col(acol, as, ae, c);
                    if (la < ae && acol[la] == c) {
                        m = 1;
                        z = sat_add(aval[la], bval[j]) == S(0);
                    }
                }
                const uint32_t mx = wave_excl_scan_u32(m), zx = wave_excl_scan_u32(z);
                if (j < be && !m) {
                    const uint64_t pos = (j - bs) - (mc + mx) + (la - as) - (zc + zx);
                    ccol[out + pos] = c;
                    cval[out + pos] = bval[j];
                }
                mc += wave_sum_u32(m);
                zc += wave_sum_u32(z);
            }
        }
    }
}

// identity n x n with values 1 (CsrMatrix::identity, src/graph_csr.rs:68-80)
template <typename S>
__global__ __launch_bounds__(kBlock) void k_identity(uint64_t n, uint64_t *rp, uint32_t *col, S *val) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i <= n; i += (uint64_t)gridDim.x * kBlock) {
        rp[i] = i;
        if (i < n) {
            col[i] = (uint32_t)i;
            val[i] = S(1);
        }
    }
}

// any difference between two u64 / u32 arrays of the same length sets *flag (mapped host word)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_diff(const T *a, const T *b, uint64_t len, unsigned long long *flag) {
    bool d = false;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < len; i += (uint64_t)gridDim.x * kBlock)
        d |= a[i] != b[i];
    if (__ballot(d) && lane_id() == 0)
        __hip_atomic_store(flag, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// connected_components on the closure K of A + I (src/graph_csr.rs:580-603). The reference gives
// node i the id of the smallest j with K(i,j) > 0 and K(j,i) > 0 (mutual reachability is an
// equivalence once K is transitively closed, so no label is ever overwritten), ids numbered in
// order of those smallest members. Here: low[i] = that smallest j (one wave per row, K's row i in
// ascending chunks, each candidate j <= i checked by a binary search of row j for i; the diagonal
// ends the search at the latest), root[i] = (low[i] == i); ids = exclusive scan of root, read at low.
__global__ __launch_bounds__(kBlock) void k_cc_low(const uint64_t *rp, const uint32_t *col, uint64_t n,
                                                   uint32_t *low, uint64_t *root) {
    constexpr int kWpb = kBlock / kWave;
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    for (uint64_t i = (uint64_t)blockIdx.x * kWpb + wv; i < n; i += (uint64_t)gridDim.x * kWpb) {
        const uint64_t s = rp[i], e = rp[i + 1];
        uint32_t best = (uint32_t)i;
        for (uint64_t base = s; base < e; base += kWave) {
            const uint64_t t = base + lane;
            bool hit = false;
            uint32_t j = 0xFFFFFFFFu;
            if (t < e) {
                j = col[t];
                if (j <= i) {
                    const uint64_t js = rp[j], je = rp[j + 1];
                    const uint64_t p = lower_bound_col(col, js, je, (uint32_t)i);
                    hit = p < je && col[p] == (uint32_t)i;
                }
            }
            const unsigned long long m = __ballot(hit);
            if (m) {  // columns ascend with the lane: the lowest hit lane holds the smallest j
                best = readlane_u32(j, (int)__builtin_ctzll(m));
                break;
            }
            if (readlane_u32(j, kWave - 1) >= (uint32_t)i) break;  // past the diagonal
        }
        if (lane == 0) {
            low[i] = best;
            root[i] = best == (uint32_t)i ? 1u : 0u;
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_cc_label(const uint32_t *low, const uint64_t *ids, uint64_t n,
                                                     uint64_t *comp) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
        comp[i] = ids[low[i]];
}

}  // namespace slat
