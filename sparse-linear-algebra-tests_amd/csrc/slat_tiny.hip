// slat_tiny.hip — the whole SpGEMM in ONE kernel for small products (SURVEY.md §8(d) config C3's
// small cells: 5^3 .. 10^3 tori, ~100 .. 1000 rows), where the regular pipeline's five launches
// (ELL build, symbolic, scan, numeric, completion word) cost more than the work: each launch is a
// few microseconds of host time and a few of dispatch on the device.
//
// k_tiny: a cooperative grid (every block resident, at most one per CU), one wavefront per row:
//   1. symbolic: sym_row's bitmap count of each row (B walked in CSR form: no ELL image to build);
//   2. a grid barrier (a monotonic arrival counter, so nothing is reset between calls);
//   3. every block scans all row counts (<= kTinyRows, u32 sums: nnz(C) < 2^32 at this size) and
//      writes the whole row_ptr itself — identical values from every block, so no second barrier
//      is needed before a block reads the offsets of its rows;
//   4. numeric: numeric_rows' bitmap / rank / accumulate / emit of each row (its non-zero counts go
//      to a second array: other blocks may still be reading the symbolic counts);
//   5. the last block stores the call's completion word (signal_done).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "slat_launch.hpp"
#include "spgemm_kernels.hpp"

using namespace slat;

namespace {

template <typename Sem>
__global__ __launch_bounds__(kBlock) void k_tiny(Args p, uint64_t *counts2, unsigned long long *bar,
                                                 unsigned long long target) {
    using I = uint32_t;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
    constexpr int kWpb = kBlock / kWave;
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint64_t gw = (uint64_t)blockIdx.x * kWpb + wv, nw = (uint64_t)gridDim.x * kWpb;
    const uint64_t n = p.nrows;
    // 1. symbolic counts
    {
        uint32_t *L0 = (uint32_t *)smem8 + (size_t)wv * p.ww;
        for (uint32_t w = lane; w < p.ww; w += kWave) L0[w] = 0;
        wave_sync();
        unsigned long long flops = 0;
        for (uint64_t row = gw; row < n; row += nw) {
            const uint64_t cnt = sym_row<I, false, 0>(p, row, false, L0, flops);
            if (lane == 0) p.counts[row] = cnt;
        }
    }
    // 2. every block's counts are out before any block scans them
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        atomicAdd(bar, 1ull);
        // bounded: a counter out of step with the host's count (which no correct call leaves)
        // ends the kernel with a trap after 2 s instead of hanging the device
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
        while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) __builtin_trap();
        }
        __threadfence();
    }
    __syncthreads();
    // 3. row_ptr: thread t sums rows [t * per, (t + 1) * per), then a block scan of the sums
    {
        uint32_t *sh = (uint32_t *)smem8;  // wave totals
        const uint64_t per = (n + kBlock - 1) / kBlock;
        const uint64_t r0 = min<uint64_t>(n, threadIdx.x * per), r1 = min<uint64_t>(n, r0 + per);
        uint32_t sum = 0, mx = 0;
        for (uint64_t r = r0; r < r1; ++r) {
            const uint32_t c = (uint32_t)p.counts[r];
            sum += c;
            mx = max(mx, c);
        }
        const uint32_t incl = wave_incl_scan(sum, 0u, [](uint32_t x, uint32_t y) { return x + y; });
        mx = wave_max_u32(mx);
        if (lane == kWave - 1) sh[wv] = incl;
        if (lane == 0) sh[kWpb + wv] = mx;
        __syncthreads();
        uint32_t base = 0, tot = 0, mxa = 0;
#pragma unroll
        for (int w = 0; w < kWpb; ++w) {
            base += w < wv ? sh[w] : 0u;
            tot += sh[w];
            mxa = max(mxa, sh[kWpb + w]);
        }
        uint64_t run = base + incl - sum;
        if (threadIdx.x == 0) p.c_rp[0] = 0;
        for (uint64_t r = r0; r < r1; ++r) {
            run += (uint32_t)p.counts[r];
            p.c_rp[r + 1] = run;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            // nnz and the max row for the host; returned values, so both have landed before this
            // block reports done
            const unsigned long long o0 =
                __hip_atomic_exchange(&p.host_out[0], (unsigned long long)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const unsigned long long o1 =
                __hip_atomic_exchange(&p.host_out[1], (unsigned long long)mxa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            asm volatile("" ::"v"(o0), "v"(o1));
        }
        __threadfence_block();
        __syncthreads();
    }
    // 4. numeric, 5. completion word
    Args q = p;
    q.counts = counts2;
    numeric_rows<Sem, I, false, 0>(q, smem8, wv, gw, nw);
    signal_done(q);
}

template <typename Sem>
hipError_t launch(dim3 grid, size_t lds, hipStream_t s, const Args &a, uint64_t *counts2, unsigned long long *bar,
                  unsigned long long target) {
    Args aa = a;
    void *args[] = {&aa, &counts2, &bar, &target};
    return hipLaunchCooperativeKernel((const void *)k_tiny<Sem>, grid, dim3(kBlock), args, (unsigned)lds, s);
}

}  // namespace

hipError_t slat_launch_tiny(int sem, dim3 grid, size_t lds, hipStream_t s, const Args &a, uint64_t *counts2,
                            unsigned long long *bar, unsigned long long target) {
    switch (sem) {
    case kSemU32: return launch<SemU32>(grid, lds, s, a, counts2, bar, target);
    case kSemSat64: return launch<SemSat64>(grid, lds, s, a, counts2, bar, target);
    case kSemF64: return launch<SemF64>(grid, lds, s, a, counts2, bar, target);
    default: return launch<SemF64Any>(grid, lds, s, a, counts2, bar, target);
    }
}
