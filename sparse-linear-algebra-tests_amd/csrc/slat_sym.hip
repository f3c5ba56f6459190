// slat_sym.hip — the symbolic kernel instances (slat_launch.hpp), in a translation unit of their own
// so they build beside the numeric ones.
#include <hip/hip_runtime.h>

#include "slat_launch.hpp"
#include "spgemm_kernels.hpp"

using namespace slat;

hipError_t slat_launch_symbolic(int mode, bool idx32, bool ell, dim3 grid, size_t lds, hipStream_t s, const Args &a) {
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(kBlock), lds, s, a);
        return hipGetLastError();
    };
    if (mode == 1)
        return idx32 ? (ell ? go(k_symbolic<uint32_t, true, 1>) : go(k_symbolic<uint32_t, false, 1>))
                     : (ell ? go(k_symbolic<uint64_t, true, 1>) : go(k_symbolic<uint64_t, false, 1>));
    if (mode == 4)  // single-window launches with stored bitmaps and B's ELL image (spgemm_stored.hpp)
        return ell ? (idx32 ? go(k_symbolic<uint32_t, true, 4>) : go(k_symbolic<uint64_t, true, 4>)) : hipErrorInvalidValue;
    if (mode == 2)
        return idx32 ? (ell ? go(k_symbolic<uint32_t, true, 2>) : go(k_symbolic<uint32_t, false, 2>))
                     : (ell ? go(k_symbolic<uint64_t, true, 2>) : go(k_symbolic<uint64_t, false, 2>));
    return idx32 ? (ell ? go(k_symbolic<uint32_t, true>) : go(k_symbolic<uint32_t, false>))
                 : (ell ? go(k_symbolic<uint64_t, true>) : go(k_symbolic<uint64_t, false>));
}

hipError_t slat_launch_symbolic_short(bool idx32, bool ell, dim3 grid, size_t lds, hipStream_t s, const Args &a) {
    if (idx32) {
        if (ell)
            hipLaunchKernelGGL((k_symbolic_short<uint32_t, false>), grid, dim3(kBlock), lds, s, a);
        else
            hipLaunchKernelGGL((k_symbolic_short<uint32_t, true>), grid, dim3(kBlock), lds, s, a);
    } else {
        if (ell)
            hipLaunchKernelGGL((k_symbolic_short<uint64_t, false>), grid, dim3(kBlock), lds, s, a);
        else
            hipLaunchKernelGGL((k_symbolic_short<uint64_t, true>), grid, dim3(kBlock), lds, s, a);
    }
    return hipGetLastError();
}

int slat_symbolic_short_blocks_per_cu(bool idx32, bool ell, size_t lds) {
    static thread_local int cache_nb[4] = {};
    static thread_local size_t cache_lds[4] = {};
    const int ci = (idx32 ? 1 : 0) | (ell ? 2 : 0);
    if (cache_lds[ci] == lds && cache_nb[ci] > 0) return cache_nb[ci];
    int nb = 0;
    hipError_t e;
    if (idx32)
        e = ell ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_symbolic_short<uint32_t, false>, kBlock, lds)
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_symbolic_short<uint32_t, true>, kBlock, lds);
    else
        e = ell ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_symbolic_short<uint64_t, false>, kBlock, lds)
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_symbolic_short<uint64_t, true>, kBlock, lds);
    nb = (e == hipSuccess && nb > 0) ? nb : 1;
    cache_lds[ci] = lds;
    cache_nb[ci] = nb;
    return nb;
}

int slat_symbolic_listed_blocks_per_cu(bool idx32, bool ell, size_t lds) {
    static thread_local int cache_nb[4] = {};
    static thread_local size_t cache_lds[4] = {};
    const int ci = (idx32 ? 1 : 0) | (ell ? 2 : 0);
    if (cache_lds[ci] == lds && cache_nb[ci] > 0) return cache_nb[ci];
    int nb = 0;
    auto q = [&](auto kern) { return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, kBlock, lds); };
    const hipError_t e = idx32 ? (ell ? q(k_symbolic<uint32_t, true, 2>) : q(k_symbolic<uint32_t, false, 2>))
                               : (ell ? q(k_symbolic<uint64_t, true, 2>) : q(k_symbolic<uint64_t, false, 2>));
    nb = (e == hipSuccess && nb > 0) ? nb : 1;
    cache_lds[ci] = lds;
    cache_nb[ci] = nb;
    return nb;
}
