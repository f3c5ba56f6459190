// slat_num.hip — the numeric kernel instances of ONE value semiring (-DSLAT_SEM=id, slat_launch.hpp):
// the Makefile compiles this file once per semiring, so the instances build in parallel.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "slat_launch.hpp"
#include "spgemm_kernels.hpp"

#ifndef SLAT_SEM
#error "compile with -DSLAT_SEM=<semiring id>"
#endif

using namespace slat;

namespace {
using Sem = std::conditional_t<SLAT_SEM == kSemU32, SemU32,
            std::conditional_t<SLAT_SEM == kSemSat64, SemSat64,
            std::conditional_t<SLAT_SEM == kSemF64, SemF64, SemF64Any>>>;

// the instance of (mode, offsets, B form); F(kernel) is called with its function pointer
template <typename F>
hipError_t with_instance(int mode, bool idx32, bool ell, F &&f) {
    if (mode == 3) {  // batched short rows (integer semirings and f64 in any order; B as ELL or CSR)
        if constexpr (std::is_same_v<Sem, SemU32>)
            return idx32 ? (ell ? f(k_numeric_short_u32<uint32_t, false>) : f(k_numeric_short_u32<uint32_t, true>))
                         : (ell ? f(k_numeric_short_u32<uint64_t, false>) : f(k_numeric_short_u32<uint64_t, true>));
        else if constexpr (!Sem::kOrdered)
            return idx32 ? (ell ? f(k_numeric_short<Sem, uint32_t, false>) : f(k_numeric_short<Sem, uint32_t, true>))
                         : (ell ? f(k_numeric_short<Sem, uint64_t, false>) : f(k_numeric_short<Sem, uint64_t, true>));
        else
            return hipErrorInvalidValue;
    }
    // wide launches: the hash category (mode 1) and the window category (mode 2) are instances of
    // their own, so neither path's registers burden the other
    if (mode == 1)
        return idx32 ? (ell ? f(k_numeric<Sem, uint32_t, true, 1>) : f(k_numeric<Sem, uint32_t, false, 1>))
                     : (ell ? f(k_numeric<Sem, uint64_t, true, 1>) : f(k_numeric<Sem, uint64_t, false, 1>));
    if (mode == 4) {  // single-window launches with stored bitmaps and B's ELL image (unordered semirings)
        if constexpr (!Sem::kOrdered)
            return idx32 ? f(k_numeric<Sem, uint32_t, true, 4>) : f(k_numeric<Sem, uint64_t, true, 4>);
        else
            return hipErrorInvalidValue;
    }
    if (mode == 2)
        return idx32 ? (ell ? f(k_numeric<Sem, uint32_t, true, 2>) : f(k_numeric<Sem, uint32_t, false, 2>))
                     : (ell ? f(k_numeric<Sem, uint64_t, true, 2>) : f(k_numeric<Sem, uint64_t, false, 2>));
    return idx32 ? (ell ? f(k_numeric<Sem, uint32_t, true>) : f(k_numeric<Sem, uint32_t, false>))
                 : (ell ? f(k_numeric<Sem, uint64_t, true>) : f(k_numeric<Sem, uint64_t, false>));
}
}  // namespace

template <>
hipError_t slat_launch_numeric_t<SLAT_SEM>(int mode, bool idx32, bool ell, dim3 grid, size_t lds, hipStream_t s,
                                           const Args &a) {
    return with_instance(mode, idx32, ell, [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(kBlock), lds, s, a);
        return hipGetLastError();
    });
}

template <>
int slat_numeric_blocks_per_cu_t<SLAT_SEM>(int mode, bool idx32, bool ell, size_t lds) {
    // cached per (instance, LDS size): the query costs microseconds of host time per call
    static thread_local int cache_nb[32] = {};
    static thread_local size_t cache_lds[32] = {};
    const int ci = (idx32 ? 1 : 0) | (ell ? 2 : 0) | (mode << 2);
    if (cache_lds[ci] == lds && cache_nb[ci] > 0) return cache_nb[ci];
    int nb = 0;
    const hipError_t e = with_instance(mode, idx32, ell, [&](auto kern) {
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, kBlock, lds);
    });
    nb = (e == hipSuccess && nb > 0) ? nb : 1;
    cache_lds[ci] = lds;
    cache_nb[ci] = nb;
    return nb;
}
