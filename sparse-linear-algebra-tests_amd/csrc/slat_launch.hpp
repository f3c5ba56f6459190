// slat_launch.hpp — launchers of the SpGEMM kernel instances. The numeric instances of one value
// semiring live in one translation unit (slat_num.hip, compiled once per semiring with -DSLAT_SEM=id)
// and the symbolic ones in slat_sym.hip, so the library's kernels build in parallel.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace slat {
struct Args;
}

// value semirings by id (the SLAT_SEM of each slat_num.hip object)
enum { kSemU32 = 0, kSemSat64 = 1, kSemF64 = 2, kSemF64Any = 3, kSemCount = 4 };

// numeric launch modes: 0 every row by bitmap windows; 1 one row per LDS hash table; 2 the listed
// (window-category) rows of a wide launch; 3 batched short rows (integer semirings, ELL B); 4 every row
// of a single-window launch with stored bitmaps and B's ELL image (unordered semirings)
template <int SEM>
hipError_t slat_launch_numeric_t(int mode, bool idx32, bool ell, dim3 grid, size_t lds, hipStream_t s,
                                 const slat::Args &a);
// resident 256-thread blocks per CU of that numeric instance at `lds` bytes (cached per thread)
template <int SEM>
int slat_numeric_blocks_per_cu_t(int mode, bool idx32, bool ell, size_t lds);

template <> hipError_t slat_launch_numeric_t<kSemU32>(int, bool, bool, dim3, size_t, hipStream_t, const slat::Args &);
template <> hipError_t slat_launch_numeric_t<kSemSat64>(int, bool, bool, dim3, size_t, hipStream_t, const slat::Args &);
template <> hipError_t slat_launch_numeric_t<kSemF64>(int, bool, bool, dim3, size_t, hipStream_t, const slat::Args &);
template <> hipError_t slat_launch_numeric_t<kSemF64Any>(int, bool, bool, dim3, size_t, hipStream_t, const slat::Args &);
template <> int slat_numeric_blocks_per_cu_t<kSemU32>(int, bool, bool, size_t);
template <> int slat_numeric_blocks_per_cu_t<kSemSat64>(int, bool, bool, size_t);
template <> int slat_numeric_blocks_per_cu_t<kSemF64>(int, bool, bool, size_t);
template <> int slat_numeric_blocks_per_cu_t<kSemF64Any>(int, bool, bool, size_t);

static inline hipError_t slat_launch_numeric(int sem, int mode, bool idx32, bool ell, dim3 grid, size_t lds,
                                             hipStream_t s, const slat::Args &a) {
    switch (sem) {
    case kSemU32: return slat_launch_numeric_t<kSemU32>(mode, idx32, ell, grid, lds, s, a);
    case kSemSat64: return slat_launch_numeric_t<kSemSat64>(mode, idx32, ell, grid, lds, s, a);
    case kSemF64: return slat_launch_numeric_t<kSemF64>(mode, idx32, ell, grid, lds, s, a);
    default: return slat_launch_numeric_t<kSemF64Any>(mode, idx32, ell, grid, lds, s, a);
    }
}
static inline int slat_numeric_blocks_per_cu(int sem, int mode, bool idx32, bool ell, size_t lds) {
    switch (sem) {
    case kSemU32: return slat_numeric_blocks_per_cu_t<kSemU32>(mode, idx32, ell, lds);
    case kSemSat64: return slat_numeric_blocks_per_cu_t<kSemSat64>(mode, idx32, ell, lds);
    case kSemF64: return slat_numeric_blocks_per_cu_t<kSemF64>(mode, idx32, ell, lds);
    default: return slat_numeric_blocks_per_cu_t<kSemF64Any>(mode, idx32, ell, lds);
    }
}

// symbolic: mode 0 every row by windows, 1 one row per hash table, 2 the listed / window rows, 4 every
// row of a single-window launch that stores its bitmaps, B's ELL image (lds: sym_stored_words per wave)
hipError_t slat_launch_symbolic(int mode, bool idx32, bool ell, dim3 grid, size_t lds, hipStream_t s,
                                const slat::Args &a);
// the whole product of a small call in one kernel (slat_tiny.hip): status / epoch: the look-back
// words of the blocks' offsets (as k_scan_rows'), maxw: the epoch-tagged max-row word
hipError_t slat_launch_tiny(int sem, dim3 grid, size_t lds, hipStream_t s, const slat::Args &a,
                            unsigned long long *status, uint32_t epoch, unsigned long long *maxw);
// the batched short-row symbolic of wide launches (lists the other rows for mode 2)
// (ell: B's ELL image; else B read in CSR form, < 2^32 entries)
hipError_t slat_launch_symbolic_short(bool idx32, bool ell, dim3 grid, size_t lds, hipStream_t s, const slat::Args &a);
// resident 256-thread blocks per CU of that instance at `lds` bytes (cached per thread)
int slat_symbolic_short_blocks_per_cu(bool idx32, bool ell, size_t lds);
// resident blocks per CU of the listed-row (window) symbolic instance, mode 2
int slat_symbolic_listed_blocks_per_cu(bool idx32, bool ell, size_t lds);


// rows of at most slat_lane_cap() products in one kernel, a row per lane (slat_lane.hip): n rows in
// ceil(n / 64) one-wave blocks, status = look-back words (>= the block count), maxw = max-row word;
// sets host_out[3] when a row has more products than the cap
uint32_t slat_lane_cap();
uint32_t slat_lane_rows();  // rows per block
hipError_t slat_launch_lane(int sem, dim3 grid, hipStream_t s, const slat::Args &a, unsigned long long *status,
                            uint32_t epoch, unsigned long long *maxw);
