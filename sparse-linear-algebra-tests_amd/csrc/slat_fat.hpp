// slat_fat.hpp — the fat-row category's launch record and host entry points (slat_fat.hip), shared
// with the SpGEMM orchestration (slat_api.hip).
#pragma once
#include <stdint.h>

#include "slat_internal.hpp"
#include "spgemm_kernels.hpp"

namespace slat {
struct FatArgs {
    Args a;
    uint32_t *list;             // fat rows
    unsigned int *cnt;          // their number
    uint8_t *mark;              // [n] 1 = fat
    unsigned long long *cmask;  // [list position] touched accumulator chunks (bit c: chunk c; 64 max)
    uint32_t csh;               // log2 of the chunk mask's granule (columns per mask bit)
    // B split by column granule (numeric pass; null = none): split[k * nch1 + g] = the offset in B
    // row k of its first entry with column >= g << gsh (g = 0 .. nch1 - 1, the last = len). The
    // granule is the accumulator chunk, or for f64 in the reference's order one wave's slice of it
    // split_abs: the entries hold absolute offsets in B (B of < 2^32 entries), so a walk loads the
    // part's bounds from the table alone, without B's row pointer (one random cache line per A
    // entry and chunk instead of two: C5's fold order read 50 GB in k_fr_numeric, mostly these)
    const uint32_t *split;
    uint32_t nch1;
    uint32_t gsh;
    uint32_t split_abs;
    // products bucketed by accumulator chunk (integer semirings and f64 in any order; null = none):
    // each block's region of bcap (column, product) pairs at bcol / bval + blockIdx.x * bcap
    uint32_t *bcol;
    void *bval;
    uint32_t bcap;
    // row tickets (SLAT_FAT_TICKET; the context's ticket word, zero between launches): rows by a
    // counter instead of a fixed stride over the blocks
    unsigned long long *tq;
    uint64_t fat_min;  // products per row from which a row is fat (slat_fat_min)
    uint32_t sym_bits;  // k_fr_symbolic's bitmap columns per pass (slat_fat_symbolic)
    uint32_t buckets;   // SLAT_FLAG_FAT_BUCKETS: products bucketed by chunk in HBM (fr_num)
};
}  // namespace slat

// B (CSR) bucketed by column granule of 2^shift columns on stream s: split[k * nch1 + g] = the offset
// in B row k of its first column >= g << shift, g in [0, nch1) (the last = the row's length); abs:
// the absolute offset in B instead (B of < 2^32 entries)
hipError_t slat_launch_splits(slat_ctx *ctx, const uint64_t *b_rp, const uint32_t *b_col, uint64_t nb, uint32_t nch1,
                              uint32_t shift, uint32_t *split, hipStream_t s, uint32_t abs = 0);
// products per row from which a row takes the fat-row kernels: 2048 with `flat` (B in CSR form, a
// semiring that adds with atomics: the flattened walk), else 8192
uint64_t slat_fat_min(bool flat);
// workspace bytes of the category for n rows
size_t slat_fat_ws(uint64_t n);
// mark and list the rows of >= fat_min products (sets a.fr_mark); nothing comes back to the host
slat_status slat_fat_select(slat_ctx *ctx, slat::Args &a, void *ws, uint64_t fat_min, slat::FatArgs *out);
slat_status slat_fat_symbolic(slat_ctx *ctx, slat::FatArgs &f, const slat::Args &a, bool idx32);
slat_status slat_fat_numeric(slat_ctx *ctx, slat::FatArgs &f, const slat::Args &a, int32_t dtype, bool f64any, bool idx32);
