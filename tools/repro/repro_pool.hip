// repro_pool.hip — runtime-only check of the stream-ordered pool (hipMallocAsync / hipFreeAsync), for
// the anomaly of round 1 (DESIGN.md "Device memory"): after a small generation had freed pool blocks,
// a fresh 324 MB block read back zeros for a 26 MiB range of one kernel's writes.
//
// The sequence mirrors the old library's generator path on one stream: a 30^3 generation (lattice
// triplets 8.4 MB, from_coo scratch ~50 MB, outputs, thin scratch), every block written by a kernel and
// freed with hipFreeAsync, then the 100^3 lattice's 312 MB triplet block (rows | cols | vals, u32 each)
// written by one kernel — every thread writes its row id and its column id into the two halves — and
// read back. Both release thresholds (0 = the default, UINT64_MAX = keep everything cached) and 5
// repetitions each, after a control run of the same sequence with plain hipMalloc / hipFree; prints
// the wrong words per block (how many are zero, where they end). Exit status 1 if any pool run is wrong.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
            return 2;                                                                          \
        }                                                                                      \
    } while (0)

__global__ void k_fill(uint32_t *p, uint64_t n, uint32_t salt) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)(i * 2654435761u) ^ salt;
}

// the lattice kernel's pattern: triplet t = (node, neighbour): rows[t] = node, cols[t] = neighbour
__global__ void k_trip(uint32_t *rows, uint32_t *cols, uint32_t *vals, uint64_t nt) {
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += (uint64_t)gridDim.x * blockDim.x) {
        rows[t] = (uint32_t)(t / 26);
        cols[t] = (uint32_t)((t * 7919u) % 1000000u);
        vals[t] = 1u;
    }
}

static int run(uint64_t threshold, int rep, bool pool_alloc) {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipMemPool_t pool;
    CK(hipDeviceGetDefaultMemPool(&pool, 0));
    CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &threshold));
    // phase 1: the 30^3 generation's blocks (bytes), written then freed in stream order
    const size_t small[] = {8424064, 50544000, 5616064, 20000000, 3000000, 16848000, 2200000, 9000000};
    std::vector<void *> held;
    for (size_t b : small) {
        void *p = nullptr;
        if (pool_alloc) CK(hipMallocAsync(&p, b, s));
        else CK(hipMalloc(&p, b));
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, s, (uint32_t *)p, b / 4, (uint32_t)b);
        CK(hipGetLastError());
        held.push_back(p);
        if (held.size() % 2 == 0) {  // free in pairs, like the generator's scratch going out of scope
            if (pool_alloc) {
                CK(hipFreeAsync(held[held.size() - 2], s));
                CK(hipFreeAsync(held[held.size() - 1], s));
            } else {
                CK(hipStreamSynchronize(s));
                CK(hipFree(held[held.size() - 2]));
                CK(hipFree(held[held.size() - 1]));
            }
        }
    }
    CK(hipStreamSynchronize(s));
    // phase 2: the 100^3 lattice triplets
    const uint64_t nt = 26000000ull;
    void *blk = nullptr;
    if (pool_alloc) CK(hipMallocAsync(&blk, nt * 12 + 64, s));
    else CK(hipMalloc(&blk, nt * 12 + 64));
    uint32_t *rows = (uint32_t *)blk, *cols = rows + nt, *vals = cols + nt;
    hipLaunchKernelGGL(k_trip, dim3(2048), dim3(256), 0, s, rows, cols, vals, nt);
    CK(hipGetLastError());
    std::vector<uint32_t> h(nt * 3);
    CK(hipMemcpyAsync(h.data(), blk, nt * 12, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    uint64_t bad_r = 0, bad_c = 0, bad_v = 0, zeros = 0, last = 0, shown = 0;
    for (uint64_t t = 0; t < nt; ++t) {
        if (h[t] != (uint32_t)(t / 26)) {
            ++bad_r;
            zeros += h[t] == 0;
            last = t;
            if (shown < 4) {
                std::printf("  row word %llu (byte %llu): got %u, wrote %u\n", (unsigned long long)t,
                            (unsigned long long)t * 4, h[t], (uint32_t)(t / 26));
                ++shown;
            }
        }
        if (h[nt + t] != (uint32_t)((t * 7919u) % 1000000u)) ++bad_c;
        if (h[2 * nt + t] != 1u) ++bad_v;
    }
    std::printf("%s threshold %s rep %d: block %p, wrong rows %llu (%llu of them zero, last at byte %llu) cols %llu "
                "vals %llu\n", pool_alloc ? "hipMallocAsync" : "hipMalloc", threshold ? "max" : "0", rep, blk,
                (unsigned long long)bad_r, (unsigned long long)zeros, (unsigned long long)last * 4,
                (unsigned long long)bad_c, (unsigned long long)bad_v);
    CK(hipStreamSynchronize(s));
    if (pool_alloc) CK(hipFreeAsync(blk, s));
    else CK(hipFree(blk));
    CK(hipStreamSynchronize(s));
    CK(hipStreamDestroy(s));
    return (bad_r || bad_c || bad_v) ? 1 : 0;
}

int main() {
    int rc = 0;
    int ctl = 0;
    for (int rep = 0; rep < 3; ++rep) ctl |= run(0, rep, false);  // control: plain hipMalloc
    for (int rep = 0; rep < 3; ++rep) {
        rc |= run(0, rep, true);
        rc |= run(UINT64_MAX, rep, true);
    }
    std::printf("control (hipMalloc): %s\n", ctl ? "WRONG words too" : "every word read back as written");
    std::printf(rc ? "REPRODUCED: wrong words read back\n" : "not reproduced: every word read back as written\n");
    return rc;
}
