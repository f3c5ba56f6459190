// repro_radix.cpp — runtime/library-only check of hipcub::DeviceRadixSort::SortPairs (rocPRIM) for the
// anomaly of round 1 (slat_coo.hip): with a partial top 8-bit digit (end_bit 49), 3.4M (row<<32|col)
// keys came back in a wrong order. Sorts such keys (a thinned 3-D lattice's triplets, shuffled, and
// uniform random ones) with end_bit 41..64 and with the whole-digit rounding the library now uses,
// then checks order and that the values are the matching permutation, with every buffer from hipMalloc
// and then from the stream-ordered pool. Exit status 1 if a hipMalloc-buffer sort is wrong.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
            return 2;                                                                          \
        }                                                                                      \
    } while (0)

static bool g_pool = false;  // buffers from the stream-ordered pool (after some churn) instead of hipMalloc

static hipError_t get(void **p, size_t b) {
    if (!g_pool) return hipMalloc(p, b);
    const hipError_t e = hipMallocAsync(p, b, 0);
    if (e == hipSuccess) (void)hipMemsetAsync(*p, 0xA5, 64, 0);
    return e;
}
static void put(void *p) {
    if (g_pool) (void)hipFreeAsync(p, 0);
    else (void)hipFree(p);
}

static int check(const std::vector<uint64_t> &keys, int end_bit, const char *what) {
    const size_t n = keys.size();
    uint64_t *dk, *dk2;
    uint32_t *dv, *dv2;
    CK(get((void **)&dk, n * 8));
    CK(get((void **)&dk2, n * 8));
    CK(get((void **)&dv, n * 4));
    CK(get((void **)&dv2, n * 4));
    std::vector<uint32_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0u);
    CK(hipMemcpy(dk, keys.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, idx.data(), n * 4, hipMemcpyHostToDevice));
    size_t tb = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, dk, dk2, dv, dv2, (int)n, 0, end_bit));
    void *tmp;
    CK(get(&tmp, tb));
    CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, dk, dk2, dv, dv2, (int)n, 0, end_bit));
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> ok(n);
    std::vector<uint32_t> ov(n);
    CK(hipMemcpy(ok.data(), dk2, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ov.data(), dv2, n * 4, hipMemcpyDeviceToHost));
    size_t bad_order = 0, bad_pair = 0;
    std::vector<char> seen(n, 0);
    // only the sorted bits [0, end_bit) order the output; higher bits keep input order among equals
    const uint64_t mask = end_bit >= 64 ? ~0ull : ((1ull << end_bit) - 1);
    for (size_t i = 0; i < n; ++i) {
        if (i && (ok[i - 1] & mask) > (ok[i] & mask)) ++bad_order;
        if (ov[i] >= n || seen[ov[i]] || keys[ov[i]] != ok[i]) ++bad_pair;
        if (ov[i] < n) seen[ov[i]] = 1;
    }
    std::printf("%-9s %-34s n=%zu end_bit=%d: out-of-order %zu, wrong pairs %zu\n", g_pool ? "pool" : "hipMalloc",
                what, n, end_bit, bad_order, bad_pair);
    put(dk);
    put(dk2);
    put(dv);
    put(dv2);
    put(tmp);
    CK(hipDeviceSynchronize());
    return (bad_order || bad_pair) ? 1 : 0;
}

int main() {
    std::mt19937_64 g(42);
    int rc = 0;
    // a thinned 3-D Moore lattice of side 50 (125000 nodes: 17-bit rows -> 49-bit keys), ~27 e/n
    const uint32_t side = 50, nn = side * side * side;
    std::vector<uint64_t> lat;
    for (uint32_t v = 0; v < nn; ++v) {
        const int x = v / (side * side), y = (v / side) % side, z = v % side;
        for (int d = 0; d < 27; ++d) {
            const int dx = d / 9 - 1, dy = (d / 3) % 3 - 1, dz = d % 3 - 1;
            const uint32_t u = ((x + dx + side) % side) * side * side + ((y + dy + side) % side) * side + (z + dz + side) % side;
            lat.push_back(((uint64_t)v << 32) | u);
        }
    }
    std::shuffle(lat.begin(), lat.end(), g);  // triplets arrive unordered
    lat.resize(3400000);
    for (int eb : {49, 50, 56, 64}) rc |= check(lat, eb, "lattice (row<<32|col), 3.4M");
    std::vector<uint64_t> rnd(3400000);
    for (auto &k : rnd) k = g() & ((1ull << 49) - 1);
    for (int eb : {41, 49, 56, 64}) rc |= check(rnd, eb, "uniform 49-bit keys, 3.4M");
    std::vector<uint64_t> big(12000000);
    for (auto &k : big) k = g() & ((1ull << 49) - 1);
    for (int eb : {49, 56}) rc |= check(big, eb, "uniform 49-bit keys, 12M");
    std::printf(rc ? "hipMalloc buffers: a sort returned a wrong order\n" : "hipMalloc buffers: every sort correct\n");
    // the same sorts with every buffer from the stream-ordered pool (the round-1 library's scratch)
    g_pool = true;
    int rp = 0;
    for (int eb : {49, 56}) rp |= check(lat, eb, "lattice (row<<32|col), 3.4M");
    for (int eb : {49, 56}) rp |= check(big, eb, "uniform 49-bit keys, 12M");
    std::printf(rp ? "pool buffers: a sort returned a wrong order\n" : "pool buffers: every sort correct\n");
    return rc;
}
