// ubench_lds.hip — LDS cost per wave-instruction on gfx950 for the access shapes of the SpGEMM
// accumulator: random addresses inside a per-wave region (like ranks / bitmap words), 64 lanes.
// Experiments only; not part of the product.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_lds.hip -o tools/bin/ubench_lds
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                                     \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);                              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

constexpr int kIters = 2048;
constexpr int kRegionWords = 2048;  // 8 KB per wave

// OP: 0 read_b32, 1 read_b64, 2 add_u32 (no ret), 3 add_u64 (no ret), 4 or_b32 (no ret),
//     5 write_b32, 6 add_u64 half the lanes, 7 read_b64 conflict-free, 8 add_u64 conflict-free,
//     9 add_u32 returning, 10 write_b64
template <int OP>
__global__ __launch_bounds__(256) void k_lds(uint32_t *out, int waves_per_block, uint32_t seed) {
    extern __shared__ uint32_t sm[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (wv >= waves_per_block) return;
    uint32_t *reg = sm + wv * kRegionWords;
    for (int i = lane; i < kRegionWords; i += 64) reg[i] = i;
    __builtin_amdgcn_wave_barrier();
    uint32_t x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
    uint32_t acc = 0;
    unsigned long long *reg64 = (unsigned long long *)reg;
#pragma unroll 8
    for (int it = 0; it < kIters; ++it) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        const uint32_t a = x & (kRegionWords - 1), a2 = x & (kRegionWords / 2 - 1);
        if constexpr (OP == 0) acc += reg[a];
        if constexpr (OP == 1) acc += (uint32_t)reg64[a2];
        if constexpr (OP == 2) atomicAdd(&reg[a], 1u);
        if constexpr (OP == 3) atomicAdd(&reg64[a2], 1ull);
        if constexpr (OP == 4) atomicOr(&reg[a], 1u << (x >> 27));
        if constexpr (OP == 5) reg[a] = x;
        if constexpr (OP == 6) {
            if (x & 0x10000) atomicAdd(&reg64[a2], 1ull);
        }
        if constexpr (OP == 7) acc += (uint32_t)reg64[(lane + it * 64) & (kRegionWords / 2 - 1)];
        if constexpr (OP == 8) atomicAdd(&reg64[(lane + it * 64) & (kRegionWords / 2 - 1)], 1ull);
        if constexpr (OP == 9) acc += atomicAdd(&reg[a], 1u);
        if constexpr (OP == 10) reg64[a2] = x;
    }
    __builtin_amdgcn_wave_barrier();
    acc += reg[lane];
    if (acc == 0x12345678u) out[0] = acc;
}

template <int OP>
static void run(const char *name, int cus, int wpb, int bpc) {
    uint32_t *out;
    CHK(hipMalloc(&out, 4));
    const int grid = cus * bpc * 8;  // 8 rounds of full residency
    const size_t lds = (size_t)wpb * kRegionWords * 4;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_lds<OP>, dim3(grid), dim3(256), lds, 0, out, wpb, 1u);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0, 0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_lds<OP>, dim3(grid), dim3(256), lds, 0, out, wpb, 7u + r);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double instr_per_cu = (double)grid * wpb * kIters * 5 / cus;
    const double cyc = ms * 1e-3 * 2.4e9;
    printf("%-28s waves/CU~%2d  %.2f cycles per wave-instruction per CU  (%.1f us/launch)\n", name, wpb * bpc,
           cyc / instr_per_cu, ms * 1e3 / 5);
    CHK(hipFree(out));
}

int main() {
    hipDeviceProp_t pr;
    CHK(hipGetDeviceProperties(&pr, 0));
    const int cus = pr.multiProcessorCount;
    for (int bpc : {1, 2, 4}) {
        run<0>("ds_read_b32 random", cus, 4, bpc);
        run<1>("ds_read_b64 random", cus, 4, bpc);
        run<7>("ds_read_b64 linear", cus, 4, bpc);
        run<2>("ds_add_u32 random", cus, 4, bpc);
        run<3>("ds_add_u64 random", cus, 4, bpc);
        run<8>("ds_add_u64 linear", cus, 4, bpc);
        run<6>("ds_add_u64 random half", cus, 4, bpc);
        run<4>("ds_or_b32 random", cus, 4, bpc);
        run<5>("ds_write_b32 random", cus, 4, bpc);
        run<10>("ds_write_b64 random", cus, 4, bpc);
        run<9>("ds_add_rtn_u32 random", cus, 4, bpc);
    }
    return 0;
}
