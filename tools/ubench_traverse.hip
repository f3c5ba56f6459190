// ubench_traverse.hip — stage-by-stage cost of the row traversal on the bench workload
// (30^3 torus, A^6 * A). Builds the inputs through libslat, then times kernel variants that
// each add one stage of the product walk. Experiments only; not part of the product.
//   hipcc -O3 --offload-arch=gfx950 -I../include tools/ubench_traverse.hip -L... -lslat
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "slat.h"

#define CHK(x)                                                                                     \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);                              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

constexpr int W = 64;

__device__ __forceinline__ uint32_t dpp_incl_scan(uint32_t v) {
    // wave64 inclusive prefix sum with DPP row shifts + row broadcasts (GCN idiom)
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

struct P {
    const uint64_t *a_rp;
    const uint32_t *a_col;
    const uint64_t *b_rp;
    const uint32_t *b_col;
    uint32_t n;
    uint32_t *out;
    const uint4 *ell;   // row-major padded ELL of B: row k = ell[k*wq .. k*wq+wq), 0xFFFFFFFF pads
    uint32_t wq;        // uint4 per row
};

__global__ void k_build_ell(const uint64_t *rp, const uint32_t *col, uint32_t n, uint32_t wq, uint32_t *ell) {
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
        const uint32_t s = (uint32_t)rp[k], len = (uint32_t)rp[k + 1] - s;
        for (uint32_t u = 0; u < wq * 4; ++u) ell[k * wq * 4 + u] = u < len ? col[s + u] : 0xFFFFFFFFu;
    }
}

// MODE 0: row loop only; 1: + a_col; 2: + b_rp; 3: + lane-per-A loop over b_col;
//      4: flattened via LDS expansion (write jdx per product) + b_col; 5: 4 + DPP scan only
template <int MODE>
__global__ __launch_bounds__(256) void k_trav(P p) {
    constexpr bool kNeedRp = MODE >= 2 && MODE != 6;
    __shared__ uint32_t stage[4][64 * 16];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t acc = 0;
    for (uint32_t row = blockIdx.x * 4 + wv; row < p.n; row += gridDim.x * 4) {
        const uint32_t a0 = (uint32_t)p.a_rp[row], a1 = (uint32_t)p.a_rp[row + 1];
        if constexpr (MODE >= 1) {
            for (uint32_t base = a0; base < a1; base += W) {
                const uint32_t idx = base + lane;
                uint32_t k = 0, bs = 0, be = 0;
                if (idx < a1) k = p.a_col[idx];
                if constexpr (MODE == 1) acc += k;
                if constexpr (kNeedRp) {
                    if (idx < a1) {
                        bs = (uint32_t)p.b_rp[k];
                        be = (uint32_t)p.b_rp[k + 1];
                    }
                    if constexpr (MODE == 2) acc += bs + be;
                }
                if constexpr (MODE == 6) {
                    if (idx < a1) {
                        const uint4 *r = p.ell + (size_t)k * p.wq;
                        uint4 q = r[0];
                        acc += q.x + (q.y != 0xFFFFFFFFu ? q.y : 0) + (q.z != 0xFFFFFFFFu ? q.z : 0);
                        for (uint32_t t = 1; t < p.wq && q.w != 0xFFFFFFFFu; ++t) {
                            acc += q.w;
                            q = r[t];
                            acc += q.x + q.y + q.z;
                        }
                    }
                }
                if constexpr (MODE == 3) {
                    for (uint32_t j = bs; j < be; ++j) acc += p.b_col[j];
                }
                if constexpr (MODE == 4 || MODE == 5) {
                    const uint32_t len = be - bs;
                    const uint32_t incl = dpp_incl_scan(len);
                    const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
                    uint32_t o = incl - len;
                    for (uint32_t j = bs; j < be; ++j, ++o)
                        if (o < 64 * 16) stage[wv][o] = j;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    if constexpr (MODE == 4) {
                        for (uint32_t q = lane; q < total && q < 64 * 16; q += W) acc += p.b_col[stage[wv][q]];
                    } else {
                        acc += total;
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
        if (lane == 0) p.out[row] = acc;
    }
    if (acc == 0xdeadbeef) p.out[0] = 1;
}

template <int MODE>
static float run(const P &p, int grid, int reps) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_trav<MODE>, dim3(grid), dim3(256), 0, 0, p);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_trav<MODE>, dim3(grid), dim3(256), 0, 0, p);
    CHK(hipEventRecord(b, 0));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    return ms / reps * 1000.f;
}

int main() {
    slat_ctx *ctx;
    if (slat_ctx_create(0, &ctx) != SLAT_OK) return 1;
    uint64_t dims[3] = {30, 30, 30};
    slat_host_csr full, a;
    slat_host_lattice(dims, 3, 1, &full);
    slat_rng rng;
    uint8_t seed[32];
    for (int i = 0; i < 32; ++i) seed[i] = 42;
    slat_rng_seed(&rng, seed);
    slat_host_thin(&full, &rng, 3.0 / 26.0, &a);
    slat_csr_view hv = {a.n, a.n, a.nnz, a.row_ptr, a.col_idx, a.values, SLAT_U32, SLAT_HOST, 0};
    slat_csr dA, dP, tmp;
    slat_csr_create(ctx, &hv, &dA);
    slat_csr_view vA = slat_csr_view_of(&dA);
    dP = dA;
    bool own = false;
    for (int k = 2; k < 7; ++k) {
        slat_csr_view vP = slat_csr_view_of(&dP);
        slat_spgemm(ctx, &vP, &vA, &tmp, 0);
        if (own) slat_csr_free(ctx, &dP);
        dP = tmp;
        own = true;
    }
    printf("A^6 nnz=%lu\n", (unsigned long)dP.nnz);
    uint32_t *out;
    CHK(hipMalloc(&out, dP.n_rows * 4));
    const uint32_t wq = (uint32_t)((dA.max_row_nnz + 3) / 4);
    uint32_t *ell;
    CHK(hipMalloc(&ell, (size_t)dA.n_rows * wq * 16));
    hipLaunchKernelGGL(k_build_ell, dim3(256), dim3(256), 0, 0, dA.row_ptr, dA.col_idx, (uint32_t)dA.n_rows, wq, ell);
    CHK(hipDeviceSynchronize());
    P p{dP.row_ptr, dP.col_idx, dA.row_ptr, dA.col_idx, (uint32_t)dP.n_rows, out, (const uint4 *)ell, wq};
    for (int grid : {1024, 2048, 4096}) {
        printf("grid %d: rows-only %.1f us | +a_col %.1f | +b_rp %.1f | +lane-per-A b_col %.1f | LDS-expand b_col %.1f | "
               "LDS-expand no b_col %.1f\n",
               grid, run<0>(p, grid, 20), run<1>(p, grid, 20), run<2>(p, grid, 20), run<3>(p, grid, 20),
               run<4>(p, grid, 20), run<5>(p, grid, 20));
        printf("grid %d: ELL row-major dwordx4 %.1f us\n", grid, run<6>(p, grid, 20));
    }
    return 0;
}
