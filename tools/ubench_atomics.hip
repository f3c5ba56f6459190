// ubench_atomics.hip — cost of the device-wide counters a one-pass (symbolic + numeric) kernel would
// need on gfx950: a ticket counter on one address, per-chunk counters, and the row-prefix protocol
// (row statuses + chunk sums) over 27 000 rows taken round-robin by a resident grid.
// Experiments only; not part of the product.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_atomics.hip -o tools/bin/ubench_atomics
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                                     \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);                              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

typedef unsigned long long u64;
__device__ __forceinline__ u64 ld(u64 *x) { return __hip_atomic_load(x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st(u64 *x, u64 v) { __hip_atomic_store(x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// fake per-row work: `spin` iterations of dependent VALU
__device__ __forceinline__ uint32_t work(uint32_t x, int spin) {
    for (int i = 0; i < spin; ++i) x = x * 1664525u + 1013904223u;
    return x;
}

// 1. tickets: every wave takes rows from one counter until n
__global__ __launch_bounds__(256) void k_tickets(u64 *ctr, uint32_t n, int spin, uint32_t *sink) {
    uint32_t x = threadIdx.x, done = 0;
    while (true) {
        u64 t = 0;
        if ((threadIdx.x & 63) == 0) t = atomicAdd(ctr, 1ull);
        t = __builtin_amdgcn_readfirstlane((uint32_t)t);
        if (t >= n) break;
        x = work(x + (uint32_t)t, spin);
        ++done;
    }
    if (x == 0x12345678u) sink[0] = done;
}

// 2. round-robin rows (resident grid), one non-returning atomic per row on its chunk word
__global__ __launch_bounds__(256) void k_chunks(u64 *chunk, uint32_t n, uint32_t csh, int spin, uint32_t *sink) {
    const uint32_t waves = gridDim.x * 4, gid = blockIdx.x * 4 + threadIdx.x / 64;
    uint32_t x = threadIdx.x;
    for (uint32_t r = gid; r < n; r += waves) {
        x = work(x + r, spin);
        if ((threadIdx.x & 63) == 0) atomicAdd(&chunk[r >> csh], (1ull << 40) + (x & 7));
    }
    if (x == 0x12345678u) sink[0] = x;
}

// 3. latency: one wave, a chain of dependent agent-scope loads (pointer chase), and of returning atomics
__global__ void k_latency(u64 *chain, int iters, u64 *out, u64 *ctr) {
    u64 p = 0;
    u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) p = ld(&chain[p]);
    u64 t1 = __builtin_readcyclecounter();
    u64 q = 0;
    for (int i = 0; i < iters; ++i) q += atomicAdd(ctr, 1ull + (q & 0));
    u64 t2 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) {
        out[0] = (t1 - t0) / iters;
        out[1] = (t2 - t1) / iters;
        out[2] = p + q;
    }
}

// 4. the row-prefix protocol. Row r (round-robin over a resident grid): count c(r) (from its index),
// publish status[r] = tag | c, add (1 << 40) + c to chunk[r >> 8] (a done count and a sum), then its
// exclusive prefix: the sum of every earlier chunk (each complete: done == 256; the walk stops at a
// chunk holding its inclusive prefix in incl[]) + the statuses of the earlier rows of its own chunk.
// A chunk's last row publishes the chunk's inclusive prefix. rp[r + 1] = prefix + c.
constexpr uint32_t kCsh = 8, kCRows = 1u << kCsh;
__device__ __forceinline__ uint32_t row_count(uint32_t r) { return (r * 2654435761u >> 23) & 511; }
__global__ __launch_bounds__(256) void k_prefix(u64 *status, u64 *chunk, u64 *incl, uint32_t n, uint32_t epoch,
                                                int spin1, int spin2, u64 *rp, u64 *stall) {
    const uint32_t waves = gridDim.x * 4, gid = blockIdx.x * 4 + threadIdx.x / 64;
    const int lane = threadIdx.x & 63;
    const u64 tag = (u64)epoch << 40;
    uint32_t x = threadIdx.x;
    u64 polls = 0;
    for (uint32_t r = gid; r < n; r += waves) {
        x = work(x + r, spin1);  // the bitmap pass
        const uint32_t c = row_count(r) + (x == 0x12345678u);
        if (lane == 0) {
            st(&status[r], tag | c);
            atomicAdd(&chunk[r >> kCsh], (1ull << 40) + c);
        }
        x = work(x, spin2);  // the accumulate pass
        // own chunk's earlier rows: lanes hold 4 each
        const uint32_t c0 = r & ~(kCRows - 1);
        u64 own = 0;
        while (true) {
            bool ok = true;
            u64 s = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t j = c0 + (uint32_t)lane * 4 + i;
                if (j < r) {
                    const u64 v = ld(&status[j]);
                    ok = ok && (v >> 40) == epoch;
                    s += v & ((1ull << 40) - 1);
                }
            }
            if (__ballot(!ok) == 0) {
                own = s;
                break;
            }
            ++polls;
            __builtin_amdgcn_s_sleep(1);
        }
        for (int d = 32; d; d >>= 1) own += __shfl_xor(own, d);
        // earlier chunks: walk back 64 per round to the nearest inclusive prefix
        u64 before = 0;
        for (int64_t k0 = (int64_t)(r >> kCsh) - 1; k0 >= 0; k0 -= 64) {
            const int64_t k = k0 - lane;
            u64 cw = 0, iw = 0;
            bool ok = true;
            while (true) {
                ok = true;
                if (k >= 0) {
                    iw = ld(&incl[k]);
                    if ((iw >> 40) != epoch) {
                        cw = ld(&chunk[k]);
                        ok = (cw >> 40) == kCRows;
                    }
                }
                // lanes past the nearest inclusive do not matter
                const u64 inc = __ballot(k >= 0 && (iw >> 40) == epoch);
                const int last = inc ? __builtin_ctzll(inc) : 64;
                if (__ballot(!ok && lane < last) == 0) break;
                ++polls;
                __builtin_amdgcn_s_sleep(1);
            }
            const u64 inc = __ballot(k >= 0 && (iw >> 40) == epoch);
            const int last = inc ? __builtin_ctzll(inc) : 64;
            u64 v = 0;
            if (k >= 0 && lane < last) v = cw & ((1ull << 40) - 1);
            if (k >= 0 && lane == last) v = iw & ((1ull << 40) - 1);
            for (int d = 32; d; d >>= 1) v += __shfl_xor(v, d);
            before += v;
            if (inc) break;
        }
        const u64 pre = before + own;
        if (lane == 0) {
            rp[r + 1] = pre + c;
            if ((r & (kCRows - 1)) == kCRows - 1 || r == n - 1) st(&incl[r >> kCsh], tag | (pre + c));
        }
    }
    if (lane == 0) atomicAdd(stall, polls);
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 27000;
    int dev_cu = 0;
    CHK(hipDeviceGetAttribute(&dev_cu, hipDeviceAttributeMultiprocessorCount, 0));
    u64 *buf;
    CHK(hipMalloc(&buf, 64 << 20));
    uint32_t *sink;
    CHK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    auto timed = [&](auto launch) {
        launch();
        CHK(hipDeviceSynchronize());
        float best = 1e9;
        for (int i = 0; i < 5; ++i) {
            CHK(hipEventRecord(e0));
            launch();
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        return best * 1e3f;
    };
    const int grids[] = {dev_cu, dev_cu * 3};
    for (int spin : {0, 200}) {
        for (int g : grids) {
            float t = timed([&] {
                CHK(hipMemsetAsync(buf, 0, 8));
                hipLaunchKernelGGL(k_tickets, dim3(g), dim3(256), 0, 0, buf, n, spin, sink);
            });
            float tb = timed([&] { hipLaunchKernelGGL(k_chunks, dim3(g), dim3(256), 0, 0, buf + 64, n, 8, spin, sink); });
            float t0 = timed([&] { CHK(hipMemsetAsync(buf, 0, 8)); });
            printf("spin %d grid %d: tickets %.2f us (memset %.2f), chunk counters %.2f us\n", spin, g, t, t0, tb);
        }
    }
    // latency
    {
        std::vector<u64> h(4096);
        for (int i = 0; i < 4096; ++i) h[i] = (i * 1031 + 17) & 4095;  // stride-1031 chase
        CHK(hipMemcpy(buf + 8192, h.data(), 4096 * 8, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_latency, dim3(1), dim3(64), 0, 0, buf + 8192, 1000, buf + 16384, buf + 16400);
        u64 o[3];
        CHK(hipMemcpy(o, buf + 16384, 24, hipMemcpyDeviceToHost));
        printf("latency (cycles of s_memrealtime... readcyclecounter): agent load %llu, returning atomic %llu\n", o[0], o[1]);
    }
    // prefix protocol
    {
        const uint32_t nch = (n + kCRows - 1) / kCRows;
        u64 *status = buf + 32768, *chunk = status + n + 64, *incl = chunk + nch + 64, *rp = incl + nch + 64,
            *stall = rp + n + 64;
        std::vector<u64> ref(n + 1, 0);
        for (uint32_t r = 0; r < n; ++r) ref[r + 1] = ref[r] + ((r * 2654435761u >> 23) & 511);
        uint32_t epoch = 1;
        for (int spin : {0, 500, 2000}) {
            for (int g : grids) {
                float best = 1e9;
                u64 polls = 0;
                bool okall = true;
                for (int rep = 0; rep < 4; ++rep) {
                    CHK(hipMemsetAsync(chunk, 0, nch * 8));
                    CHK(hipMemsetAsync(stall, 0, 8));
                    ++epoch;
                    CHK(hipEventRecord(e0));
                    hipLaunchKernelGGL(k_prefix, dim3(g), dim3(256), 0, 0, status, chunk, incl, n, epoch, spin, spin,
                                       rp, stall);
                    CHK(hipEventRecord(e1));
                    CHK(hipEventSynchronize(e1));
                    float ms;
                    CHK(hipEventElapsedTime(&ms, e0, e1));
                    if (rep) best = ms < best ? ms : best;
                    std::vector<u64> got(n + 1);
                    CHK(hipMemcpy(got.data() + 1, rp + 1, n * 8, hipMemcpyDeviceToHost));
                    for (uint32_t r = 1; r <= n; ++r) okall = okall && got[r] == ref[r];
                    CHK(hipMemcpy(&polls, stall, 8, hipMemcpyDeviceToHost));
                }
                // the same work without the protocol
                float tw = timed([&] { hipLaunchKernelGGL(k_chunks, dim3(g), dim3(256), 0, 0, buf + 64, n, 8, 2 * spin, sink); });
                printf("prefix spin %d grid %d: %.2f us (work alone %.2f us), polls %llu, %s\n", spin, g, best * 1e3f, tw,
                       polls, okall ? "ok" : "WRONG");
            }
        }
    }
    return 0;
}
