// Host round trip of a synchronous call on this runtime: launch N small kernels, then wait.
// Measures the per-call floor that bench.py's one-call-per-step protocol pays between calls.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_touch(unsigned *x, unsigned v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) x[0] = v;
}
struct Big {
    unsigned long long w[40];  // 320 B of kernel arguments, like the library's Args
};
__global__ void k_big(Big b, unsigned *x) {
    if (threadIdx.x == 0 && blockIdx.x == 0) x[0] = (unsigned)b.w[3];
}
__global__ void k_flag(volatile unsigned *host_flag, unsigned v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        __threadfence_system();
        host_flag[0] = v;
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned *d;
    CK(hipMalloc(&d, 256));
    unsigned *h;
    CK(hipHostMalloc(&h, 64, hipHostMallocMapped));
    unsigned *hd;
    CK(hipHostGetDevicePointer((void **)&hd, h, 0));
    const int iters = 2000;
    auto spin = [&]() { while (hipStreamQuery(s) == hipErrorNotReady) {} };
    for (int nk : {1, 4}) {
        for (int i = 0; i < 200; ++i) { for (int k = 0; k < nk; ++k) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, d, i); spin(); }
        double t0 = now_us();
        for (int i = 0; i < iters; ++i) { for (int k = 0; k < nk; ++k) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, d, i); spin(); }
        std::printf("%d kernel(s) + hipStreamQuery spin: %.2f us/call\n", nk, (now_us() - t0) / iters);
        t0 = now_us();
        for (int i = 0; i < iters; ++i) { for (int k = 0; k < nk; ++k) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, d, i); CK(hipStreamSynchronize(s)); }
        std::printf("%d kernel(s) + hipStreamSynchronize: %.2f us/call\n", nk, (now_us() - t0) / iters);
        t0 = now_us();
        for (int i = 0; i < iters; ++i) {
            for (int k = 0; k + 1 < nk; ++k) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, d, i);
            hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, hd, (unsigned)(i + 1));
            while (((volatile unsigned *)h)[0] != (unsigned)(i + 1)) {}
        }
        CK(hipStreamSynchronize(s));
        std::printf("%d kernel(s) + mapped host flag spin: %.2f us/call\n", nk, (now_us() - t0) / iters);
        h[0] = 0;
    }
    // the same 4 launches captured in a graph
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, d, k);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 200; ++i) { CK(hipGraphLaunch(ge, s)); spin(); }
    double t0 = now_us();
    for (int i = 0; i < iters; ++i) { CK(hipGraphLaunch(ge, s)); spin(); }
    std::printf("graph of 4 kernels + hipStreamQuery spin: %.2f us/call\n", (now_us() - t0) / iters);
    t0 = now_us();
    for (int i = 0; i < iters; ++i) { for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, d, i); }
    CK(hipStreamSynchronize(s));
    std::printf("enqueue only, 4 kernels: %.2f us/call\n", (now_us() - t0) / iters);
    Big b{};
    t0 = now_us();
    for (int i = 0; i < iters; ++i) {
        b.w[3] = i;
        for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, s, b, d);
    }
    CK(hipStreamSynchronize(s));
    std::printf("enqueue only, 4 kernels with 320-byte arguments: %.2f us/call\n", (now_us() - t0) / iters);
    t0 = now_us();
    for (int i = 0; i < iters; ++i) {
        b.w[3] = i;
        for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, s, b, d);
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, hd, (unsigned)(i + 1));
        while (((volatile unsigned *)h)[0] != (unsigned)(i + 1)) {}
    }
    std::printf("3 kernels with 320-byte arguments + flag kernel, spin: %.2f us/call\n", (now_us() - t0) / iters);
    return 0;
}
