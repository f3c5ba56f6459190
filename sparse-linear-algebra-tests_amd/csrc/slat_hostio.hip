// slat_hostio.hip — host <-> device copies of the drop-in's host-resident arrays.
//
// The reference's calling convention is Vec in, Vec out (CsrMatrix::matmul(&self, &Self) -> Self,
// src/graph_csr.rs:306-346; its benches time exactly that, src/graph_magnus.rs:758-772), so a Rust
// or C++ caller hands the library PAGEABLE host memory. The HIP runtime copies pageable memory through
// its own bounce buffers with one host thread (the headline's 147 MB took 9.9 ms end to end, 15 GB/s).
// Here every pageable segment goes through a per-context ring of page-locked slots instead:
//   * H2D: chunk i is copied into slot i % K by the context's worker threads (a parallel memcpy),
//     then DMA'd to the device; the memcpy of chunk i + 1 runs under chunk i's DMA;
//   * D2H: the first K chunks' DMAs are queued at once; while they run, the threads touch every
//     page of the caller's arrays (a fresh Vec / np.empty is unmapped memory: its first write faults
//     and the kernel zeroes the page, 2 MB at a time under transparent huge pages — done by one
//     thread inside the copies, that took 8 of the 10 ms of the headline's end-to-end call); then
//     chunk i's memcpy out of its slot runs under the DMAs of chunks i + 1 .. i + K - 1, and the
//     slot is refilled with chunk i + K.
// Page-locked segments (slat_host_alloc, pinned_empty) skip the ring: one DMA each.
// The C ABI is unchanged: slat_csr_create / slat_csr_to_host / the host-residency SpGEMM use it.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "slat_internal.hpp"

namespace {

constexpr size_t kChunk = (size_t)8 << 20;  // bytes per staging slot
constexpr int kSlots = 4;                    // slots in the ring (32 MB page-locked per context)
constexpr size_t kParMin = (size_t)1 << 20;  // below this a memcpy stays on the calling thread

// How the host threads are told about a job: a generation counter they spin on for a while after a
// job (a transfer is a burst of chunk copies ~100 us apart), then sleep on a condition variable.
class CopyPool {
  public:
    explicit CopyPool(int threads) : n_(threads) {
        for (int w = 1; w < n_; ++w) th_.emplace_back([this, w] { run(w); });
    }
    ~CopyPool() {
        stop_.store(true);
        {
            std::lock_guard<std::mutex> lk(m_);
            cv_.notify_all();
        }
        for (auto &t : th_) t.join();
    }
    // dst[0, bytes) = src[0, bytes), split over the pool's threads in page-aligned pieces
    void copy(void *dst, const void *src, size_t bytes) {
        if (n_ <= 1 || bytes < kParMin) {
            std::memcpy(dst, src, bytes);
            return;
        }
        touch_ = false;
        dst_ = (char *)dst;
        src_ = (const char *)src;
        bytes_ = bytes;
        piece_ = ((bytes + n_ - 1) / n_ + 4095) & ~(size_t)4095;
        launch();
    }
    // one write per 4 KiB page of dst[0, bytes) (the contents are garbage afterwards), split over the
    // threads in 2 MiB-aligned pieces so no two threads fault the same huge page
    void touch(void *dst, size_t bytes) {
        if (bytes < kParMin) return;
        touch_ = true;
        dst_ = (char *)dst;
        src_ = nullptr;
        bytes_ = bytes;
        piece_ = ((bytes + n_ - 1) / n_ + ((size_t)2 << 20) - 1) & ~(((size_t)2 << 20) - 1);
        launch();
    }

  private:
    void launch() {
        pending_.store(n_ - 1);
        gen_.fetch_add(1);
        if (sleepers_.load() > 0) {
            std::lock_guard<std::mutex> lk(m_);
            cv_.notify_all();
        }
        part(0);
        while (pending_.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
    }
    void part(int w) {
        const size_t lo = (size_t)w * piece_;
        if (lo >= bytes_) return;
        const size_t len = std::min(piece_, bytes_ - lo);
        if (touch_) {
            // piece boundaries on absolute 2 MiB addresses (huge pages are aligned there)
            const uintptr_t h = ((uintptr_t)2 << 20) - 1, b0 = (uintptr_t)dst_, b1 = b0 + bytes_;
            const uintptr_t s = w == 0 ? b0 : std::min(b1, (b0 + lo + h) & ~h);
            const uintptr_t e = std::min(b1, (b0 + lo + len + h) & ~h);
            for (uintptr_t a = s; a < e; a = (a | 4095) + 1) *(volatile char *)a = 0;
        } else {
            std::memcpy(dst_ + lo, src_ + lo, len);
        }
    }
    void run(int w) {
        uint64_t seen = 0;
        for (;;) {
            int spins = 0;
            uint64_t g;
            while ((g = gen_.load()) == seen) {
                if (stop_.load()) return;
                if (++spins < (1 << 14)) {
                    __builtin_ia32_pause();
                    continue;
                }
                std::unique_lock<std::mutex> lk(m_);
                sleepers_.fetch_add(1);
                cv_.wait(lk, [&] { return gen_.load() != seen || stop_.load(); });
                sleepers_.fetch_sub(1);
                spins = 0;
            }
            seen = g;
            part(w);
            pending_.fetch_sub(1, std::memory_order_release);
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> pending_{0}, sleepers_{0};
    std::atomic<bool> stop_{false};
    std::mutex m_;
    std::condition_variable cv_;
    bool touch_ = false;
    char *dst_ = nullptr;
    const char *src_ = nullptr;
    size_t bytes_ = 0, piece_ = 0;
};

int pool_threads() {
    if (const char *e = std::getenv("SLAT_HOST_THREADS")) return std::max(1, std::min(64, std::atoi(e)));
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(8u, hc ? hc : 1u));
}

// A/B (variant builds): SLAT_HOSTIO=runtime (hipMemcpyAsync of the pageable memory itself, the runtime's
// bounce buffers) | register (hipHostRegister of the caller's arrays for the copy)
int hostio_mode() {
    static const int m = [] {
        const char *e = slat_ab_knob("SLAT_HOSTIO");
        if (e && !std::strcmp(e, "runtime")) return 1;
        if (e && !std::strcmp(e, "register")) return 2;
        return 0;
    }();
    return m;
}

// what a "host" segment's memory really is: pageable (0), page-locked host memory from hipHostMalloc
// or hipHostRegister (1), or device / managed memory the runtime knows (2: copied with
// hipMemcpyDefault, which reads the direction from the pointers, never through the staging ring)
int mem_kind(const void *p) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    if (at.type == hipMemoryTypeHost) return 1;
    if (at.type == hipMemoryTypeManaged || at.type == hipMemoryTypeDevice) return 2;
    return 0;
}
bool is_pinned(const void *p) { return mem_kind(p) != 0; }

}  // namespace

struct slat_hostio {
    CopyPool pool{pool_threads()};
    char *slot[kSlots] = {};
    hipEvent_t ev[kSlots] = {};
    bool ok = false;
    slat_hostio() {
        ok = true;
        for (int i = 0; i < kSlots; ++i) {
            if (hipHostMalloc((void **)&slot[i], kChunk, hipHostMallocDefault) != hipSuccess ||
                hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess)
                ok = false;
        }
        if (!ok) (void)hipGetLastError();
    }
    ~slat_hostio() {
        for (int i = 0; i < kSlots; ++i) {
            if (slot[i]) (void)hipHostFree(slot[i]);
            if (ev[i]) (void)hipEventDestroy(ev[i]);
        }
    }
};

void slat_hostio_destroy(slat_ctx *ctx) {
    delete ctx->hio;
    ctx->hio = nullptr;
}

static slat_status get_io(slat_ctx *ctx, slat_hostio **io) {
    if (!ctx->hio) ctx->hio = new slat_hostio();
    if (!ctx->hio->ok) return fail(ctx, SLAT_EOOM, "page-locked staging ring allocation failed");
    *io = ctx->hio;
    return SLAT_OK;
}

namespace {
struct Chunk {
    char *host;
    char *dev;
    size_t bytes;
};

// pageable segments cut into ring-sized chunks; page-locked ones queued as one DMA each
void plan(const slat_hostseg *segs, int n, bool to_dev, hipStream_t s, std::vector<Chunk> &out, hipError_t &err) {
    for (int i = 0; i < n; ++i) {
        const slat_hostseg &g = segs[i];
        if (!g.bytes) continue;
        if (const int kind = mem_kind(g.host)) {
            const hipMemcpyKind mk = kind == 2 ? hipMemcpyDefault : to_dev ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
            const hipError_t e = to_dev ? hipMemcpyAsync(g.dev, g.host, g.bytes, mk, s)
                                        : hipMemcpyAsync(g.host, g.dev, g.bytes, mk, s);
            if (e != hipSuccess) err = e;
            continue;
        }
        for (size_t o = 0; o < g.bytes; o += kChunk)
            out.push_back({(char *)g.host + o, (char *)g.dev + o, std::min(kChunk, g.bytes - o)});
    }
}
}  // namespace

slat_status slat_copy_h2d(slat_ctx *ctx, const slat_hostseg *segs, int n) {
    hipStream_t s = ctx->stream;
    if (hostio_mode() == 1) {
        for (int i = 0; i < n; ++i)
            if (segs[i].bytes) SLAT_HIP(ctx, hipMemcpyAsync(segs[i].dev, segs[i].host, segs[i].bytes, hipMemcpyHostToDevice, s));
        SLAT_HIP(ctx, hipStreamSynchronize(s));
        return SLAT_OK;
    }
    if (hostio_mode() == 2) {
        for (int i = 0; i < n; ++i) {
            if (!segs[i].bytes) continue;
            const bool reg = !is_pinned(segs[i].host) &&
                             hipHostRegister(segs[i].host, segs[i].bytes, hipHostRegisterDefault) == hipSuccess;
            (void)hipGetLastError();
            SLAT_HIP(ctx, hipMemcpyAsync(segs[i].dev, segs[i].host, segs[i].bytes, hipMemcpyHostToDevice, s));
            SLAT_HIP(ctx, hipStreamSynchronize(s));
            if (reg) (void)hipHostUnregister(segs[i].host);
        }
        return SLAT_OK;
    }
    std::vector<Chunk> ch;
    hipError_t err = hipSuccess;
    plan(segs, n, true, s, ch, err);
    SLAT_HIP(ctx, err);
    if (!ch.empty()) {
        slat_hostio *io = nullptr;
        slat_status st = get_io(ctx, &io);
        if (st) return st;
        for (size_t i = 0; i < ch.size(); ++i) {
            const int k = (int)(i % kSlots);
            if (i >= (size_t)kSlots) SLAT_HIP(ctx, hipEventSynchronize(io->ev[k]));  // the slot's last DMA is done
            io->pool.copy(io->slot[k], ch[i].host, ch[i].bytes);
            SLAT_HIP(ctx, hipMemcpyAsync(ch[i].dev, io->slot[k], ch[i].bytes, hipMemcpyHostToDevice, s));
            SLAT_HIP(ctx, hipEventRecord(io->ev[k], s));
        }
    }
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    return SLAT_OK;
}

slat_status slat_copy_d2h(slat_ctx *ctx, const slat_hostseg *segs, int n) {
    hipStream_t s = ctx->stream;
    if (hostio_mode() == 1) {
        for (int i = 0; i < n; ++i)
            if (segs[i].bytes) SLAT_HIP(ctx, hipMemcpyAsync(segs[i].host, segs[i].dev, segs[i].bytes, hipMemcpyDeviceToHost, s));
        SLAT_HIP(ctx, hipStreamSynchronize(s));
        return SLAT_OK;
    }
    if (hostio_mode() == 2) {
        for (int i = 0; i < n; ++i) {
            if (!segs[i].bytes) continue;
            const bool reg = !is_pinned(segs[i].host) &&
                             hipHostRegister(segs[i].host, segs[i].bytes, hipHostRegisterDefault) == hipSuccess;
            (void)hipGetLastError();
            SLAT_HIP(ctx, hipMemcpyAsync(segs[i].host, segs[i].dev, segs[i].bytes, hipMemcpyDeviceToHost, s));
            SLAT_HIP(ctx, hipStreamSynchronize(s));
            if (reg) (void)hipHostUnregister(segs[i].host);
        }
        return SLAT_OK;
    }
    std::vector<Chunk> ch;
    hipError_t err = hipSuccess;
    plan(segs, n, false, s, ch, err);
    SLAT_HIP(ctx, err);
    if (!ch.empty()) {
        slat_hostio *io = nullptr;
        slat_status st = get_io(ctx, &io);
        if (st) return st;
        auto issue = [&](size_t i) -> hipError_t {
            const int k = (int)(i % kSlots);
            hipError_t e = hipMemcpyAsync(io->slot[k], ch[i].dev, ch[i].bytes, hipMemcpyDeviceToHost, s);
            return e == hipSuccess ? hipEventRecord(io->ev[k], s) : e;
        };
        // (SLAT_HOSTIO_CLOCK, variant builds: the host split of the copy on stderr)
        static const bool clk = slat_ab_knob("SLAT_HOSTIO_CLOCK") != nullptr;
        using clock = std::chrono::steady_clock;
        double t_issue = 0, t_touch = 0, t_wait = 0, t_copy = 0;
        auto t = clock::now();
        auto lap = [&](double &acc) {
            if (!clk) return;
            const auto now = clock::now();
            acc += std::chrono::duration<double, std::micro>(now - t).count();
            t = now;
        };
        for (size_t i = 0; i < ch.size() && i < (size_t)kSlots; ++i) SLAT_HIP(ctx, issue(i));
        lap(t_issue);
        // fault in the destination pages under those DMAs (pageable segments only)
        for (int i = 0; i < n; ++i)
            if (segs[i].bytes && !is_pinned(segs[i].host)) io->pool.touch(segs[i].host, segs[i].bytes);
        lap(t_touch);
        for (size_t i = 0; i < ch.size(); ++i) {
            const int k = (int)(i % kSlots);
            SLAT_HIP(ctx, hipEventSynchronize(io->ev[k]));
            lap(t_wait);
            io->pool.copy(ch[i].host, io->slot[k], ch[i].bytes);
            lap(t_copy);
            if (i + kSlots < ch.size()) SLAT_HIP(ctx, issue(i + kSlots));
            lap(t_issue);
        }
        if (clk)
            std::fprintf(stderr, "d2h %zu chunks: issue %.0f touch %.0f wait %.0f copy %.0f us\n", ch.size(), t_issue, t_touch,
                         t_wait, t_copy);
    }
    SLAT_HIP(ctx, hipStreamSynchronize(s));
    return SLAT_OK;
}
