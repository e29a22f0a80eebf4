// Host-side ceilings of the close-time ingest: what one node's host can feed
// its GPUs when every diff comes from the DB as pageable bytes (cycle_manager.py:243-250).
//
//   read     T threads sum a pageable buffer (host-DRAM read bandwidth)
//   copy     T threads copy pageable -> pageable with non-temporal stores (DRAM read + write)
//   stage    T threads copy pageable -> page-locked with non-temporal stores: the library's
//            staging copy pool (pgh_api.cpp copy_stream, CopyPool in pgh_ctx.h) alone, no DMA
//   register hipHostRegister + hipHostUnregister of fresh pageable buffers of one diff's size
//            (page-locking a message in place instead of copying it); register_parallel: T threads
//   h2d      page-locked -> GPU 0 DMA (hipMemcpyAsync)
//   stage+h2d  the staging copy with T threads while GPU 0's DMA reads the other page-locked half
//            (the two compete for DRAM as in a close)
//
// Build: hipcc -O3 -std=c++17 -mavx2 -pthread tools/host_budget.cpp -o tools/_host_budget
// Run:   tools/_host_budget [GiB per buffer, default 4]   -> one JSON line on stdout
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

namespace {

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void run_threads(int t, const std::function<void(int)>& f) {
    std::vector<std::thread> ts;
    for (int k = 1; k < t; ++k) ts.emplace_back(f, k);
    f(0);
    for (auto& x : ts) x.join();
}

uint64_t read_sum(const uint8_t* p, size_t n) {
    __m256i acc = _mm256_setzero_si256();
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_load_si256((const __m256i*)(p + i));
        const __m256i b = _mm256_load_si256((const __m256i*)(p + i + 32));
        const __m256i c = _mm256_load_si256((const __m256i*)(p + i + 64));
        const __m256i d = _mm256_load_si256((const __m256i*)(p + i + 96));
        acc = _mm256_add_epi64(acc, _mm256_add_epi64(_mm256_add_epi64(a, b), _mm256_add_epi64(c, d)));
    }
    alignas(32) uint64_t v[4];
    _mm256_store_si256((__m256i*)v, acc);
    return v[0] + v[1] + v[2] + v[3];
}

void copy_nt(uint8_t* dst, const uint8_t* src, size_t n) {  // both 32-byte aligned, n % 128 == 0
    for (size_t i = 0; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256((const __m256i*)(src + i));
        const __m256i b = _mm256_loadu_si256((const __m256i*)(src + i + 32));
        const __m256i c = _mm256_loadu_si256((const __m256i*)(src + i + 64));
        const __m256i d = _mm256_loadu_si256((const __m256i*)(src + i + 96));
        _mm256_stream_si256((__m256i*)(dst + i), a);
        _mm256_stream_si256((__m256i*)(dst + i + 32), b);
        _mm256_stream_si256((__m256i*)(dst + i + 64), c);
        _mm256_stream_si256((__m256i*)(dst + i + 96), d);
    }
    _mm_sfence();
}

uint8_t* pageable(size_t n) {
    void* p = nullptr;
    if (posix_memalign(&p, 2 << 20, n) != 0) { std::fprintf(stderr, "alloc %zu failed\n", n); std::exit(1); }
    std::memset(p, 1, n);  // fault in
    return (uint8_t*)p;
}

// GB/s of `bytes` moved by T threads each doing f(k, lo, hi) on its slice; best of `reps`
double rate(int t, size_t bytes, int reps, const std::function<void(int, size_t, size_t)>& f) {
    double best = 1e30;
    for (int r = 0; r < reps; ++r) {
        const double t0 = now_s();
        run_threads(t, [&](int k) {
            const size_t per = (bytes / t) & ~(size_t)127;
            const size_t lo = per * k, hi = k == t - 1 ? (bytes & ~(size_t)127) : lo + per;
            f(k, lo, hi);
        });
        best = std::min(best, now_s() - t0);
    }
    return bytes / best / 1e9;
}

#define HIPCK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(2); } \
    } while (0)

}  // namespace

int main(int argc, char** argv) {
    const size_t gib = argc > 1 ? (size_t)std::atoll(argv[1]) : 4;
    const size_t n = gib << 30;
    const int tmax = (int)std::thread::hardware_concurrency();
    std::vector<int> threads = {1, 2, 4, 8, 16};
    uint8_t* a = pageable(n);
    uint8_t* b = pageable(n);
    std::atomic<uint64_t> sink{0};
    std::string js = "{\"tool\": \"tools/host_budget.cpp\", \"buffer_GiB\": " + std::to_string(gib) +
                     ", \"hardware_concurrency\": " + std::to_string(tmax);
    auto series = [&](const char* name, const std::function<double(int)>& g) {
        js += std::string(", \"") + name + "_GBps\": {";
        for (size_t i = 0; i < threads.size(); ++i) {
            char buf[64];
            std::snprintf(buf, sizeof buf, "%s\"%d\": %.1f", i ? ", " : "", threads[i], g(threads[i]));
            js += buf;
        }
        js += "}";
        std::fprintf(stderr, "%s done\n", name);
    };
    series("read", [&](int t) {
        return rate(t, n, 3, [&](int, size_t lo, size_t hi) { sink += read_sum(a + lo, hi - lo); });
    });
    series("copy_pageable", [&](int t) {
        return rate(t, n, 3, [&](int, size_t lo, size_t hi) { copy_nt(b + lo, a + lo, hi - lo); });
    });
    // page-locked staging ring, as the library's (two halves); the copy pool fills it from pageable bytes
    const size_t pin_n = std::min(n, (size_t)2 << 30);
    uint8_t* pin = nullptr;
    HIPCK(hipHostMalloc((void**)&pin, pin_n, hipHostMallocDefault));
    std::memset(pin, 0, pin_n);
    series("stage_to_pinned", [&](int t) {
        return rate(t, pin_n, 3, [&](int, size_t lo, size_t hi) { copy_nt(pin + lo, a + lo, hi - lo); });
    });
    // one ResNet-18 diff's payload (46.8 MB): page-lock it in place instead of copying it
    {
        const size_t m = 46758048;
        const int k = 16;
        std::vector<uint8_t*> bufs;
        for (int i = 0; i < k; ++i) bufs.push_back(pageable(m));
        double t0 = now_s();
        for (auto* p : bufs) HIPCK(hipHostRegister(p, m, hipHostRegisterDefault));
        const double reg = now_s() - t0;
        t0 = now_s();
        for (auto* p : bufs) HIPCK(hipHostUnregister(p));
        const double unreg = now_s() - t0;
        char buf[200];
        std::snprintf(buf, sizeof buf, ", \"register_GBps\": %.1f, \"unregister_GBps\": %.1f, \"register_ms_per_47MB\": %.3f",
                      k * m / reg / 1e9, k * m / unreg / 1e9, reg / k * 1e3);
        js += buf;
        for (auto* p : bufs) std::free(p);
    }
    // page-locking in parallel: T threads each register + unregister their own 47 MB buffers (does
    // pinning scale with threads, as a group's per-GPU ingest threads would need?)
    {
        const size_t m = 46758048;
        const int per = 4;
        std::vector<uint8_t*> bufs;
        for (int i = 0; i < 16 * per; ++i) bufs.push_back(pageable(m));
        series("register_parallel", [&](int t) {
            const double t0 = now_s();
            run_threads(t, [&](int k) {
                for (int i = 0; i < per; ++i) HIPCK(hipHostRegister(bufs[(size_t)(k * per + i)], m, hipHostRegisterDefault));
            });
            const double dt = now_s() - t0;
            run_threads(t, [&](int k) {
                for (int i = 0; i < per; ++i) HIPCK(hipHostUnregister(bufs[(size_t)(k * per + i)]));
            });
            return (double)t * per * m / dt / 1e9;
        });
        for (auto* p : bufs) std::free(p);
    }
    // DMA alone, then the staging copy beside it
    uint8_t* d = nullptr;
    HIPCK(hipSetDevice(0));
    HIPCK(hipMalloc((void**)&d, pin_n));
    hipStream_t s;
    HIPCK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HIPCK(hipMemcpyAsync(d, pin, pin_n, hipMemcpyHostToDevice, s));
    HIPCK(hipStreamSynchronize(s));
    double best = 1e30;
    for (int r = 0; r < 3; ++r) {
        const double t0 = now_s();
        HIPCK(hipMemcpyAsync(d, pin, pin_n, hipMemcpyHostToDevice, s));
        HIPCK(hipStreamSynchronize(s));
        best = std::min(best, now_s() - t0);
    }
    char buf[160];
    std::snprintf(buf, sizeof buf, ", \"h2d_pinned_GBps\": %.1f", pin_n / best / 1e9);
    js += buf;
    std::fprintf(stderr, "h2d done\n");
    series("stage_beside_h2d", [&](int t) {
        // the copy fills the first half while the DMA reads the second half over and over
        const size_t half = pin_n / 2;
        std::atomic<bool> stop{false};
        std::thread dma([&] {
            HIPCK(hipSetDevice(0));
            while (!stop) {
                HIPCK(hipMemcpyAsync(d, pin + half, half, hipMemcpyHostToDevice, s));
                HIPCK(hipStreamSynchronize(s));
            }
        });
        const double g = rate(t, half, 3, [&](int, size_t lo, size_t hi) { copy_nt(pin + lo, a + lo, hi - lo); });
        stop = true;
        dma.join();
        return g;
    });
    js += "}";
    std::printf("%s\n", js.c_str());
    (void)hipFree(d);
    (void)hipHostFree(pin);
    std::free(a);
    std::free(b);
    return sink == 42 ? 3 : 0;
}
