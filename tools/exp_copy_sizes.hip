// HBM <-> page-locked host copy rate by copy size, and for one 47 MB transfer split over k
// streams at once.  exp_pinned_kinds measured 27.4 GB/s for one 47 MB copy of every allocation
// kind, while 2 GB copies (host_budget) and the library's 128 MiB staging fills run at ~57 GB/s.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/exp_copy_sizes.hip -o tools/_exp_copy_sizes
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(2); } \
    } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
    const size_t maxn = 2ull << 30;
    uint8_t *d = nullptr, *h = nullptr;
    CK(hipMalloc((void**)&d, maxn));
    CK(hipMemset(d, 3, maxn));
    CK(hipHostMalloc((void**)&h, maxn, hipHostMallocDefault));
    std::memset(h, 1, maxn);
    std::vector<hipStream_t> ss(8);
    for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // wall time (host) of k concurrent pieces covering n bytes, best of reps
    auto run = [&](size_t n, int k, bool d2h, int reps) {
        double best = 1e30;
        for (int r = 0; r < reps; ++r) {
            CK(hipDeviceSynchronize());
            const double t0 = now();
            const size_t per = (n / k + 4095) & ~(size_t)4095;
            for (int i = 0; i < k; ++i) {
                const size_t off = per * i;
                if (off >= n) break;
                const size_t len = std::min(per, n - off);
                if (d2h) CK(hipMemcpyAsync(h + off, d + off, len, hipMemcpyDeviceToHost, ss[i]));
                else CK(hipMemcpyAsync(d + off, h + off, len, hipMemcpyHostToDevice, ss[i]));
            }
            for (int i = 0; i < k; ++i) CK(hipStreamSynchronize(ss[i]));
            best = std::min(best, now() - t0);
        }
        return n / best / 1e9;
    };
    std::string js = "{\"tool\": \"tools/exp_copy_sizes.hip\"";
    for (int dir = 0; dir < 2; ++dir) {
        const bool d2h = dir == 0;
        js += std::string(", \"") + (d2h ? "d2h" : "h2d") + "_GBps_by_size\": {";
        const size_t sizes[] = {1u << 20, 8u << 20, 46758048, 128u << 20, 512u << 20, 2ull << 30};
        bool first = true;
        for (size_t n : sizes) {
            char b[80];
            std::snprintf(b, sizeof b, "%s\"%zu\": %.1f", first ? "" : ", ", n, run(n, 1, d2h, 7));
            js += b;
            first = false;
        }
        js += "}";
        js += std::string(", \"") + (d2h ? "d2h" : "h2d") + "_47MB_GBps_by_streams\": {";
        first = true;
        for (int k : {1, 2, 4, 8}) {
            char b[80];
            std::snprintf(b, sizeof b, "%s\"%d\": %.1f", first ? "" : ", ", k, run(46758048, k, d2h, 7));
            js += b;
            first = false;
        }
        js += "}";
    }
    js += "}";
    std::printf("%s\n", js.c_str());
    return 0;
}
