// H2D experiment (not product code): one pinned-host -> HBM stream vs two or four concurrent
// streams (each copying its share), to see whether more DMA queues beat the single-stream rate.
// Build: hipcc -O3 --offload-arch=gfx950 tools/exp_h2d.hip -o tools/_exp_h2d
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

int main() {
    const size_t total = 2ull << 30;  // 2 GiB per trial
    void* h;
    CK(hipHostMalloc(&h, total, 0));
    memset(h, 1, total);
    void* d;
    CK(hipMalloc(&d, total));
    for (int ns : {1, 2, 4}) {
        std::vector<hipStream_t> st(ns);
        for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        for (size_t piece : {64ull << 20, 512ull << 20}) {
            double best = 0;
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipDeviceSynchronize());
                auto t0 = std::chrono::steady_clock::now();
                size_t off = 0;
                int k = 0;
                while (off < total) {
                    const size_t n = std::min(piece, total - off);
                    CK(hipMemcpyAsync((char*)d + off, (char*)h + off, n, hipMemcpyHostToDevice, st[k % ns]));
                    off += n;
                    ++k;
                }
                CK(hipDeviceSynchronize());
                const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                best = std::max(best, total / s / 1e9);
            }
            printf("{\"streams\": %d, \"piece_MB\": %zu, \"GBps\": %.2f}\n", ns, piece >> 20, best);
            fflush(stdout);
        }
        for (auto& s : st) CK(hipStreamDestroy(s));
    }
    return 0;
}
