// D2H / H2D rates of one 47 MB copy (a ResNet-18 checkpoint) between HBM and page-locked host
// memory of each allocation kind: hipHostMalloc Default / NonCoherent / Coherent / WriteCombined /
// NumaUser, and hipHostRegister'd malloc memory.  The library stages through such buffers (its
// pinned ring, the peek buffer, report blocks); exp_d2h_engine measured 1.63 ms (29 GB/s) for the
// D2H into Default memory.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/exp_pinned_kinds.hip -o tools/_exp_pinned_kinds
#include <hip/hip_runtime.h>

#include <algorithm>
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

int main() {
    const size_t n = 46758048ull;
    uint8_t* d = nullptr;
    CK(hipMalloc((void**)&d, n));
    CK(hipMemset(d, 3, n));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    struct Kind { const char* name; unsigned flags; bool reg; };
    std::vector<Kind> kinds = {{"default", hipHostMallocDefault, false},
                               {"noncoherent", hipHostMallocNonCoherent, false},
                               {"coherent", hipHostMallocCoherent, false},
                               {"writecombined", hipHostMallocWriteCombined, false},
                               {"numauser", hipHostMallocNumaUser, false},
                               {"registered", 0, true}};
    std::string js = "{\"tool\": \"tools/exp_pinned_kinds.hip\", \"bytes\": " + std::to_string(n);
    for (auto& k : kinds) {
        uint8_t* h = nullptr;
        if (k.reg) {
            h = (uint8_t*)std::aligned_alloc(4096, (n + 4095) / 4096 * 4096);
            std::memset(h, 1, n);
            CK(hipHostRegister(h, n, hipHostRegisterDefault));
        } else {
            if (hipHostMalloc((void**)&h, n, k.flags) != hipSuccess) {
                (void)hipGetLastError();
                js += std::string(", \"") + k.name + "\": null";
                continue;
            }
            std::memset(h, 1, n);
        }
        auto rate = [&](bool d2h) {
            std::vector<float> t;
            for (int r = 0; r < 7; ++r) {
                CK(hipEventRecord(a, s));
                if (d2h) CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s));
                else CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
                CK(hipEventRecord(b, s));
                CK(hipStreamSynchronize(s));
                float x = 0;
                CK(hipEventElapsedTime(&x, a, b));
                t.push_back(x);
            }
            std::sort(t.begin(), t.end());
            return t[t.size() / 2];
        };
        const float dh = rate(true), hd = rate(false);
        char buf[200];
        std::snprintf(buf, sizeof buf, ", \"%s\": {\"d2h_ms\": %.4f, \"d2h_GBps\": %.1f, \"h2d_ms\": %.4f, \"h2d_GBps\": %.1f}",
                      k.name, dh, n / dh / 1e6, hd, n / hd / 1e6);
        js += buf;
        if (k.reg) { CK(hipHostUnregister(h)); std::free(h); }
        else CK(hipHostFree(h));
    }
    js += "}";
    std::printf("%s\n", js.c_str());
    return 0;
}
