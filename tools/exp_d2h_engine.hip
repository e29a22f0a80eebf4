// Which engine should carry the report-time close's 47 MB HBM -> page-locked host copy while the
// last fold ranges still run?  hipMemcpyAsync(DeviceToHost) from HBM into page-locked memory ran as
// blit kernels (__amd_rocclr_copyBuffer in every trace), which take CUs and HBM from the fold
// (r03am: the 8 FINAL ranges 1.08 ms beside the D2H pieces vs 0.65 ms alone).  This measures, on
// one GPU: a read-bound kernel shaped like the fold (sums a 3.7 GB buffer: 80 ResNet-18 rows) alone,
// the 47 MB copy alone, and both together on two streams -- for the copy kinds DeviceToHost and
// DeviceToDeviceNoCU (a copy engine, no CUs), and in 8 MiB pieces as the library issues it.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/exp_d2h_engine.hip -o tools/_exp_d2h_engine
// Run:   tools/_exp_d2h_engine          -> one JSON line
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(2); } \
    } while (0)

__global__ __launch_bounds__(256) void k_read(const float4* __restrict__ a, size_t n4, float* out) {
    float s = 0.f;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;  // keep the loads
}

struct Timing { float kernel_ms, copy_ms, both_ms; };

int main() {
    const size_t fold_bytes = 80ull * 46758048ull, copy_bytes = 46758048ull, piece = 8u << 20;
    float4* big = nullptr;
    float* out = nullptr;
    uint8_t *src = nullptr, *host = nullptr;
    CK(hipMalloc((void**)&big, fold_bytes));
    CK(hipMemset(big, 0, fold_bytes));
    CK(hipMalloc((void**)&out, 64));
    CK(hipMalloc((void**)&src, copy_bytes));
    CK(hipMemset(src, 1, copy_bytes));
    CK(hipHostMalloc((void**)&host, copy_bytes, hipHostMallocDefault));
    hipStream_t sk, sc;
    CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
    hipEvent_t k0, k1, c0, c1;
    for (auto* e : {&k0, &k1, &c0, &c1}) CK(hipEventCreate(e));
    const int grid = 256 * 8;
    auto kernel = [&] {
        CK(hipEventRecord(k0, sk));
        k_read<<<grid, 256, 0, sk>>>(big, fold_bytes / 16, out);
        CK(hipEventRecord(k1, sk));
    };
    auto copy = [&](hipMemcpyKind kind, bool pieces) {
        CK(hipEventRecord(c0, sc));
        if (pieces) {
            for (size_t off = 0; off < copy_bytes; off += piece)
                CK(hipMemcpyAsync(host + off, src + off, std::min(piece, copy_bytes - off), kind, sc));
        } else {
            CK(hipMemcpyAsync(host, src, copy_bytes, kind, sc));
        }
        CK(hipEventRecord(c1, sc));
    };
    auto ms = [](hipEvent_t a, hipEvent_t b) { float x = 0; CK(hipEventElapsedTime(&x, a, b)); return x; };
    auto run = [&](hipMemcpyKind kind, bool pieces, int reps) {
        std::vector<float> ka, ca, kb, cb, both;
        for (int r = 0; r < reps; ++r) {
            kernel(); CK(hipDeviceSynchronize()); ka.push_back(ms(k0, k1));
            copy(kind, pieces); CK(hipDeviceSynchronize()); ca.push_back(ms(c0, c1));
            kernel(); copy(kind, pieces); CK(hipDeviceSynchronize());
            kb.push_back(ms(k0, k1)); cb.push_back(ms(c0, c1));
            float t0 = 0;
            CK(hipEventElapsedTime(&t0, k0, c1));
            both.push_back(std::max(ms(k0, k1), t0));
        }
        auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
        char buf[300];
        std::snprintf(buf, sizeof buf,
                      "{\"kernel_alone_ms\": %.4f, \"copy_alone_ms\": %.4f, \"kernel_beside_copy_ms\": %.4f, "
                      "\"copy_beside_kernel_ms\": %.4f, \"span_ms\": %.4f}",
                      med(ka), med(ca), med(kb), med(cb), med(both));
        return std::string(buf);
    };
    kernel(); copy(hipMemcpyDeviceToHost, false); CK(hipDeviceSynchronize());  // warm-up
    std::string js = "{\"tool\": \"tools/exp_d2h_engine.hip\", \"fold_bytes\": " + std::to_string(fold_bytes) +
                     ", \"copy_bytes\": " + std::to_string(copy_bytes);
    js += ", \"d2h_whole\": " + run(hipMemcpyDeviceToHost, false, 9);
    js += ", \"d2h_pieces\": " + run(hipMemcpyDeviceToHost, true, 9);
    js += ", \"nocu_whole\": " + run(hipMemcpyDeviceToDeviceNoCU, false, 9);
    js += ", \"nocu_pieces\": " + run(hipMemcpyDeviceToDeviceNoCU, true, 9);
    bool same = true;
    std::vector<uint8_t> chk(1 << 20);
    CK(hipMemcpy(chk.data(), src, chk.size(), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < chk.size(); ++i) same = same && host[i] == chk[i];
    js += std::string(", \"nocu_bytes_ok\": ") + (same ? "true" : "false") + "}";
    std::printf("%s\n", js.c_str());
    return 0;
}
