// K5 (k_gather_f32) launch shapes, measured alone: a ResNet-18 report (62 float payloads at the
// byte offsets a State message puts them, most not 4-byte aligned) gathered from a DMA'd message
// into a blocked slab row (256 KiB blocks, 100 rows), HIP events around each of 30 launches per variant, each right after
// the message's DMA from page-locked memory (as on the report path), variants
// interleaved.  Variants: the chunk of floats per workgroup (1024 / 2048 / 4096 / 8192) and, for
// 4096, the four 16-byte loads of a lane issued before any store.  Every variant's row is compared
// with a host gather.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/exp_gather.hip -o tools/_exp_gather
// Run:   tools/_exp_gather          -> one JSON line
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../pygrid_amd/csrc/pgh_kernels.h"

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(2); } \
    } while (0)

using pgh::GChunk;
using pgh::SlabMap;
constexpr int BLOCK = 256;

// the library's form: lane loop, one 16-byte load then its store
__global__ __launch_bounds__(BLOCK) void k_loop(const uint8_t* bytes, const GChunk* tab, float* row, SlabMap m) {
    const GChunk ch = tab[blockIdx.x];
    const int head = (int)min((int64_t)ch.n, (4 - (ch.dst & 3)) & 3);
    const int body = (ch.n - head) & ~3;
    const uint32_t sh = (uint32_t)(ch.src & 3);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(bytes + (ch.src & ~int64_t(3)));
    auto one = [&](int t) {
        const uint32_t lo = w[t];
        const uint32_t v = sh ? __builtin_amdgcn_alignbyte(w[t + 1], lo, sh) : lo;
        row[m.at(ch.dst + t)] = __uint_as_float(v);
    };
    if ((int)threadIdx.x < head) one((int)threadIdx.x);
    const int tail0 = head + body;
    if ((int)threadIdx.x < ch.n - tail0) one(tail0 + (int)threadIdx.x);
    for (int q = (int)threadIdx.x * 4; q < body; q += BLOCK * 4) {
        const int t = head + q;
        uint4 a;
        __builtin_memcpy(&a, w + t, 16);
        float4 o;
        if (sh) {
            const uint32_t e = w[t + 4];
            o.x = __uint_as_float(__builtin_amdgcn_alignbyte(a.y, a.x, sh));
            o.y = __uint_as_float(__builtin_amdgcn_alignbyte(a.z, a.y, sh));
            o.z = __uint_as_float(__builtin_amdgcn_alignbyte(a.w, a.z, sh));
            o.w = __uint_as_float(__builtin_amdgcn_alignbyte(e, a.w, sh));
        } else {
            o = make_float4(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), __uint_as_float(a.w));
        }
        *reinterpret_cast<float4*>(row + m.at(ch.dst + t)) = o;
    }
}

// every load of the lane (up to U) issued before the first store
template <int U>
__global__ __launch_bounds__(BLOCK) void k_batched(const uint8_t* bytes, const GChunk* tab, float* row, SlabMap m) {
    const GChunk ch = tab[blockIdx.x];
    const int head = (int)min((int64_t)ch.n, (4 - (ch.dst & 3)) & 3);
    const int body = (ch.n - head) & ~3;
    const uint32_t sh = (uint32_t)(ch.src & 3);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(bytes + (ch.src & ~int64_t(3)));
    auto one = [&](int t) {
        const uint32_t lo = w[t];
        const uint32_t v = sh ? __builtin_amdgcn_alignbyte(w[t + 1], lo, sh) : lo;
        row[m.at(ch.dst + t)] = __uint_as_float(v);
    };
    if ((int)threadIdx.x < head) one((int)threadIdx.x);
    const int tail0 = head + body;
    if ((int)threadIdx.x < ch.n - tail0) one(tail0 + (int)threadIdx.x);
    uint4 a[U];
    uint32_t e[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int q = ((int)threadIdx.x + u * BLOCK) * 4;
        if (q < body) {
            __builtin_memcpy(&a[u], w + head + q, 16);
            e[u] = sh ? w[head + q + 4] : 0u;
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int q = ((int)threadIdx.x + u * BLOCK) * 4;
        if (q < body) {
            float4 o;
            if (sh) {
                o.x = __uint_as_float(__builtin_amdgcn_alignbyte(a[u].y, a[u].x, sh));
                o.y = __uint_as_float(__builtin_amdgcn_alignbyte(a[u].z, a[u].y, sh));
                o.z = __uint_as_float(__builtin_amdgcn_alignbyte(a[u].w, a[u].z, sh));
                o.w = __uint_as_float(__builtin_amdgcn_alignbyte(e[u], a[u].w, sh));
            } else {
                o = make_float4(__uint_as_float(a[u].x), __uint_as_float(a[u].y), __uint_as_float(a[u].z),
                                __uint_as_float(a[u].w));
            }
            *reinterpret_cast<float4*>(row + m.at(ch.dst + head + q)) = o;
        }
    }
}

static const int64_t NUMEL[] = {9408, 64, 64, 36864, 64, 64, 36864, 64, 64, 36864, 64, 64, 36864, 64, 64, 73728,
                                128, 128, 147456, 128, 128, 8192, 128, 128, 147456, 128, 128, 147456, 128, 128,
                                294912, 256, 256, 589824, 256, 256, 32768, 256, 256, 589824, 256, 256, 589824, 256,
                                256, 1179648, 512, 512, 2359296, 512, 512, 131072, 512, 512, 2359296, 512, 512,
                                2359296, 512, 512, 512000, 1000};

int main() {
    const int T = (int)(sizeof NUMEL / sizeof NUMEL[0]);
    // message layout: each payload behind a few dozen bytes of framing of varying length
    std::vector<int64_t> src(T);
    int64_t pos = 61, P = 0;
    for (int t = 0; t < T; ++t) {
        pos += 23 + (t * 7) % 19;
        src[t] = pos;
        pos += 4 * NUMEL[t];
        P += NUMEL[t];
    }
    const size_t msg = (size_t)pos + 64;
    const int64_t ld = 65536, rows = 100, nb = (P + ld - 1) / ld, slot = 37;
    SlabMap m{ld, rows * ld, 16, ld - 1, 0};
    std::vector<uint8_t> h(msg);
    for (size_t i = 0; i < msg; ++i) h[i] = (uint8_t)(i * 2654435761u >> 13);
    uint8_t* d_msg = nullptr;
    float* d_slab = nullptr;
    CK(hipMalloc((void**)&d_msg, msg));
    CK(hipMemcpy(d_msg, h.data(), msg, hipMemcpyHostToDevice));
    CK(hipMalloc((void**)&d_slab, (size_t)nb * rows * ld * 4));
    float* row = d_slab + slot * ld;
    std::vector<float> want((size_t)P);
    {
        int64_t o = 0;
        for (int t = 0; t < T; ++t) {
            std::memcpy(&want[(size_t)o], h.data() + src[t], 4 * NUMEL[t]);
            o += NUMEL[t];
        }
    }
    auto table = [&](int C) {
        std::vector<GChunk> tab;
        int64_t dst = 0;
        for (int t = 0; t < T; ++t) {
            for (int64_t k = 0; k < NUMEL[t]; k += C)
                tab.push_back({src[t] + 4 * k, dst + k, (int32_t)std::min<int64_t>(C, NUMEL[t] - k), 0});
            dst += NUMEL[t];
        }
        GChunk* d = nullptr;
        CK(hipMalloc((void**)&d, tab.size() * sizeof(GChunk)));
        CK(hipMemcpy(d, tab.data(), tab.size() * sizeof(GChunk), hipMemcpyHostToDevice));
        return std::make_pair(d, (int)tab.size());
    };
    struct V { const char* name; int C; int kind; };
    const V vars[] = {{"loop_1024", 1024, 0}, {"loop_2048", 2048, 0}, {"loop_4096", 4096, 0}, {"loop_8192", 8192, 0},
                      {"batched_1024", 1024, 1}, {"batched_2048", 2048, 2}, {"batched_4096", 4096, 4}};
    const int NV = (int)(sizeof vars / sizeof vars[0]);
    std::vector<std::pair<GChunk*, int>> tabs;
    for (auto& v : vars) tabs.push_back(table(v.C));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto launch = [&](int i) {
        const auto& t = tabs[i];
        const int k = vars[i].kind;
        if (k == 0) k_loop<<<t.second, BLOCK, 0, s>>>(d_msg, t.first, row, m);
        else if (k == 1) k_batched<1><<<t.second, BLOCK, 0, s>>>(d_msg, t.first, row, m);
        else if (k == 2) k_batched<2><<<t.second, BLOCK, 0, s>>>(d_msg, t.first, row, m);
        else k_batched<4><<<t.second, BLOCK, 0, s>>>(d_msg, t.first, row, m);
    };
    std::vector<float> got((size_t)P);
    std::vector<std::vector<float>> per(NV);
    std::string ok;
    for (int i = 0; i < NV; ++i) {  // correctness + warm-up
        CK(hipMemset(d_slab, 0, (size_t)nb * rows * ld * 4));
        launch(i);
        CK(hipStreamSynchronize(s));
        for (int64_t j = 0; j < nb; ++j) {
            const int64_t n = std::min(ld, P - j * ld);
            CK(hipMemcpy(&got[(size_t)(j * ld)], row + j * rows * ld, 4 * n, hipMemcpyDeviceToHost));
        }
        ok += std::string(i ? ", " : "") + "\"" + vars[i].name + "\": " +
              (std::memcmp(got.data(), want.data(), 4 * (size_t)P) == 0 ? "true" : "false");
    }
    // each timed launch follows the message's DMA from page-locked memory, as on the report path
    uint8_t* h_pin = nullptr;
    CK(hipHostMalloc((void**)&h_pin, msg, hipHostMallocDefault));
    std::memcpy(h_pin, h.data(), msg);
    for (int r = 0; r < 30; ++r)
        for (int i = 0; i < NV; ++i) {
            CK(hipMemcpyAsync(d_msg, h_pin, msg, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(a, s));
            launch(i);
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            per[i].push_back(ms * 1000.f);  // us per launch
        }
    std::string js = "{\"tool\": \"tools/exp_gather.hip\", \"P\": " + std::to_string(P) + ", \"alg_bytes\": " +
                     std::to_string(8 * P) + ", \"bit_exact\": {" + ok + "}, \"us_per_launch_median\": {";
    for (int i = 0; i < NV; ++i) {
        auto v = per[i];
        std::sort(v.begin(), v.end());
        char buf[160];
        std::snprintf(buf, sizeof buf, "%s\"%s\": %.2f", i ? ", " : "", vars[i].name, v[v.size() / 2]);
        js += buf;
    }
    js += "}, \"TBps_of_8P\": {";
    for (int i = 0; i < NV; ++i) {
        auto v = per[i];
        std::sort(v.begin(), v.end());
        char buf[160];
        std::snprintf(buf, sizeof buf, "%s\"%s\": %.2f", i ? ", " : "", vars[i].name, 8.0 * P / (v[v.size() / 2] * 1e-6) / 1e12);
        js += buf;
    }
    js += "}}";
    std::printf("%s\n", js.c_str());
    return 0;
}
