// Fill experiment (not product code): is the config-4 on-device generator (k_synth_f32 kind 1:
// one splitmix64 per 4 params) bound by HBM writes or by its 64-bit hash arithmetic?  Writes one
// 500-client chunk of a 12.5M-param shard into the column-blocked slab layout (256 KiB blocks,
// DESIGN.md section 3) with:
//   const   a constant per row (pure store stream: the write ceiling of this shape)
//   kind1   the product's fast generator (one splitmix64 -> four 16-bit fields per 4 params)
//   kind2   one splitmix64 per 8 params, the second 64 bits from one xorshift step of the first
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/exp_fill.hip -o tools/_exp_fill
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int BLOCK = 256;
constexpr int64_t LD = 65536;

__device__ __forceinline__ uint64_t sm64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t xs64(uint64_t x) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
}

__device__ __forceinline__ size_t at(int64_t rows, int64_t r, int64_t i) {
    return (size_t)(i >> 16) * (size_t)(rows * LD) + (size_t)r * LD + (size_t)(i & (LD - 1));
}

__device__ __forceinline__ f32x4 four(uint64_t h, float s2) {
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (float)((int32_t)((h >> (16 * e)) & 0xFFFF) - 32768) * s2;
    return v;
}

template <int KIND>
__global__ __launch_bounds__(BLOCK) void k_fill(float* out, int64_t rows, int64_t ncols, uint64_t seed, float s2) {
    const int64_t per = KIND == 2 ? 8 : 4;
    for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
        const uint64_t key = sm64(seed ^ (uint64_t)r * 0xD1B54A32D192ED03ull);
        for (int64_t q = (int64_t)blockIdx.x * BLOCK + threadIdx.x; q < ncols / per; q += (int64_t)gridDim.x * BLOCK) {
            const int64_t g = per * q;
            if constexpr (KIND == 0) {
                f32x4 v = {s2, s2, s2, s2};
                __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(out + at(rows, r, g)));
            } else if constexpr (KIND == 1) {
                __builtin_nontemporal_store(four(sm64(key + (uint64_t)q), s2), reinterpret_cast<f32x4*>(out + at(rows, r, g)));
            } else {
                const uint64_t h = sm64(key + (uint64_t)q);
                f32x4* d = reinterpret_cast<f32x4*>(out + at(rows, r, g));
                __builtin_nontemporal_store(four(h, s2), d);
                __builtin_nontemporal_store(four(xs64(h), s2), d + 1);
            }
        }
    }
}

int main(int argc, char** argv) {
    const int64_t rows = 500, P = 12'500'000;
    const int64_t ncols = (P + LD - 1) / LD * LD;
    const size_t bytes = (size_t)rows * ncols * 4;
    float* d;
    CK(hipMalloc(&d, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    struct Case { const char* name; int kind; int gx; int gy; };
    std::vector<Case> cases;
    for (int kind : {0, 1, 2})
        for (int gx : {1024, 256})
            for (int gy : {500, 64}) cases.push_back({kind == 0 ? "const" : kind == 1 ? "kind1" : "kind2", kind, gx, gy});
    for (int rep = 0; rep < 2; ++rep) {
        for (const auto& c : cases) {
            std::vector<float> ms;
            for (int it = 0; it < 5; ++it) {
                CK(hipEventRecord(a, 0));
                const dim3 grid((unsigned)c.gx, (unsigned)c.gy);
                if (c.kind == 0) k_fill<0><<<grid, BLOCK>>>(d, rows, ncols, 7, 1e-5f);
                else if (c.kind == 1) k_fill<1><<<grid, BLOCK>>>(d, rows, ncols, 7, 1e-5f);
                else k_fill<2><<<grid, BLOCK>>>(d, rows, ncols, 7, 1e-5f);
                CK(hipGetLastError());
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float t;
                CK(hipEventElapsedTime(&t, a, b));
                ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            printf("{\"case\": \"%s_gx%d_gy%d\", \"rep\": %d, \"ms_median\": %.4f, \"write_GBps\": %.1f}\n", c.name, c.gx,
                   c.gy, rep, ms[2], bytes / (ms[2] / 1e3) / 1e9);
            fflush(stdout);
        }
    }
    CK(hipFree(d));
    return 0;
}
