// Layout experiment 2 (not product code; the r01l evidence for the column-blocked slab, results in
// profiles/r01l/layout_experiment/): row-major [rows][ld] (the product kernel on one block) vs
// column-blocked [P/B][rows][B] for the fp32 fold and the int64 share sum, interleaved rounds
// (median), plus the H2D rate of the 2-D copies a blocked slab needs.
//
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Ipygrid_amd/csrc -Iinclude \
//          tools/exp_layout2.hip pygrid_amd/csrc/pgh_kernels.hip -o tools/_exp_layout2
// Run:   tools/_exp_layout2 f32|i64|h2d
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "pgh_kernels.h"

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

template <int U, int TB>
__global__ __launch_bounds__(TB) void k_blk_f32(const float* slab, int n, int bshift, int64_t bstride, int64_t p,
                                                const float* ckpt, float* out, float divisor) {
    const int64_t i = ((int64_t)blockIdx.x * TB + threadIdx.x) * 4;
    if (i >= p) return;
    const int64_t B = (int64_t)1 << bshift;
    const float* col = slab + (i >> bshift) * bstride + (i & (B - 1));
    f32x4 acc = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(col));
    int r = 1;
    for (; r + U <= n; r += U) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(col + (size_t)(r + u) * B));
#pragma unroll
        for (int u = 0; u < U; ++u) acc = acc + v[u];
    }
    for (; r < n; ++r) acc = acc + __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(col + (size_t)r * B));
    *reinterpret_cast<f32x4*>(out + i) = *reinterpret_cast<const f32x4*>(ckpt + i) - acc / divisor;
}

template <int U, int TB, int VEC>
__global__ __launch_bounds__(TB) void k_blk_i64(const int64_t* slab, int n, int bshift, int64_t bstride, int64_t p,
                                                int64_t* sum, float* dec, float divisor) {
    const int64_t i = ((int64_t)blockIdx.x * TB + threadIdx.x) * VEC;
    if (i >= p) return;
    const int64_t B = (int64_t)1 << bshift;
    const int64_t* col = slab + (i >> bshift) * bstride + (i & (B - 1));
    using T = typename std::conditional<VEC == 2, u64x2, unsigned long long>::type;
    T acc{};
    int r = 0;
    for (; r + U <= n; r += U) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(reinterpret_cast<const T*>(col + (size_t)(r + u) * B));
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    for (; r < n; ++r) acc += __builtin_nontemporal_load(reinterpret_cast<const T*>(col + (size_t)r * B));
    if constexpr (VEC == 2) {
        for (int e = 0; e < 2; ++e) { sum[i + e] = (int64_t)acc[e]; dec[i + e] = (float)(int64_t)acc[e] / divisor; }
    } else {
        sum[i] = (int64_t)acc; dec[i] = (float)(int64_t)acc / divisor;
    }
}

struct Case {
    std::string name;
    double bytes;
    std::function<void()> f;
    std::vector<float> ms;
};

void run_cases(std::vector<Case>& cs, int rounds, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto& c : cs) c.f();
    CK(hipDeviceSynchronize());
    for (int k = 0; k < rounds; ++k)
        for (auto& c : cs) {
            CK(hipEventRecord(a, 0));
            for (int r = 0; r < reps; ++r) c.f();
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            c.ms.push_back(ms / reps);
        }
    for (auto& c : cs) {
        std::sort(c.ms.begin(), c.ms.end());
        const float med = c.ms[c.ms.size() / 2];
        printf("{\"case\": \"%s\", \"ms_median\": %.4f, \"ms_min\": %.4f, \"GBps_median\": %.1f}\n", c.name.c_str(), med,
               c.ms[0], c.bytes / (med * 1e-3) / 1e9);
    }
    fflush(stdout);
}

int ilog2(int64_t b) { int s = 0; while ((1ll << s) < b) ++s; return s; }

int main(int argc, char** argv) {
    const std::string what = argc > 1 ? argv[1] : "f32";
    const int64_t P = 11689512;
    if (what == "f32") {
        const int N = 1000;
        const int64_t ld = (P + 63) / 64 * 64;
        const int64_t Pmax = (P + 65535) / 65536 * 65536;  // room for the widest blocking
        float *slab, *acc, *ckpt, *out;
        CK(hipMalloc(&slab, (size_t)N * Pmax * 4));
        CK(hipMalloc(&acc, Pmax * 4));
        CK(hipMalloc(&ckpt, Pmax * 4));
        CK(hipMalloc(&out, Pmax * 4));
        CK(pgh::launch_synth_f32(slab, pgh::single_block(Pmax), Pmax, N, Pmax, 1, pgh::STREAM_DIFF, 0, 0, pgh::DIFF_SCALE, 0));
        CK(pgh::launch_synth_f32(ckpt, pgh::single_block(Pmax), Pmax, 1, Pmax, 1, pgh::STREAM_CKPT, 0, 0, pgh::CKPT_SCALE, 0));
        CK(hipDeviceSynchronize());
        const double alg = 4.0 * N * P + 8.0 * P;
        std::vector<Case> cs;
        for (int v : {14, 11}) {
            pgh::FedavgArgs a{};
            a.diffs = slab; a.map = pgh::single_block(ld); a.n_rows = N; a.client0 = 0; a.p = P; a.acc = acc; a.ckpt = ckpt; a.out = out;
            a.divisor = (float)N; a.flags = pgh::FL_FIRST | pgh::FL_FINAL; a.mode = pgh::MODE_MEAN; a.variant = v;
            cs.push_back({"rowmaj_v" + std::to_string(v), alg, [a] { CK(pgh::launch_fedavg(a, 0)); }, {}});
        }
        for (int64_t B : {256, 1024, 2048, 4096, 8192, 16384, 65536}) {
            const int bs = ilog2(B);
            const int64_t bstride = (int64_t)N * B;
            const unsigned g256 = (unsigned)((P / 4 + 255) / 256), g64 = (unsigned)((P / 4 + 63) / 64);
            cs.push_back({"blk" + std::to_string(B) + "_u16_tb256", alg,
                          [=] { k_blk_f32<16, 256><<<g256, 256>>>(slab, N, bs, bstride, P, ckpt, out, (float)N); }, {}});
            cs.push_back({"blk" + std::to_string(B) + "_u16_tb64", alg,
                          [=] { k_blk_f32<16, 64><<<g64, 64>>>(slab, N, bs, bstride, P, ckpt, out, (float)N); }, {}});
            cs.push_back({"blk" + std::to_string(B) + "_u8_tb256", alg,
                          [=] { k_blk_f32<8, 256><<<g256, 256>>>(slab, N, bs, bstride, P, ckpt, out, (float)N); }, {}});
        }
        run_cases(cs, 7, 2);
    } else if (what == "i64") {
        const int N = 1000, S = 2, R = N * S;
        const int64_t ld = (P + 63) / 64 * 64;
        const int64_t Pmax = (P + 65535) / 65536 * 65536;
        int64_t *slab, *sum;
        float* dec;
        uint64_t* acc;
        CK(hipMalloc(&slab, (size_t)R * Pmax * 8));
        CK(hipMalloc(&sum, Pmax * 8));
        CK(hipMalloc(&acc, Pmax * 8));
        CK(hipMalloc(&dec, Pmax * 4));
        CK(pgh::launch_synth_shares(slab, pgh::single_block(Pmax), Pmax, N, S, Pmax, 1, 0, 0, 1000.f, 0));
        CK(hipDeviceSynchronize());
        const double alg = 8.0 * R * P + 12.0 * P;
        std::vector<Case> cs;
        for (int v : {14, 11}) {
            pgh::SecaggArgs a{};
            a.shares = slab; a.map = pgh::single_block(ld); a.n_rows = R; a.p = P; a.acc = acc; a.sum_out = sum; a.dec_out = dec;
            a.divisor = 1000.f; a.flags = pgh::FL_FIRST | pgh::FL_FINAL; a.variant = v;
            cs.push_back({"rowmaj_v" + std::to_string(v), alg, [a] { CK(pgh::launch_secagg(a, 0)); }, {}});
        }
        for (int64_t B : {128, 512, 2048, 8192, 32768}) {
            const int bs = ilog2(B);
            const int64_t bstride = (int64_t)R * B;
            const unsigned g2 = (unsigned)((P / 2 + 255) / 256), g2s = (unsigned)((P / 2 + 63) / 64),
                           g1 = (unsigned)((P + 63) / 64);
            cs.push_back({"blk" + std::to_string(B) + "_vec2_u16_tb256", alg,
                          [=] { k_blk_i64<16, 256, 2><<<g2, 256>>>(slab, R, bs, bstride, P, sum, dec, 1000.f); }, {}});
            cs.push_back({"blk" + std::to_string(B) + "_vec2_u16_tb64", alg,
                          [=] { k_blk_i64<16, 64, 2><<<g2s, 64>>>(slab, R, bs, bstride, P, sum, dec, 1000.f); }, {}});
            cs.push_back({"blk" + std::to_string(B) + "_vec1_u32_tb64", alg,
                          [=] { k_blk_i64<32, 64, 1><<<g1, 64>>>(slab, R, bs, bstride, P, sum, dec, 1000.f); }, {}});
        }
        run_cases(cs, 5, 1);
    } else if (what == "lat") {  // small-copy latency: 2-D vs per-block 1-D vs one 1-D (host wall clock)
        const int64_t B = 65536, nb = 4;
        const size_t bytes = (size_t)nb * B * 4;
        void* h;
        CK(hipHostMalloc(&h, bytes, 0));
        memset(h, 1, bytes);
        void* hp = malloc(bytes);
        memset(hp, 1, bytes);
        float* d;
        CK(hipMalloc(&d, (size_t)16 * nb * B * 4));
        float* lin;
        CK(hipMalloc(&lin, bytes));
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        auto wall = [&](const char* name, std::function<void()> f) {
            for (int k = 0; k < 3; ++k) { f(); CK(hipStreamSynchronize(s)); }
            std::vector<double> t;
            for (int k = 0; k < 20; ++k) {
                auto t0 = std::chrono::steady_clock::now();
                f();
                auto t1 = std::chrono::steady_clock::now();
                CK(hipStreamSynchronize(s));
                auto t2 = std::chrono::steady_clock::now();
                t.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
                t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            }
            std::vector<double> tot, call;
            for (size_t k = 0; k < t.size(); k += 2) { tot.push_back(t[k]); call.push_back(t[k + 1]); }
            std::sort(tot.begin(), tot.end());
            std::sort(call.begin(), call.end());
            printf("{\"case\": \"%s\", \"us_total_median\": %.1f, \"us_call_median\": %.1f}\n", name, tot[tot.size() / 2],
                   call[call.size() / 2]);
            fflush(stdout);
        };
        wall("1d_pinned_1MB", [&] { CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s)); });
        wall("2d_pinned_4x256K", [&] {
            CK(hipMemcpy2DAsync(d, (size_t)16 * B * 4, h, B * 4, B * 4, nb, hipMemcpyHostToDevice, s));
        });
        wall("4x1d_pinned_256K", [&] {
            for (int j = 0; j < nb; ++j)
                CK(hipMemcpyAsync(d + (size_t)j * 16 * B, (char*)h + (size_t)j * B * 4, B * 4, hipMemcpyHostToDevice, s));
        });
        wall("1d_pinned+2d_d2d", [&] {
            CK(hipMemcpyAsync(lin, h, bytes, hipMemcpyHostToDevice, s));
            CK(hipMemcpy2DAsync(d, (size_t)16 * B * 4, lin, B * 4, B * 4, nb, hipMemcpyDeviceToDevice, s));
        });
        wall("2d_pinned_4x256K_stream0", [&] {
            CK(hipMemcpy2DAsync(d, (size_t)16 * B * 4, h, B * 4, B * 4, nb, hipMemcpyHostToDevice, s));
        });
    } else {  // h2d
        const size_t bytes = (size_t)P * 4;
        const int R = 64;
        void* h;
        CK(hipHostMalloc(&h, bytes, 0));
        memset(h, 1, bytes);
        float* d;
        const int64_t Pmax = (P + 65535) / 65536 * 65536;
        CK(hipMalloc(&d, (size_t)R * Pmax * 4));
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        auto timeit = [&](const char* name, std::function<void(int)> f) {
            f(0);
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(a, s));
            for (int k = 0; k < 16; ++k) f(k % R);
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("{\"case\": \"%s\", \"GBps\": %.2f}\n", name, 16.0 * bytes / (ms * 1e-3) / 1e9);
            fflush(stdout);
        };
        timeit("h2d_1d", [&](int k) { CK(hipMemcpyAsync(d + (size_t)k * Pmax, h, bytes, hipMemcpyHostToDevice, s)); });
        for (int64_t B : {1024, 4096, 16384, 65536, 262144}) {
            const int64_t nb = P / B;
            std::string nm = "h2d_2d_B" + std::to_string(B);
            timeit(nm.c_str(), [&](int k) {
                CK(hipMemcpy2DAsync(d + (size_t)k * B, (size_t)R * B * 4, h, B * 4, B * 4, nb, hipMemcpyHostToDevice, s));
            });
        }
    }
    return 0;
}
