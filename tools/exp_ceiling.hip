// Read-ceiling experiment (not product code): how fast can MI355X stream 46.8 GB of HBM with
// different access shapes?  Compared against the product fold on the same bytes.
//   chunkC_uU_tbT : each workgroup reads a contiguous C-byte chunk (16 B / lane, U loads in
//                   flight per lane), chunks assigned round-robin to workgroups (grid-stride)
//   fold          : pgh::launch_fedavg, column-blocked slab, auto variant (the product)
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Ipygrid_amd/csrc -Iinclude \
//          tools/exp_ceiling.hip pygrid_amd/csrc/pgh_kernels.hip -o tools/_exp_ceiling
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

template <int U, int TB>
__global__ __launch_bounds__(TB) void k_chunks(const f32x4* x, int64_t n16, int64_t chunk16, float* out) {
    f32x4 acc = {0, 0, 0, 0};
    const int64_t nchunks = (n16 + chunk16 - 1) / chunk16;
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const int64_t base = c * chunk16, end = std::min(n16, base + chunk16);
        int64_t i = base + threadIdx.x;
        for (; i + (U - 1) * TB < end; i += U * TB) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(x + i + u * TB);
#pragma unroll
            for (int u = 0; u < U; ++u) acc += v[u];
        }
        for (; i < end; i += TB) acc += __builtin_nontemporal_load(x + i);
    }
    out[(int64_t)blockIdx.x * TB + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

int main() {
    const int64_t P = 11689512;
    const int N = 1000;
    const int64_t B = 65536, nb = (P + B - 1) / B;
    const size_t bytes = (size_t)N * nb * B * 4;
    float *slab, *acc, *ckpt, *out, *red;
    CK(hipMalloc(&slab, bytes));
    CK(hipMalloc(&acc, nb * B * 4));
    CK(hipMalloc(&ckpt, nb * B * 4));
    CK(hipMalloc(&out, nb * B * 4));
    CK(hipMalloc(&red, 256ull << 20));
    pgh::SlabMap m{B, (int64_t)N * B, 16, B - 1, 0};
    CK(pgh::launch_synth_f32(slab, m, nb * B, N, P, 1, pgh::STREAM_DIFF, 0, 0, pgh::DIFF_SCALE, 0));
    CK(pgh::launch_synth_f32(ckpt, pgh::single_block(nb * B), nb * B, 1, P, 1, pgh::STREAM_CKPT, 0, 0, pgh::CKPT_SCALE, 0));
    CK(hipDeviceSynchronize());
    struct Case { std::string name; double bytes; std::function<void()> f; std::vector<float> ms; };
    std::vector<Case> cs;
    const double alg = 4.0 * N * P + 8.0 * P;
    pgh::FedavgArgs a{};
    a.diffs = slab; a.map = m; a.n_rows = N; a.client0 = 0; a.p = P; a.acc = acc; a.ckpt = ckpt; a.out = out;
    a.divisor = (float)N; a.flags = pgh::FL_FIRST | pgh::FL_FINAL; a.mode = pgh::MODE_MEAN; a.variant = -1;
    cs.push_back({"fold_auto", alg, [a] { CK(pgh::launch_fedavg(a, 0)); }, {}});
    const int64_t n16 = (int64_t)(bytes / 16);
    for (int64_t C : {65536, 262144, 1048576, 4194304})
        for (int g : {2048, 8192, 32768}) {
            const int64_t c16 = C / 16;
            cs.push_back({"chunk" + std::to_string(C >> 10) + "K_u8_tb256_g" + std::to_string(g), (double)bytes,
                          [=] { k_chunks<8, 256><<<g, 256>>>((const f32x4*)slab, n16, c16, red); }, {}});
            cs.push_back({"chunk" + std::to_string(C >> 10) + "K_u16_tb512_g" + std::to_string(g / 2), (double)bytes,
                          [=] { k_chunks<16, 512><<<g / 2, 512>>>((const f32x4*)slab, n16, c16, red); }, {}});
        }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& c : cs) c.f();
    CK(hipDeviceSynchronize());
    for (int round = 0; round < 5; ++round)
        for (auto& c : cs) {
            CK(hipEventRecord(e0, 0));
            c.f();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            c.ms.push_back(ms);
        }
    for (auto& c : cs) {
        std::sort(c.ms.begin(), c.ms.end());
        const float med = c.ms[c.ms.size() / 2];
        printf("{\"case\": \"%s\", \"ms_median\": %.4f, \"GBps\": %.1f}\n", c.name.c_str(), med, c.bytes / (med * 1e-3) / 1e9);
    }
    return 0;
}
