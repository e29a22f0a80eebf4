// Which first copy on a fresh stream makes the HIP runtime carry that stream's later HBM -> host
// copies on an SDMA engine instead of blit kernels (__amd_rocclr_copyBuffer, which take CUs from the
// fold beside them: profiles/r05d/, r06d/)?  For each priming variant a fresh non-blocking stream
// gets the priming copy (synchronised), then six 8 MiB D2H pieces into page-locked memory while a
// read-bound kernel runs on another stream -- the report-time close's shape.  Run it under
// `rocprofv3 --kernel-trace --memory-copy-trace`: per variant, the pieces show up either as
// DEVICE_TO_HOST memory copies (SDMA) or as copyBuffer kernels (blit).  The variant tag is the
// grid size of a marker kernel launched before its pieces (g = 64 * (variant + 1)).
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/exp_d2h_prime.hip -o tools/_exp_d2h_prime
// Run:   tools/_exp_d2h_prime
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                            \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(2); } \
    } while (0)

__global__ __launch_bounds__(256) void k_read(const float4* __restrict__ a, size_t n4, float* out) {
    float s = 0.f;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;  // never true: keeps the loads
}

__global__ void k_marker(float* out) {
    if (threadIdx.x == 1000) out[0] = 1.f;  // never true
}

int main() {
    const size_t piece = 8u << 20, pieces = 6, big = (size_t)4 << 30;  // 4 GiB read-bound load
    float* d_big = nullptr;
    float* d_src = nullptr;
    float* d_small = nullptr;
    CK(hipMalloc(&d_big, big));
    CK(hipMemset(d_big, 0, big));
    CK(hipMalloc(&d_src, piece * pieces));
    CK(hipMemset(d_src, 1, piece * pieces));
    CK(hipMalloc(&d_small, 16 << 20));
    uint8_t* h_cells = nullptr;
    uint8_t* h_prime = nullptr;
    CK(hipHostMalloc((void**)&h_cells, piece * pieces, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&h_prime, 16 << 20, hipHostMallocDefault));
    std::memset(h_prime, 0, 16 << 20);
    hipStream_t load;
    CK(hipStreamCreateWithFlags(&load, hipStreamNonBlocking));
    // variant: 0 no priming, 1 64 B H2D, 2 4 KiB H2D, 3 2 MiB H2D, 4 8 MiB H2D, 5 8 MiB D2H,
    //          6 2 MiB H2D + 8 MiB D2H, 7 a blocking stream (default flags), 8 2 MiB H2D and an
    //          H2D stream busy beside the pieces (the last reports' copies)
    const size_t prime_bytes[] = {0, 64, 4096, 2u << 20, 8u << 20, 0, 2u << 20, 0, 2u << 20};
    const int n_var = 9;
    hipStream_t h2ds;
    CK(hipStreamCreateWithFlags(&h2ds, hipStreamNonBlocking));
    CK(hipMemcpyAsync(d_small, h_prime, 2u << 20, hipMemcpyHostToDevice, h2ds));
    CK(hipStreamSynchronize(h2ds));
    for (int v = 0; v < n_var; ++v) {
        hipStream_t s;
        if (v == 7) CK(hipStreamCreate(&s));
        else CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        if (prime_bytes[v]) CK(hipMemcpyAsync(d_small, h_prime, prime_bytes[v], hipMemcpyHostToDevice, s));
        if (v == 5 || v == 6) CK(hipMemcpyAsync(h_prime, d_small, 8u << 20, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        k_marker<<<64 * (v + 1), 64, 0, load>>>(d_small);
        k_read<<<4096, 256, 0, load>>>((const float4*)d_big, big / 16, d_small);
        if (v == 8)
            for (int j = 0; j < 6; ++j) CK(hipMemcpyAsync(d_small, h_prime, 8u << 20, hipMemcpyHostToDevice, h2ds));
        for (size_t j = 0; j < pieces; ++j)
            CK(hipMemcpyAsync(h_cells + j * piece, (const uint8_t*)d_src + j * piece, piece, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        CK(hipStreamSynchronize(load));
        CK(hipStreamSynchronize(h2ds));
        CK(hipStreamDestroy(s));
    }
    std::printf("{\"variants\": %d, \"pieces\": %zu, \"piece_bytes\": %zu}\n", n_var, pieces, piece);
    CK(hipHostFree(h_cells));
    CK(hipHostFree(h_prime));
    CK(hipFree(d_big));
    CK(hipFree(d_src));
    CK(hipFree(d_small));
    return 0;
}
