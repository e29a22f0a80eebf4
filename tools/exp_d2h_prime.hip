// Which first copy on a fresh stream makes the HIP runtime carry that stream's later HBM -> host
// copies on an SDMA engine instead of blit kernels (__amd_rocclr_copyBuffer, which take CUs from the
// fold beside them: profiles/r05d/, r06d/)?  For each priming variant a fresh non-blocking stream
// gets the priming copy (synchronised), then six 8 MiB D2H pieces into page-locked memory while a
// read-bound kernel runs on another stream -- the report-time close's shape.  Run it under
// `rocprofv3 --kernel-trace --memory-copy-trace`: per variant, the pieces show up either as
// DEVICE_TO_HOST memory copies (SDMA) or as copyBuffer kernels (blit).  The variant tag is the
// grid size of a marker kernel launched before its pieces (g = 64 * (variant + 1)).
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/exp_d2h_prime.hip -o tools/_exp_d2h_prime -lhsa-runtime64
// Run:   tools/_exp_d2h_prime
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
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
    // The library's sequence, one difference at a time (variant tags 9..14):
    //  9  cells allocated after the stream, an event recorded after each piece, 64 B H2D priming
    // 10  as 9, the pieces issued from another host thread
    // 11  as 9, each piece issued only once the host sees an event on the fold's stream complete
    // 12  as 9, the cells allocated hipHostMallocNumaUser
    // 13  as 9 without the priming copy
    // 14  as 11, the fold split in ranges with an event after each (the FINAL pass's marks)
    std::vector<hipEvent_t> evs(pieces), marks(pieces);
    for (auto& e : evs) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : marks) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (int v = 9; v <= 14; ++v) {
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        uint8_t* cells = nullptr;
        CK(hipHostMalloc((void**)&cells, piece * pieces, v == 12 ? hipHostMallocNumaUser : hipHostMallocDefault));
        if (v != 13) {
            CK(hipMemcpyAsync(d_small, h_prime, 64, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
        }
        k_marker<<<64 * (v + 1), 64, 0, load>>>(d_small);
        if (v == 14) {
            for (size_t j = 0; j < pieces; ++j) {
                k_read<<<4096, 256, 0, load>>>((const float4*)d_big + j * (big / 16 / pieces), big / 16 / pieces, d_small);
                CK(hipEventRecord(marks[j], load));
            }
        } else {
            k_read<<<4096, 256, 0, load>>>((const float4*)d_big, big / 16, d_small);
            for (size_t j = 0; j < pieces; ++j) CK(hipEventRecord(marks[j], load));
        }
        auto issue = [&] {
            for (size_t j = 0; j < pieces; ++j) {
                if (v == 11 || v == 14)
                    while (hipEventQuery(marks[j]) == hipErrorNotReady) std::this_thread::yield();
                CK(hipMemcpyAsync(cells + j * piece, (const uint8_t*)d_src + j * piece, piece, hipMemcpyDeviceToHost, s));
                CK(hipEventRecord(evs[j], s));
            }
            for (auto& e : evs) CK(hipEventSynchronize(e));
        };
        if (v == 10) std::thread(issue).join();
        else issue();
        CK(hipStreamSynchronize(load));
        CK(hipStreamDestroy(s));
        CK(hipHostFree(cells));
    }
    // 15: the last reports' H2D on a HIP stream and the six D2H pieces as HSA copies pinned to one SDMA
    //     engine that hsa_amd_memory_copy_engine_status reports free (the highest), completion by
    //     HSA signals -- do the two directions overlap (PCIe full duplex) when they are on two engines?
    // 16: the same with the engine the runtime recommends (hsa_amd_memory_get_preferred_copy_engine)
    struct Agents { hsa_agent_t gpu{}, cpu{}; int gpus = 0; } ag;
    if (hsa_init() != HSA_STATUS_SUCCESS) { std::fprintf(stderr, "hsa_init failed\n"); return 2; }
    hsa_iterate_agents([](hsa_agent_t a, void* p) -> hsa_status_t {
        auto* g = (Agents*)p;
        hsa_device_type_t t;
        hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
        if (t == HSA_DEVICE_TYPE_GPU && g->gpus++ == 0) g->gpu = a;
        if (t == HSA_DEVICE_TYPE_CPU && g->cpu.handle == 0) g->cpu = a;
        return HSA_STATUS_SUCCESS;
    }, &ag);
    uint32_t free_mask = 0, pref_mask = 0;
    hsa_status_t st1 = hsa_amd_memory_copy_engine_status(ag.cpu, ag.gpu, &free_mask);
    hsa_status_t st2 = hsa_amd_memory_get_preferred_copy_engine(ag.cpu, ag.gpu, &pref_mask);
    std::printf("{\"d2h_free_engines\": \"0x%x\", \"st\": %d, \"d2h_preferred\": \"0x%x\", \"st2\": %d}\n", free_mask,
                (int)st1, pref_mask, (int)st2);
    uint32_t h_free = 0;
    hsa_amd_memory_copy_engine_status(ag.gpu, ag.cpu, &h_free);
    std::printf("{\"h2d_free_engines\": \"0x%x\"}\n", h_free);
    std::vector<hsa_signal_t> sig(pieces);
    for (auto& x : sig) hsa_signal_create(1, 0, nullptr, &x);
    // 17: the pieces alternate over the recommended engines (two in flight), beside the H2D
    // 18: as 17 without the H2D (the D2H alone)
    for (int v = 15; v <= 18; ++v) {
        uint32_t mask = v == 15 ? free_mask : (pref_mask ? pref_mask : free_mask);
        if (!mask) { std::printf("{\"variant\": %d, \"skipped\": \"no engine\"}\n", v); continue; }
        int bit = 31;
        while (bit >= 0 && !(mask & (1u << bit))) --bit;
        if (v >= 16) { bit = 0; while (bit < 32 && !(mask & (1u << bit))) ++bit; }
        int bit2 = bit + 1;
        while (v >= 17 && bit2 < 32 && !(mask & (1u << bit2))) ++bit2;
        if (bit2 >= 32) bit2 = bit;
        k_marker<<<64 * (v + 1), 64, 0, load>>>(d_small);
        k_read<<<4096, 256, 0, load>>>((const float4*)d_big, big / 16, d_small);
        if (v != 18)
            for (int j = 0; j < 6; ++j) CK(hipMemcpyAsync(d_small, h_prime, 8u << 20, hipMemcpyHostToDevice, h2ds));
        for (size_t j = 0; j < pieces; ++j) {
            const int b = (v >= 17 && (j & 1)) ? bit2 : bit;
            hsa_signal_store_relaxed(sig[j], 1);
            hsa_status_t e = hsa_amd_memory_async_copy_on_engine(h_cells + j * piece, ag.cpu, (const uint8_t*)d_src + j * piece,
                                                                 ag.gpu, piece, 0, nullptr, sig[j],
                                                                 (hsa_amd_sdma_engine_id_t)(1u << b), true);
            if (e != HSA_STATUS_SUCCESS) { std::printf("{\"variant\": %d, \"copy_on_engine\": %d}\n", v, (int)e); return 3; }
        }
        for (auto& x : sig) hsa_signal_wait_scacquire(x, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
        CK(hipStreamSynchronize(h2ds));
        CK(hipStreamSynchronize(load));
        std::printf("{\"variant\": %d, \"engine_bit\": %d}\n", v, bit);
    }
    for (auto& x : sig) hsa_signal_destroy(x);
    std::printf("{\"variants\": %d, \"pieces\": %zu, \"piece_bytes\": %zu}\n", n_var + 8, pieces, piece);
    CK(hipHostFree(h_cells));
    CK(hipHostFree(h_prime));
    CK(hipFree(d_big));
    CK(hipFree(d_src));
    CK(hipFree(d_small));
    return 0;
}
