// K4 alone: a ResNet-18-sized payload of packed int64 varints (P values, uniform random: ~9.5 bytes
// each, like secagg shares) resident in HBM, decoded REPS times back to back by
// pgh::launch_varint_decode (the library's own launcher, linked from libpygrid_hip.so), timed with
// HIP events, the output checked against the host's values.  No PCIe, no other stream beside it:
// the kernel's own rate.
//   hipcc -O2 -std=c++17 -Ipygrid_amd/csrc tools/exp_varint.cpp -Lpygrid_amd -lpygrid_hip \
//         -Wl,-rpath,'$ORIGIN/../pygrid_amd' -o tools/_exp_varint && tools/_exp_varint [P] [reps] [kind]
// kind: 0 uniform int64 (default), 1 mixed lengths 1..10 bytes, 2 one-byte values.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "pgh_kernels.h"

#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

int main(int argc, char** argv) {
    const int64_t P = argc > 1 ? std::atoll(argv[1]) : 11689512;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 50;
    const int kind = argc > 3 ? std::atoi(argv[3]) : 0;
    std::mt19937_64 rng(7);
    std::vector<int64_t> vals((size_t)P);
    for (auto& v : vals) {
        const uint64_t r = rng();
        if (kind == 0) v = (int64_t)r;
        else if (kind == 1) v = (int64_t)(r >> (rng() % 64));
        else v = (int64_t)(r & 127);
    }
    std::vector<uint8_t> bytes;
    bytes.reserve((size_t)P * 10 + 64);
    for (int64_t v : vals) {
        uint64_t u = (uint64_t)v;
        while (u >= 0x80) { bytes.push_back((uint8_t)(u | 0x80)); u >>= 7; }
        bytes.push_back((uint8_t)u);
    }
    const size_t nb = bytes.size();
    bytes.resize(nb + 64, 0);
    uint8_t* d_bytes = nullptr;
    int64_t* d_row = nullptr;
    HC(hipMalloc(&d_bytes, bytes.size()));
    HC(hipMalloc(&d_row, (size_t)P * 8));
    HC(hipMemcpy(d_bytes, bytes.data(), bytes.size(), hipMemcpyHostToDevice));
    const pgh::SlabMap m = pgh::single_block(P);
    hipStream_t s;
    HC(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    HC(hipEventCreate(&e0));
    HC(hipEventCreate(&e1));
    std::printf("P=%lld, %zu varint bytes (%.2f per value), kind %d, %d launches\n", (long long)P, nb,
                (double)nb / (double)P, kind, reps);
    std::vector<pgh::VChunk> tab;  // the host's cut (pgh_ingest.cpp plan_share_msg): VARINT_CHUNK bytes
    int64_t first = 0;
    for (size_t a = 0; a < nb; a += pgh::VARINT_CHUNK) {
        const size_t len = std::min(nb - a, (size_t)pgh::VARINT_CHUNK);
        tab.push_back(pgh::VChunk{(int64_t)a, 0, first, (int32_t)len, 0});
        for (size_t i = a; i < a + len; ++i) first += bytes[i] < 0x80;
    }
    pgh::VChunk* d_tab = nullptr;
    HC(hipMalloc(&d_tab, tab.size() * sizeof(pgh::VChunk)));
    HC(hipMemcpy(d_tab, tab.data(), tab.size() * sizeof(pgh::VChunk), hipMemcpyHostToDevice));
    HC(hipMemset(d_row, 0xAB, (size_t)P * 8));
    HC(pgh::launch_varint_decode(d_bytes, d_tab, (int)tab.size(), d_row, m, 0, P, s));  // warm-up
    HC(hipStreamSynchronize(s));
    HC(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) HC(pgh::launch_varint_decode(d_bytes, d_tab, (int)tab.size(), d_row, m, 0, P, s));
    HC(hipEventRecord(e1, s));
    HC(hipEventSynchronize(e1));
    float ms = 0.f;
    HC(hipEventElapsedTime(&ms, e0, e1));
    std::vector<int64_t> got((size_t)P);
    HC(hipMemcpy(got.data(), d_row, (size_t)P * 8, hipMemcpyDeviceToHost));
    const bool ok = std::memcmp(got.data(), vals.data(), (size_t)P * 8) == 0;
    const double us = 1e3 * ms / reps;
    std::printf("k_varint_decode (%zu chunks) %8.2f us per launch  %6.0f GB/s of varint bytes  %6.0f GB/s HBM "
                "(in + 8 B out)  %s\n", tab.size(), us, nb / us / 1e3, (nb + 8.0 * P) / us / 1e3,
                ok ? "bit-exact" : "MISMATCH");
    HC(hipFree(d_tab));
    if (!ok) return 2;
    return 0;
}
