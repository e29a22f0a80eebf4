// The report-time close's device pipeline in isolation: a FINAL fold pass over 72 rows of a
// ResNet-18-sized shard as 12 ranges of 4 MiB of output on one stream, and the 47 MB result's D2H
// in 8 MiB pieces on a copy stream, each piece behind the two ranges that wrote it -- the shape of
// pgh_slots.cpp's slot fold + stage_d2h_pieces.  A kernel + copy trace of the real close
// (profiles/r05d/) showed (a) 17-22 us of idle between consecutive ranges, each followed by two
// timing events and a mark, and (b) ranges running beside a D2H piece that HIP executed as a blit
// kernel ending only when that blit ended (183-190 us instead of 48): the range's end-of-kernel
// system-scope release waits behind the blit's writes to host memory.  This measures what the
// event flags and the place of the cross-stream wait do to the span (first launch -> last byte on
// the host), and checks every piece's bytes against a copy taken after a full device sync.
//
// Variants (one letter each): timing events around every range: n = none, d = default flags,
//   f = hipEventDisableSystemFence, v = hipEventReleaseToDevice; marks: d / f / v; wait: g = the
//   copy stream waits on the marks (GPU side), h = the host waits for each mark, then issues;
//   optional 4th letter, the last report's 47 MB H2D into row 0 issued just before the close
//   (the close's trigger comes while it is in flight): w = the fold waits for all of it,
//   c = it is issued as 12 range-aligned chunks with an event each and fold range k waits only
//   for chunk k, a = the same with the chunks alternating over two streams (the D2H pieces on
//   their own stream either way).  Also reported: the 47 MB H2D alone as one copy, as 12 or 6
//   chunks on one stream and as 12 chunks alternating over two streams.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/exp_close_pipeline.hip -o tools/_exp_close_pipeline
// Run:   tools/_exp_close_pipeline [reps] [variant ...]   -> one JSON line
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                           \
        }                                                                                           \
    } while (0)

constexpr int ROWS = 72;
constexpr size_t P = 11689512;              // ResNet-18 params
constexpr size_t RANGE = (4u << 20) / 4;    // floats of output per range
constexpr size_t PIECE = 8u << 20;          // D2H bytes per piece

// out[i] = ckpt[i] - (sum_r rows[r][i]) / ROWS over [lo, hi): the FINAL pass's arithmetic shape.
__global__ __launch_bounds__(256) void k_range(const float4* __restrict__ rows, const float4* __restrict__ ckpt,
                                               float4* __restrict__ out, size_t lo4, size_t hi4, size_t ld4) {
    for (size_t i = lo4 + (size_t)blockIdx.x * 256 + threadIdx.x; i < hi4; i += (size_t)gridDim.x * 256) {
        float4 s = rows[i];
        for (int r = 1; r < ROWS; ++r) {
            const float4 v = rows[(size_t)r * ld4 + i];
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        const float4 c = ckpt[i];
        const float inv = 1.0f / ROWS;
        out[i] = make_float4(c.x - s.x * inv, c.y - s.y * inv, c.z - s.z * inv, c.w - s.w * inv);
    }
}

__global__ void k_perturb(float4* ckpt, size_t n4, float d) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n4) ckpt[i].x += d;
}

static unsigned flags_of(char c) {
    switch (c) {
    case 'f': return hipEventDisableTiming | hipEventDisableSystemFence;
    case 'v': return hipEventDisableTiming | hipEventReleaseToDevice;
    default: return hipEventDisableTiming;
    }
}
static unsigned timing_flags_of(char c) {
    switch (c) {
    case 'f': return hipEventDisableSystemFence;
    case 'v': return hipEventReleaseToDevice;
    default: return hipEventDefault;
    }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 12;
    std::vector<std::string> variants;
    for (int i = 2; i < argc; ++i) variants.push_back(argv[i]);
    if (variants.empty()) variants = {"ddg", "ndg", "ffg", "vvg", "nfg", "nvg", "ndh", "nfh"};
    const size_t ld = (P + 63) / 64 * 64, ld4 = ld / 4;
    float *rows = nullptr, *ckpt = nullptr, *out = nullptr;
    CK(hipMalloc((void**)&rows, ROWS * ld * 4));
    CK(hipMalloc((void**)&ckpt, ld * 4));
    CK(hipMalloc((void**)&out, ld * 4));
    {
        std::vector<float> h(ld);
        for (size_t i = 0; i < ld; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
        for (int r = 0; r < ROWS; ++r) CK(hipMemcpy(rows + (size_t)r * ld, h.data(), ld * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(ckpt, h.data(), ld * 4, hipMemcpyHostToDevice));
    }
    uint8_t *host = nullptr, *want = nullptr, *report = nullptr;
    const size_t bytes = P * 4;
    CK(hipHostMalloc((void**)&host, bytes, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&want, bytes, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&report, bytes, hipHostMallocDefault));
    {
        std::vector<float> h(P);
        for (size_t i = 0; i < P; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
        std::memcpy(report, h.data(), bytes);
    }
    hipStream_t sf, sc, sh, sh2;
    CK(hipStreamCreateWithFlags(&sf, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sh, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sh2, hipStreamNonBlocking));
    std::map<std::string, std::vector<double>> h2d_ms;
    for (int rep = 0; rep < 11; ++rep) {
        for (const char* how : {"whole", "chunks12", "chunks6", "chunks12_2streams"}) {
            const std::string hw = how;
            const size_t chunk = hw == "whole" ? bytes : hw == "chunks6" ? (8u << 20) : (4u << 20);
            CK(hipDeviceSynchronize());
            const auto a = std::chrono::steady_clock::now();
            for (size_t off = 0, k = 0; off < bytes; off += chunk, ++k)
                CK(hipMemcpyAsync((uint8_t*)rows + off, report + off, std::min(chunk, bytes - off),
                                  hipMemcpyHostToDevice, (hw == "chunks12_2streams" && (k & 1)) ? sh2 : sh));
            CK(hipStreamSynchronize(sh));
            CK(hipStreamSynchronize(sh2));
            if (rep) h2d_ms[hw].push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count());
        }
    }
    const int K = (int)((P + RANGE - 1) / RANGE);
    const int NP = (int)((bytes + PIECE - 1) / PIECE);
    std::map<std::string, std::vector<double>> span;
    std::map<std::string, int> bad;
    for (int rep = 0; rep < reps + 1; ++rep) {
        for (const std::string& v : variants) {
            // a new result every run (so a stale read shows): nudge the checkpoint
            k_perturb<<<(ld4 + 255) / 256, 256, 0, sf>>>((float4*)ckpt, ld4, 1.0f);
            CK(hipStreamSynchronize(sf));
            std::vector<hipEvent_t> ta, tb, mk(K);
            for (int k = 0; k < K; ++k) {
                CK(hipEventCreateWithFlags(&mk[k], flags_of(v[1])));
                if (v[0] != 'n') {
                    hipEvent_t a, b;
                    CK(hipEventCreateWithFlags(&a, timing_flags_of(v[0])));
                    CK(hipEventCreateWithFlags(&b, timing_flags_of(v[0])));
                    ta.push_back(a);
                    tb.push_back(b);
                }
            }
            hipEvent_t done;
            CK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
            std::vector<hipEvent_t> hv(K);
            for (auto& e : hv) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            std::memset(host, 0, bytes);
            const char h2d = v.size() > 3 ? v[3] : 'x';
            const auto t0 = std::chrono::steady_clock::now();
            if (h2d == 'w') {
                CK(hipMemcpyAsync(rows, report, bytes, hipMemcpyHostToDevice, sh));
                CK(hipEventRecord(hv[0], sh));
                CK(hipStreamWaitEvent(sf, hv[0], 0));
            } else if (h2d == 'c' || h2d == 'a') {
                for (int k = 0; k < K; ++k) {
                    const size_t lo = k * RANGE, hi = std::min(P, (k + 1) * RANGE);
                    hipStream_t st = (h2d == 'a' && (k & 1)) ? sh2 : sh;
                    CK(hipMemcpyAsync(rows + lo, report + lo * 4, (hi - lo) * 4, hipMemcpyHostToDevice, st));
                    CK(hipEventRecord(hv[k], st));
                }
            }
            for (int k = 0; k < K; ++k) {
                const size_t lo = k * RANGE, hi = std::min(P, (k + 1) * RANGE);
                if (h2d == 'c' || h2d == 'a') CK(hipStreamWaitEvent(sf, hv[k], 0));
                if (v[0] != 'n') CK(hipEventRecord(ta[k], sf));
                k_range<<<1024, 256, 0, sf>>>((const float4*)rows, (const float4*)ckpt, (float4*)out, lo / 4,
                                              (hi + 3) / 4, ld4);
                if (v[0] != 'n') CK(hipEventRecord(tb[k], sf));
                CK(hipEventRecord(mk[k], sf));
            }
            for (int p = 0; p < NP; ++p) {
                const size_t off = p * PIECE, len = std::min(PIECE, bytes - off);
                const int last = (int)std::min<size_t>(K - 1, (off + len - 1) / 4 / RANGE);
                if (v[2] == 'h') {
                    CK(hipEventSynchronize(mk[last]));
                } else {
                    for (int k = (int)(off / 4 / RANGE); k <= last; ++k) CK(hipStreamWaitEvent(sc, mk[k], 0));
                }
                CK(hipMemcpyAsync(host + off, (const uint8_t*)out + off, len, hipMemcpyDeviceToHost, sc));
            }
            CK(hipEventRecord(done, sc));
            CK(hipEventSynchronize(done));
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(want, out, bytes, hipMemcpyDeviceToHost));
            if (std::memcmp(host, want, bytes) != 0) ++bad[v];
            if (rep) span[v].push_back(ms);
            for (auto e : mk) CK(hipEventDestroy(e));
            for (auto e : hv) CK(hipEventDestroy(e));
            for (auto e : ta) CK(hipEventDestroy(e));
            for (auto e : tb) CK(hipEventDestroy(e));
            CK(hipEventDestroy(done));
        }
    }
    std::printf("{\"tool\": \"tools/exp_close_pipeline.hip\", \"rows\": %d, \"ranges\": %d, \"pieces\": %d, \"reps\": %d, "
                "\"variants\": {", ROWS, K, NP, reps);
    bool first = true;
    for (auto& kv : span) {
        auto s = kv.second;
        std::sort(s.begin(), s.end());
        std::printf("%s\"%s\": {\"median_ms\": %.4f, \"min_ms\": %.4f, \"max_ms\": %.4f, \"stale_runs\": %d}",
                    first ? "" : ", ", kv.first.c_str(), s[s.size() / 2], s.front(), s.back(), bad[kv.first]);
        first = false;
    }
    std::printf("}, \"h2d_47MB\": {");
    first = true;
    for (auto& kv : h2d_ms) {
        auto s2 = kv.second;
        std::sort(s2.begin(), s2.end());
        std::printf("%s\"%s\": {\"median_ms\": %.4f, \"GBps\": %.1f}", first ? "" : ", ", kv.first.c_str(),
                    s2[s2.size() / 2], bytes / (s2[s2.size() / 2] * 1e6));
        first = false;
    }
    std::printf("}}\n");
    return 0;
}
