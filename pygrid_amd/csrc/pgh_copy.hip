// libpygrid_hip: K6 k_copy_to_host -- HBM -> page-locked host memory by a kernel, for the
// report-time close's D2H pieces while the last reports' H2D still runs.  The runtime's SDMA
// copies serialise host <-> HBM traffic in both directions on one engine (a D2H queued on another
// stream starts only when the H2D ahead of it has finished; the engines the runtime recommends for
// a pinned D2H run at ~28 GB/s each: tools/exp_d2h_prime.hip, profiles/r06e/), so behind a backlog
// of report copies the close's 47 MB waited for all of it.  Stores from the CUs go out over PCIe
// beside the SDMA engine's reads: the link is full duplex.  Reference: the new checkpoint's bytes of
// cycle_manager.py:293-303.
//
// Layout: n bytes, src 16-byte aligned (a D2H piece starts at a multiple of 8 MiB of the result),
// dst a page-locked cell (8 MiB aligned within its allocation).  A grid-stride loop of 16-byte
// loads (non-temporal: read once) and 16-byte non-temporal stores to the host; the last n % 16
// bytes by one lane, 4 bytes at a time (results are float32 / int64: n is a multiple of 4).  A few
// workgroups suffice -- PCIe, not the CUs, bounds it -- and leave the rest of the chip to the fold.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pgh_copy.h"

namespace pgh {
namespace {

constexpr int COPY_BLOCK = 256;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(COPY_BLOCK) void k_copy_to_host(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                             int64_t n16, const uint32_t* __restrict__ src_tail,
                                                             uint32_t* __restrict__ dst_tail, int tail_words) {
    const int64_t stride = (int64_t)gridDim.x * COPY_BLOCK;
    for (int64_t i = (int64_t)blockIdx.x * COPY_BLOCK + threadIdx.x; i < n16; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
    if (blockIdx.x == 0 && threadIdx.x < (unsigned)tail_words) dst_tail[threadIdx.x] = src_tail[threadIdx.x];
}

}  // namespace

hipError_t launch_copy_to_host(void* dst, const void* src, size_t n, int workgroups, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (!dst || !src || (n & 3) || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15) || workgroups < 1)
        return hipErrorInvalidValue;
    const int64_t n16 = (int64_t)(n / 16);
    const int tail = (int)((n % 16) / 4);
    const int64_t need = (n16 + COPY_BLOCK - 1) / COPY_BLOCK;
    const unsigned g = (unsigned)(need < workgroups ? (need > 0 ? need : 1) : workgroups);
    k_copy_to_host<<<g, COPY_BLOCK, 0, s>>>((const u32x4*)src, (u32x4*)dst, n16,
                                            (const uint32_t*)((const uint8_t*)src + 16 * n16),
                                            (uint32_t*)((uint8_t*)dst + 16 * n16), tail);
    return hipGetLastError();
}

}  // namespace pgh
