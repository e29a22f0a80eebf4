// libpygrid_hip: K6 k_copy_to_host (pgh_copy.hip): HBM -> page-locked host memory by a kernel.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace pgh {
// n bytes (a multiple of 4) from 16-byte aligned HBM `src` to 16-byte aligned page-locked `dst`,
// by at most `workgroups` workgroups of 256 lanes on stream s.
hipError_t launch_copy_to_host(void* dst, const void* src, size_t n, int workgroups, hipStream_t s);
}  // namespace pgh
