// msw_launch.h -- per-translation-unit launchers of the SW kernel instance
// set (internal; msw_kernels.hip dispatches to them).  Each msw_launch_*.hip
// instantiates one disjoint slice of sw_kernel / sw_mixed_kernel /
// sw_multi_kernel, so the slices compile in parallel.
#pragma once
#include "msw_kernels.h"

namespace msw {

// Occupancy query mode (kernel_blocks_per_cu, msw_runtime.cpp): while this
// thread's t_occupancy is set, every launch_* below stores the blocks per CU
// of the kernel instance it would launch (its VGPRs and LDS) instead of
// launching.  The query also loads the instance's code object, so a caller
// can take that first-use cost before a timed region (msw_ctx_prepare).
extern thread_local int* t_occupancy;

template <typename... Args>
inline hipError_t launch_or_query(void (*kernel)(Args...), dim3 grid, size_t shm, hipStream_t stream, Args... args) {
    if (t_occupancy) return hipOccupancyMaxActiveBlocksPerMultiprocessor(t_occupancy, kernel, 64, shm);
    hipLaunchKernelGGL(kernel, grid, dim3(64), shm, stream, args...);
    return hipGetLastError();
}

// pairs layout, KR = 1..16 (msw_launch_pairs_lin.hip / msw_launch_pairs_aff.hip)
hipError_t launch_pairs_lin(const SwParams& p, bool coords, int kr, hipStream_t stream);
hipError_t launch_pairs_aff(const SwParams& p, bool coords, int kr, hipStream_t stream);
// pairs layout, KR = 1..16, windows from the resident genome (p.win_src;
// msw_launch_genome_lin.hip / msw_launch_genome_aff.hip)
hipError_t launch_genome_lin(const SwParams& p, bool coords, int kr, hipStream_t stream);
hipError_t launch_genome_aff(const SwParams& p, bool coords, int kr, hipStream_t stream);
// pairs layout, KR = 17..24 (G = 16: reads of 257..384 bases; msw_launch_pairs_wide.hip)
hipError_t launch_pairs_wide(const SwParams& p, bool affine, bool coords, int kr, hipStream_t stream);
// split layout, KR = 1..8 (msw_launch_split.hip)
hipError_t launch_split(const SwParams& p, bool affine, bool coords, int kr, hipStream_t stream);
// mixed grid, even KRP = 2..16 (msw_launch_mixed.hip)
hipError_t launch_mixed(const SwParams& p, bool affine, bool coords, int krp, uint32_t blocks, hipStream_t stream);
// length-bucketed grid (msw_launch_multi_lin.hip / msw_launch_multi_aff.hip)
hipError_t launch_multi_lin(const SwParams& p, const MultiTable& t, bool coords, uint32_t grid, size_t shm,
                            hipStream_t stream);
hipError_t launch_multi_aff(const SwParams& p, const MultiTable& t, bool coords, uint32_t grid, size_t shm,
                            hipStream_t stream);
// the same over KR 17..24 buckets (msw_launch_multi_wide.hip)
hipError_t launch_multi_wide(const SwParams& p, const MultiTable& t, bool affine, bool coords, uint32_t grid,
                             size_t shm, hipStream_t stream);

}  // namespace msw
