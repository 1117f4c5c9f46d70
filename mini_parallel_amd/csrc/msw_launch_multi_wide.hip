// msw_launch_multi_wide.hip -- length-bucketed SW grid over the KR 17..24
// buckets (reads of 257..384 bases), linear and affine.
#include "msw_device.h"
#include "msw_launch.h"

namespace msw {

hipError_t launch_multi_wide(const SwParams& p, const MultiTable& t, bool affine, bool coords, uint32_t grid,
                             size_t shm, hipStream_t stream) {
    if (affine) {
        if (coords) return launch_or_query(sw_multi_kernel<true, true, true>, dim3(grid), shm, stream, p, t);
        else return launch_or_query(sw_multi_kernel<true, false, true>, dim3(grid), shm, stream, p, t);
    } else {
        if (coords) return launch_or_query(sw_multi_kernel<false, true, true>, dim3(grid), shm, stream, p, t);
        else return launch_or_query(sw_multi_kernel<false, false, true>, dim3(grid), shm, stream, p, t);
    }
}

}  // namespace msw
