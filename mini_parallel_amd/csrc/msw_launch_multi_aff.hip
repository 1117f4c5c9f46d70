// msw_launch_multi_aff.hip -- length-bucketed SW grid, affine gap.
#include "msw_device.h"
#include "msw_launch.h"

namespace msw {

hipError_t launch_multi_aff(const SwParams& p, const MultiTable& t, bool coords, uint32_t grid, size_t shm,
                            hipStream_t stream) {
    if (coords) return launch_or_query(sw_multi_kernel<true, true>, dim3(grid), shm, stream, p, t);
    else return launch_or_query(sw_multi_kernel<true, false>, dim3(grid), shm, stream, p, t);
}

}  // namespace msw
