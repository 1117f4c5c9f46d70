// msw_launch_multi_lin.hip -- length-bucketed SW grid, linear gap.
#include "msw_device.h"
#include "msw_launch.h"

namespace msw {

hipError_t launch_multi_lin(const SwParams& p, const MultiTable& t, bool coords, uint32_t grid, size_t shm,
                            hipStream_t stream) {
    if (coords) return launch_or_query(sw_multi_kernel<false, true>, dim3(grid), shm, stream, p, t);
    else return launch_or_query(sw_multi_kernel<false, false>, dim3(grid), shm, stream, p, t);
}

}  // namespace msw
