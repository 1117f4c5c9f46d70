// msw_launch_split.hip -- SW kernels, split layout (KR = 1..8, every scoring kind).
#include "msw_device.h"
#include "msw_launch.h"

namespace msw {
namespace {
template <int KR>
hipError_t go(const SwParams& p, bool affine, bool coords, hipStream_t stream) {
    const uint32_t per_wave = pairs_per_wave(true, p.groups);
    const dim3 grid((p.n_slots + per_wave - 1) / per_wave);
    const size_t shm = lds_bytes(p.lds_stride, p.groups);
    if (affine) {
        if (coords) return launch_or_query(sw_kernel<KR, true, true, true>, grid, shm, stream, p);
        else return launch_or_query(sw_kernel<KR, true, false, true>, grid, shm, stream, p);
    } else {
        if (coords) return launch_or_query(sw_kernel<KR, false, true, true>, grid, shm, stream, p);
        else return launch_or_query(sw_kernel<KR, false, false, true>, grid, shm, stream, p);
    }
}
}  // namespace

hipError_t launch_split(const SwParams& p, bool affine, bool coords, int kr, hipStream_t stream) {
    switch (kr) {
        case 1: return go<1>(p, affine, coords, stream);
        case 2: return go<2>(p, affine, coords, stream);
        case 3: return go<3>(p, affine, coords, stream);
        case 4: return go<4>(p, affine, coords, stream);
        case 5: return go<5>(p, affine, coords, stream);
        case 6: return go<6>(p, affine, coords, stream);
        case 7: return go<7>(p, affine, coords, stream);
        case 8: return go<8>(p, affine, coords, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace msw
