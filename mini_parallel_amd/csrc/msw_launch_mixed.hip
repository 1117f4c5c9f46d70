// msw_launch_mixed.hip -- SW kernels, mixed grid (pairs + split waves, even KRP = 2..16).
#include "msw_device.h"
#include "msw_launch.h"

namespace msw {
namespace {
template <int KRP>
hipError_t go(const SwParams& p, bool affine, bool coords, uint32_t blocks, hipStream_t stream) {
    const size_t shm = lds_bytes(p.lds_stride, p.groups);
    if (affine) {
        if (coords) return launch_or_query(sw_mixed_kernel<KRP, true, true>, dim3(blocks), shm, stream, p);
        else return launch_or_query(sw_mixed_kernel<KRP, true, false>, dim3(blocks), shm, stream, p);
    } else {
        if (coords) return launch_or_query(sw_mixed_kernel<KRP, false, true>, dim3(blocks), shm, stream, p);
        else return launch_or_query(sw_mixed_kernel<KRP, false, false>, dim3(blocks), shm, stream, p);
    }
}
}  // namespace

hipError_t launch_mixed(const SwParams& p, bool affine, bool coords, int krp, uint32_t blocks, hipStream_t stream) {
    switch (krp) {
        case 2: return go<2>(p, affine, coords, blocks, stream);
        case 4: return go<4>(p, affine, coords, blocks, stream);
        case 6: return go<6>(p, affine, coords, blocks, stream);
        case 8: return go<8>(p, affine, coords, blocks, stream);
        case 10: return go<10>(p, affine, coords, blocks, stream);
        case 12: return go<12>(p, affine, coords, blocks, stream);
        case 14: return go<14>(p, affine, coords, blocks, stream);
        case 16: return go<16>(p, affine, coords, blocks, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace msw
