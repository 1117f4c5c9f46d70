// msw_launch_pairs_wide.hip -- SW kernels, pairs layout with 16-lane groups and
// KR = 17..24 packed rows per lane: reads of 257..384 bases (MiSeq 2 x 300)
// on the packed 16-bit kernels instead of the i32 long-pair kernel.
#include "msw_device.h"
#include "msw_launch.h"

namespace msw {
namespace {
template <int KR>
hipError_t go(const SwParams& p, bool affine, bool coords, hipStream_t stream) {
    const uint32_t per_wave = pairs_per_wave(false, p.groups);
    const dim3 grid((p.n_slots + per_wave - 1) / per_wave);
    const size_t shm = lds_bytes(p.lds_stride, p.groups);
    if (affine) {
        if (coords) return launch_or_query(sw_kernel<KR, true, true, false>, grid, shm, stream, p);
        else return launch_or_query(sw_kernel<KR, true, false, false>, grid, shm, stream, p);
    } else {
        if (coords) return launch_or_query(sw_kernel<KR, false, true, false>, grid, shm, stream, p);
        else return launch_or_query(sw_kernel<KR, false, false, false>, grid, shm, stream, p);
    }
}
}  // namespace

hipError_t launch_pairs_wide(const SwParams& p, bool affine, bool coords, int kr, hipStream_t stream) {
    switch (kr) {
        case 17: return go<17>(p, affine, coords, stream);
        case 18: return go<18>(p, affine, coords, stream);
        case 19: return go<19>(p, affine, coords, stream);
        case 20: return go<20>(p, affine, coords, stream);
        case 21: return go<21>(p, affine, coords, stream);
        case 22: return go<22>(p, affine, coords, stream);
        case 23: return go<23>(p, affine, coords, stream);
        case 24: return go<24>(p, affine, coords, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace msw
