// msw_launch_genome_lin.hip -- linear-gap SW kernels, pairs layout (KR = 1..16),
// windows read straight from the HBM-resident genome (GEN instances,
// SwParams::win_src): one-chunk msw_align_reads calls score without a window
// cut launch.  Separate units so they build beside the slab instances.
#include "msw_device.h"
#include "msw_launch.h"

namespace msw {
namespace {
template <int KR>
hipError_t go(const SwParams& p, bool coords, hipStream_t stream) {
    const uint32_t per_wave = pairs_per_wave(false, p.groups);
    const dim3 grid((p.n_slots + per_wave - 1) / per_wave);
    const size_t shm = lds_bytes(p.lds_stride, p.groups);
    if (coords) return launch_or_query(sw_kernel<KR, false, true, false, true>, grid, shm, stream, p);
    else return launch_or_query(sw_kernel<KR, false, false, false, true>, grid, shm, stream, p);
}
}  // namespace

hipError_t launch_genome_lin(const SwParams& p, bool coords, int kr, hipStream_t stream) {
    switch (kr) {
        case 1: return go<1>(p, coords, stream);
        case 2: return go<2>(p, coords, stream);
        case 3: return go<3>(p, coords, stream);
        case 4: return go<4>(p, coords, stream);
        case 5: return go<5>(p, coords, stream);
        case 6: return go<6>(p, coords, stream);
        case 7: return go<7>(p, coords, stream);
        case 8: return go<8>(p, coords, stream);
        case 9: return go<9>(p, coords, stream);
        case 10: return go<10>(p, coords, stream);
        case 11: return go<11>(p, coords, stream);
        case 12: return go<12>(p, coords, stream);
        case 13: return go<13>(p, coords, stream);
        case 14: return go<14>(p, coords, stream);
        case 15: return go<15>(p, coords, stream);
        case 16: return go<16>(p, coords, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace msw
