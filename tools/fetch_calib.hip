// FETCH_SIZE calibration for the SW kernels' two load patterns (gfx950).
// MI355X_MICROARCH.md: FETCH_SIZE reports 1/2 of the bytes of 16 B/lane
// streaming reads; other widths are uncalibrated.  The SW kernels read
// windows with 16 B/lane loads and reads with the byte pattern of
// load_read_bytes (lane lg of a G-lane group loads bytes [lg*KR, lg*KR+KR) of
// two rows).  Both kernels below read the SAME buffer (rows x stride bytes,
// every byte of [0, G*KR) of each row once); run each under
//   rocprofv3 --pmc FETCH_SIZE -- ./tools/fetch_calib MODE STRIDE KR G
// and compare: FETCH(bytes) / FETCH(vec16) is how FETCH counts the byte
// pattern relative to the calibrated 16 B loads (profiles/r02/fetch_calib.txt).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

__global__ void vec16(const uint4* __restrict__ p, uint64_t chunks, uint32_t* out) {
    uint32_t s = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < chunks; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        s ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// one 64-lane block = 64/G groups x 2 rows, like sw_kernel's pairs layout
__global__ void bytes_sw(const uint8_t* __restrict__ p, uint32_t stride, uint32_t rows, int KR, int G,
                         uint32_t* out) {
    const int lane = threadIdx.x, groups = 64 / G, g = lane / G, lg = lane - g * G;
    uint32_t s = 0;
    if (g < groups) {
        const uint32_t ra = blockIdx.x * 2 * groups + 2 * g, rb = ra + 1;
        const uint8_t* a = p + (uint64_t)min(ra, rows - 1) * stride;
        const uint8_t* b = p + (uint64_t)min(rb, rows - 1) * stride;
        for (int r = 0; r < KR; ++r) {
            const int i = min(lg * KR + r, (int)stride - 1);
            s += a[i] + b[i];
        }
    }
    out[blockIdx.x * 64 + lane] = s;
}

int main(int argc, char** argv) {
    const char* mode = argc > 1 ? argv[1] : "vec16";
    const uint32_t stride = argc > 2 ? atoi(argv[2]) : 160;
    const int KR = argc > 3 ? atoi(argv[3]) : 13, G = argc > 4 ? atoi(argv[4]) : 12;
    const uint32_t rows = 1u << 20;
    uint8_t* p;
    uint32_t* out;
    if (hipMalloc(&p, (size_t)rows * stride) != hipSuccess) return 1;
    if (hipMalloc(&out, (size_t)rows * 64 * 4) != hipSuccess) return 1;
    (void)hipMemset(p, 7, (size_t)rows * stride);
    for (int rep = 0; rep < 3; ++rep) {
        if (mode[0] == 'v') {
            const uint64_t chunks = (uint64_t)rows * stride / 16;
            hipLaunchKernelGGL(vec16, dim3(4096), dim3(256), 0, 0, (const uint4*)p, chunks, out);
        } else {
            const int groups = 64 / G;
            const uint32_t blocks = (rows + 2 * groups - 1) / (2 * groups);
            hipLaunchKernelGGL(bytes_sw, dim3(blocks), dim3(64), 0, 0, p, stride, rows, KR, G, out);
        }
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("%s stride=%u KR=%d G=%d rows=%u buffer=%llu bytes touched-per-row=%d\n", mode, stride, KR, G, rows,
           (unsigned long long)rows * stride, mode[0] == 'v' ? (int)stride : (G * KR < (int)stride ? G * KR : (int)stride));
    return 0;
}
