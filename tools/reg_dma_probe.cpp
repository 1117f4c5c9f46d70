// Host-to-device DMA from a lane file's page cache, the three ways the GPU
// lane reader can source it: the whole mapping pinned once
// (hipHostRegister), one pinned window per copy (register / copy / unregister),
// and a hipHostMalloc'ed staging buffer (pread + copy).  Per copy: the host
// time inside hipMemcpyAsync and the time to completion.
//   hipcc -O2 -o tools/bin/reg_dma_probe tools/reg_dma_probe.cpp
//   tools/bin/reg_dma_probe FILE [WINDOW_MB]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const size_t win = (size_t)(argc > 2 ? atoi(argv[2]) : 290) << 20;
    const int fd = open(argv[1], O_RDONLY);
    if (fd < 0) return 2;
    struct stat sb;
    fstat(fd, &sb);
    const size_t fsize = (size_t)sb.st_size;
    uint8_t* map = (uint8_t*)mmap(nullptr, fsize, PROT_READ, MAP_SHARED, fd, 0);
    if (map == MAP_FAILED) return 2;
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    uint8_t* d = nullptr;
    CK(hipMalloc((void**)&d, win));
    const size_t nwin = fsize / win;
    printf("{\"file_mb\": %.1f, \"window_mb\": %.1f, \"windows\": %zu}\n", fsize / 1e6, win / 1e6, nwin);
    // 1. whole mapping pinned once
    double t0 = now_ms();
    CK(hipHostRegister(map, fsize, hipHostRegisterReadOnly));
    printf("{\"mode\": \"whole\", \"register_ms\": %.2f}\n", now_ms() - t0);
    for (size_t k = 0; k < nwin; ++k) {
        const double a = now_ms();
        CK(hipMemcpyAsync(d, map + k * win, win, hipMemcpyHostToDevice, s));
        const double b = now_ms();
        CK(hipStreamSynchronize(s));
        const double c = now_ms();
        printf("{\"mode\": \"whole\", \"k\": %zu, \"call_ms\": %.2f, \"done_ms\": %.2f, \"gbps\": %.1f}\n", k, b - a,
               c - a, win / ((c - a) * 1e6));
    }
    t0 = now_ms();
    CK(hipHostUnregister(map));
    printf("{\"mode\": \"whole\", \"unregister_ms\": %.2f}\n", now_ms() - t0);
    // 2. one pinned window per copy
    for (size_t k = 0; k < nwin; ++k) {
        const double a = now_ms();
        CK(hipHostRegister(map + k * win, win, hipHostRegisterReadOnly));
        const double b = now_ms();
        CK(hipMemcpyAsync(d, map + k * win, win, hipMemcpyHostToDevice, s));
        const double c = now_ms();
        CK(hipStreamSynchronize(s));
        const double e = now_ms();
        CK(hipHostUnregister(map + k * win));
        const double f = now_ms();
        printf("{\"mode\": \"window\", \"k\": %zu, \"register_ms\": %.2f, \"call_ms\": %.2f, \"done_ms\": %.2f, "
               "\"unregister_ms\": %.2f, \"gbps\": %.1f}\n",
               k, b - a, c - b, e - b, f - e, win / ((e - b) * 1e6));
    }
    // 3. pinned staging
    uint8_t* h = nullptr;
    CK(hipHostMalloc((void**)&h, win, hipHostMallocDefault));
    for (size_t k = 0; k < nwin; ++k) {
        const double a = now_ms();
        if (pread(fd, h, win, (off_t)(k * win)) != (ssize_t)win) return 3;
        const double b = now_ms();
        CK(hipMemcpyAsync(d, h, win, hipMemcpyHostToDevice, s));
        const double c = now_ms();
        CK(hipStreamSynchronize(s));
        const double e = now_ms();
        printf("{\"mode\": \"staged\", \"k\": %zu, \"pread_ms\": %.2f, \"call_ms\": %.2f, \"done_ms\": %.2f, "
               "\"gbps\": %.1f}\n",
               k, b - a, c - b, e - b, win / ((e - b) * 1e6));
    }
    CK(hipHostFree(h));
    CK(hipFree(d));
    munmap(map, fsize);
    close(fd);
    return 0;
}
