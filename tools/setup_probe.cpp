// Where the --full-wgs setup goes (setup_phases): the HIP
// calls of msw_ctx_create, msw_genome_create and the lane reader's buffers,
// each timed, on W worker threads side by side (the CLI's two workers per GPU)
// after the runtime init, then once more serially.  One JSON line per pass.
//
//   hipcc -O2 -std=c++17 tools/setup_probe.cpp -o tools/_variants/setup_probe
//   tools/_variants/setup_probe [workers=2] [genome_mb=64]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

using Clock = std::chrono::steady_clock;
static double ms(Clock::time_point a, Clock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
}

struct Steps {
    std::vector<std::pair<std::string, double>> v;
    Clock::time_point t = Clock::now();
    void mark(const char* name) {
        const auto n = Clock::now();
        v.emplace_back(name, ms(t, n));
        t = n;
    }
    std::string json() const {
        std::string s = "{";
        for (size_t i = 0; i < v.size(); ++i) {
            char b[96];
            snprintf(b, sizeof(b), "%s\"%s\": %.2f", i ? ", " : "", v[i].first.c_str(), v[i].second);
            s += b;
        }
        return s + "}";
    }
};

#define OK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ void touch(int* p) { p[threadIdx.x] = (int)threadIdx.x; }

// one worker's setup, in the CLI's order
static Steps worker(const std::vector<uint8_t>& genome) {
    Steps s;
    OK(hipSetDevice(0));
    s.mark("set_device");
    hipDeviceProp_t prop;
    OK(hipGetDeviceProperties(&prop, 0));
    s.mark("device_properties");
    hipStream_t st[5];
    for (int k = 0; k < 5; ++k) {
        OK(hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking));
        s.mark(k == 0 ? "stream_create_1" : "stream_create_2to5");
    }
    hipEvent_t ev;
    OK(hipEventCreate(&ev));
    OK(hipEventRecord(ev, st[0]));
    s.mark("event_create_record");
    uint8_t* d_gen = nullptr;
    OK(hipMalloc((void**)&d_gen, genome.size() + 4096));
    s.mark("genome_malloc");
    OK(hipMemsetAsync(d_gen + genome.size(), 0, 4096, st[2]));
    OK(hipStreamSynchronize(st[2]));
    s.mark("genome_memset_first_blit");
    OK(hipMemcpyAsync(d_gen, genome.data(), genome.size(), hipMemcpyHostToDevice, st[2]));
    OK(hipStreamSynchronize(st[2]));
    s.mark("genome_h2d_pageable");
    const size_t batch = 1 << 20;
    void* d[8];
    for (int k = 0; k < 8; ++k) OK(hipMalloc(&d[k], batch * 4));
    s.mark("result_malloc_x8");
    void* h[2];
    for (int k = 0; k < 2; ++k) OK(hipHostMalloc(&h[k], batch * 12, hipHostMallocDefault));
    s.mark("result_host_malloc_2x12MB");
    int* dk = nullptr;
    OK(hipMalloc((void**)&dk, 256 * 4));
    hipLaunchKernelGGL(touch, dim3(1), dim3(256), 0, st[0], dk);
    OK(hipStreamSynchronize(st[0]));
    s.mark("first_kernel_launch");
    void* big = nullptr;
    OK(hipMalloc(&big, 512ull << 20));
    s.mark("reader_malloc_512MB");
    void* hp = nullptr;
    OK(hipHostMalloc(&hp, 64ull << 20, hipHostMallocDefault));
    s.mark("reader_host_malloc_64MB");
    OK(hipFree(big));
    OK(hipHostFree(hp));
    OK(hipFree(dk));
    for (int k = 0; k < 2; ++k) OK(hipHostFree(h[k]));
    for (int k = 0; k < 8; ++k) OK(hipFree(d[k]));
    OK(hipFree(d_gen));
    OK(hipEventDestroy(ev));
    for (int k = 0; k < 5; ++k) OK(hipStreamDestroy(st[k]));
    s.mark("teardown");
    return s;
}

int main(int argc, char** argv) {
    const int workers = argc > 1 ? atoi(argv[1]) : 2;
    const size_t gmb = argc > 2 ? (size_t)atoll(argv[2]) : 64;
    std::vector<uint8_t> genome(gmb << 20);
    for (size_t i = 0; i < genome.size(); ++i) genome[i] = "ACGT"[(i * 2654435761u >> 7) & 3];
    const auto t0 = Clock::now();
    int n = 0;
    OK(hipGetDeviceCount(&n));
    const auto t1 = Clock::now();
    hipDeviceProp_t prop;
    OK(hipGetDeviceProperties(&prop, 0));
    const auto t2 = Clock::now();
    printf("{\"pass\": \"init\", \"hip_get_device_count_ms\": %.2f, \"device_properties_ms\": %.2f, \"gpus\": %d}\n",
           ms(t0, t1), ms(t1, t2), n);
    for (int pass = 0; pass < 2; ++pass) {
        std::vector<Steps> res((size_t)workers);
        std::vector<std::thread> th;
        const auto p0 = Clock::now();
        for (int w = 0; w < workers; ++w) th.emplace_back([&, w]() { res[(size_t)w] = worker(genome); });
        for (auto& t : th) t.join();
        printf("{\"pass\": \"%s\", \"workers\": %d, \"wall_ms\": %.2f", pass ? "parallel_again" : "parallel_first",
               workers, ms(p0, Clock::now()));
        for (int w = 0; w < workers; ++w) printf(", \"w%d\": %s", w, res[(size_t)w].json().c_str());
        printf("}\n");
        fflush(stdout);
    }
    return 0;
}
