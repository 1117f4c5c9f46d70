// host_feed -- the host side of the config-4 GPU lane reader, measured alone
// (VERDICT r2 item 3).  Each lane stream copies its lane file's compressed
// bytes from the page cache into pinned staging the way msw_gfastq.cpp's
// fill_compressed does (positioned 8 MiB preads split over T threads into a
// hipHostMalloc'ed buffer), with no GPU kernel running; S streams run at once.
// Also measured: hipHostRegister of the mmap'ed file (the pages the page
// cache already holds, pinned in place) + a DMA of them to the GPU, the
// zero-memcpy alternative.
//
//   hipcc --offload-arch=gfx950 -O2 tools/host_feed.cpp -o tools/host_feed
//   tools/host_feed OUT.jsonl FILE...      (files should be in the page cache)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace {

using Clock = std::chrono::steady_clock;
constexpr size_t kPiece = 8u << 20;      // fill_compressed's pread piece
constexpr size_t kStage = 512u << 20;    // per stream: ~the reader's staging (half a 1 GiB span)

double secs(Clock::time_point a) { return std::chrono::duration<double>(Clock::now() - a).count(); }

size_t file_size(const char* p) {
    struct stat st;
    return stat(p, &st) == 0 ? (size_t)st.st_size : 0;
}

// stream s: file f, T threads, contiguous ranges, pieces written round-robin into a kStage ring
void stream_copy(const char* path, int T, uint8_t* stage, std::atomic<size_t>* bytes) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return;
    const size_t n = file_size(path);
    const size_t per = (n + T - 1) / T;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) {
        th.emplace_back([=]() {
            size_t off = per * t, end = std::min(n, off + per), got = 0;
            while (off < end) {
                const size_t len = std::min(kPiece, end - off);
                uint8_t* dst = stage + (off % (kStage - kPiece));
                const ssize_t r = pread(fd, dst, len, (off_t)off);
                if (r <= 0) break;
                off += (size_t)r;
                got += (size_t)r;
            }
            bytes->fetch_add(got);
        });
    }
    for (auto& x : th) x.join();
    close(fd);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s OUT.jsonl FILE...\n", argv[0]);
        return 2;
    }
    FILE* out = fopen(argv[1], "a");
    std::vector<const char*> files(argv + 2, argv + argc);
    size_t total = 0;
    for (const char* f : files) total += file_size(f);
    // warm the page cache: read every file once
    {
        std::vector<uint8_t> buf(kPiece);
        for (const char* f : files) {
            const int fd = open(f, O_RDONLY);
            while (fd >= 0 && read(fd, buf.data(), buf.size()) > 0) {
            }
            if (fd >= 0) close(fd);
        }
    }
    const int max_streams = (int)files.size();
    std::vector<uint8_t*> stage((size_t)max_streams, nullptr);
    auto t0 = Clock::now();
    for (auto& p : stage)
        if (hipHostMalloc((void**)&p, kStage, hipHostMallocDefault) != hipSuccess) {
            fprintf(stderr, "hipHostMalloc failed\n");
            return 1;
        }
    const double pin_s = secs(t0);
    fprintf(out, "{\"probe\": \"hipHostMalloc\", \"buffers\": %d, \"mb_each\": %zu, \"seconds\": %.4f, \"gb_per_s\": %.2f}\n",
            max_streams, kStage >> 20, pin_s, max_streams * (double)kStage / pin_s / 1e9);
    fflush(out);
    // pread -> pinned, S streams x T threads each
    for (int S : {1, 2, 4, 8, 16}) {
        if (S > max_streams) break;
        for (int T : {1, 2, 4, 8}) {
            double best = 1e30;
            size_t moved = 0;
            for (int rep = 0; rep < 3; ++rep) {
                std::atomic<size_t> bytes{0};
                std::vector<std::thread> ss;
                auto ts = Clock::now();
                for (int s = 0; s < S; ++s) ss.emplace_back(stream_copy, files[(size_t)s], T, stage[(size_t)s], &bytes);
                for (auto& x : ss) x.join();
                const double dt = secs(ts);
                if (dt < best) {
                    best = dt;
                    moved = bytes.load();
                }
            }
            fprintf(out, "{\"probe\": \"pread_to_pinned\", \"streams\": %d, \"threads_per_stream\": %d, "
                         "\"bytes\": %zu, \"seconds\": %.4f, \"gb_per_s\": %.2f, \"gb_per_s_per_stream\": %.2f}\n",
                    S, T, moved, best, moved / best / 1e9, moved / best / 1e9 / S);
            fflush(out);
        }
    }
    // hipHostRegister of the mmap'ed file, then one DMA to the GPU (no CPU copy)
    void* dev = nullptr;
    size_t maxf = 0;
    for (const char* f : files) maxf = std::max(maxf, file_size(f));
    if (hipMalloc(&dev, maxf) != hipSuccess) return 1;
    for (size_t i = 0; i < std::min<size_t>(files.size(), 4); ++i) {
        const size_t n = file_size(files[i]);
        const int fd = open(files[i], O_RDONLY);
        void* p = mmap(nullptr, n, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
        close(fd);
        if (p == MAP_FAILED) continue;
        for (unsigned flags : {(unsigned)hipHostRegisterReadOnly, (unsigned)hipHostRegisterDefault}) {
            auto ts = Clock::now();
            const hipError_t e = hipHostRegister(p, n, flags);
            const double reg = secs(ts);
            double dma = 0;
            if (e == hipSuccess) {
                ts = Clock::now();
                (void)hipMemcpy(dev, p, n, hipMemcpyHostToDevice);
                dma = secs(ts);
                ts = Clock::now();
                (void)hipHostUnregister(p);
            } else {
                (void)hipGetLastError();
            }
            const double unreg = e == hipSuccess ? secs(ts) : 0;
            fprintf(out, "{\"probe\": \"register_mmap\", \"file\": \"%s\", \"bytes\": %zu, \"flags\": %u, \"ok\": %s, "
                         "\"error\": \"%s\", \"register_s\": %.4f, \"dma_s\": %.4f, \"unregister_s\": %.4f, "
                         "\"register_gb_per_s\": %.2f, \"dma_gb_per_s\": %.2f}\n",
                    files[i], n, flags, e == hipSuccess ? "true" : "false", hipGetErrorString(e), reg, dma, unreg,
                    e == hipSuccess ? n / reg / 1e9 : 0.0, e == hipSuccess && dma > 0 ? n / dma / 1e9 : 0.0);
            fflush(out);
            if (e == hipSuccess) break;
        }
        munmap(p, n);
    }
    // the same bytes from pinned staging to the GPU (the reader's H2D today)
    {
        const size_t n = std::min(maxf, kStage);
        auto ts = Clock::now();
        (void)hipMemcpy(dev, stage[0], n, hipMemcpyHostToDevice);
        const double dt = secs(ts);
        fprintf(out, "{\"probe\": \"pinned_h2d\", \"bytes\": %zu, \"seconds\": %.4f, \"gb_per_s\": %.2f}\n", n, dt,
                n / dt / 1e9);
    }
    for (auto p : stage) (void)hipHostFree(p);
    (void)hipFree(dev);
    fprintf(out, "{\"probe\": \"summary\", \"files\": %zu, \"total_bytes\": %zu, \"hardware_concurrency\": %u}\n",
            files.size(), total, std::thread::hardware_concurrency());
    fclose(out);
    return 0;
}
