// stream_bench.cpp -- host-to-host streaming rate of the C ABI without any
// Python in the loop: a stream of batches (pairs cut from a resident genome,
// reads + window positions in pinned host memory) submitted with
// msw_align_reads_async, `inflight` outstanding, results back in host memory.
// Build: make -C mini_parallel_amd/csrc ../../tools/stream_bench
// Run:   tools/stream_bench [pairs_per_batch=10000] [batches=64] [inflight=2]
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "msw.h"

static void die(const char* what) {
    fprintf(stderr, "%s: %s\n", what, msw_last_error());
    exit(1);
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 10000;
    const int batches = argc > 2 ? atoi(argv[2]) : 64;
    const int inflight = argc > 3 ? atoi(argv[3]) : 2;
    const uint32_t m = 150, w = 300, rs = 160;
    msw_ctx* ctx = nullptr;
    if (msw_ctx_create(0, &ctx)) die("ctx");
    // genome: 64 Mbp of ACGT; reads copied from it (so alignments are real)
    const uint64_t glen = 64ull << 20;
    std::vector<uint8_t> genome(glen);
    std::mt19937_64 rng(1002);
    const char* acgt = "ACGT";
    for (auto& b : genome) b = (uint8_t)acgt[rng() & 3];
    msw_genome* g = nullptr;
    if (msw_genome_create(ctx, genome.data(), glen, &g)) die("genome");
    uint8_t* reads = (uint8_t*)msw_host_alloc(n * rs);
    uint16_t* rlen = (uint16_t*)msw_host_alloc(n * 2);
    int64_t* pos = (int64_t*)msw_host_alloc(n * 8);
    uint16_t* wlen = (uint16_t*)msw_host_alloc(n * 2);
    if (!reads || !rlen || !pos || !wlen) die("pinned");
    for (uint64_t i = 0; i < n; ++i) {
        pos[i] = (int64_t)(rng() % (glen - w));
        memset(reads + i * rs, 0, rs);
        memcpy(reads + i * rs, genome.data() + pos[i] + (w - m) / 2, m);
        reads[i * rs + (rng() % m)] = 'A';  // a substitution or two
        rlen[i] = (uint16_t)m;
        wlen[i] = (uint16_t)w;
    }
    const msw_scoring_t sc = {2, -1, 0, 2, 0, 0};
    const msw_read_batch_t rb = {reads, rlen, rs, pos, wlen, n};
    std::vector<std::vector<int32_t>> score(inflight, std::vector<int32_t>(n));
    std::vector<uint64_t> ticket(inflight, 0);
    auto run = [&](int count) {
        for (int b = 0; b < count; ++b) {
            const int slot = b % inflight;
            if (ticket[slot] && msw_wait(ctx, ticket[slot])) die("wait");
            msw_out_t o = {score[slot].data(), nullptr, nullptr};
            if (msw_align_reads_async(ctx, &sc, g, &rb, &o, 0, &ticket[slot])) die("submit");
        }
        for (int s = 0; s < inflight; ++s)
            if (ticket[s] && msw_wait(ctx, ticket[s])) die("wait");
        std::fill(ticket.begin(), ticket.end(), 0);
    };
    run(8);  // warm up
    const auto t0 = std::chrono::steady_clock::now();
    run(batches);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    long long sum = 0;
    for (uint64_t i = 0; i < n; ++i) sum += score[0][i];
    const double cells = (double)n * m * w * batches;
    printf("{\"pairs_per_batch\": %llu, \"batches\": %d, \"inflight\": %d, \"us_per_batch\": %.1f, "
           "\"gcups\": %.1f, \"score_sum_last\": %lld}\n",
           (unsigned long long)n, batches, inflight, s / batches * 1e6, cells / s / 1e9, sum);
    msw_genome_destroy(g);
    msw_host_free(reads);
    msw_host_free(rlen);
    msw_host_free(pos);
    msw_host_free(wlen);
    msw_ctx_destroy(ctx);
    return 0;
}
