// fastq_dump -- a C++ consumer of the host FASTQ reader (include/msw_fastq.h)
// for the sanitizer build (`make -C mini_parallel_amd/csrc asan`):
// built with -fsanitize=address,undefined against build/asan/libmsw.so, it
// runs the reader the way tests/test_fastq.py does through ctypes and prints
// what it read, so tests/test_asan.py can check the same cases against the
// restatement of aligner.rs:107-178 with every heap access checked.
//
//   fastq_dump concat PATH N            chunks of N reads (next_packed, buffer grown on `need`)
//   fastq_dump slab PATH MAX STRIDE     msw_fastq_next with pos, one call per MAX reads
//   fastq_dump packed PATH MAX CAP      msw_fastq_next_packed with a fixed cap (grown on `need`)
//   fastq_dump count PATH               msw_fastq_count_bases
// Output: one record per line ("C n" chunk header, "S len pos seq", "N need",
// "B bases reads", "T lines reads errors"); an error prints "ERR code message"
// and exits 3.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "msw.h"
#include "msw_fastq.h"

namespace {

int fail(int rc) {
    printf("ERR %d %s\n", rc, msw_last_error());
    return 3;
}

void stats(msw_fastq* fq) {
    uint64_t l = 0, r = 0, e = 0;
    msw_fastq_stats(fq, &l, &r, &e);
    printf("T %llu %llu %llu\n", (unsigned long long)l, (unsigned long long)r, (unsigned long long)e);
}

int concat(const char* path, uint64_t n) {
    msw_fastq* fq = nullptr;
    if (int rc = msw_fastq_open(path, &fq)) return fail(rc);
    std::vector<uint8_t> buf(1024);
    std::vector<uint32_t> lens(n);
    int rc = 0;
    for (;;) {
        std::string chunk;
        std::vector<uint32_t> got;
        while (got.size() < n) {
            uint64_t k = 0, nb = 0, need = 0;
            rc = msw_fastq_next_packed(fq, buf.data(), buf.size(), lens.data(), n - got.size(), &k, &nb, &need);
            if (rc) break;
            chunk.append(reinterpret_cast<const char*>(buf.data()), nb);
            got.insert(got.end(), lens.begin(), lens.begin() + (long)k);
            if (need) buf.resize(std::max<size_t>(2 * buf.size(), need));
            else if (got.size() < n) break;
        }
        if (rc || got.empty()) break;
        printf("C %zu\n", got.size());
        size_t off = 0;
        for (uint32_t L : got) {
            printf("S %u -1 %.*s\n", L, (int)L, chunk.data() + off);
            off += L;
        }
    }
    if (rc) {
        msw_fastq_close(fq);
        return fail(rc);
    }
    stats(fq);
    msw_fastq_close(fq);
    return 0;
}

int slab(const char* path, uint64_t max, uint32_t stride) {
    msw_fastq* fq = nullptr;
    if (int rc = msw_fastq_open(path, &fq)) return fail(rc);
    std::vector<uint8_t> seqs(max * stride);
    std::vector<uint16_t> lens(max);
    std::vector<int64_t> pos(max);
    for (;;) {
        std::fill(seqs.begin(), seqs.end(), 0xAB);  // padding must come back zeroed
        uint64_t k = 0;
        if (int rc = msw_fastq_next(fq, seqs.data(), lens.data(), stride, max, &k, pos.data())) {
            msw_fastq_close(fq);
            return fail(rc);
        }
        if (!k) break;
        printf("C %llu\n", (unsigned long long)k);
        for (uint64_t i = 0; i < k; ++i) {
            const uint8_t* row = seqs.data() + i * stride;
            for (uint32_t b = lens[i]; b < stride; ++b)
                if (row[b]) {
                    printf("PADERR %llu %u\n", (unsigned long long)i, b);
                    break;
                }
            printf("S %u %lld %.*s\n", lens[i], (long long)pos[i], (int)lens[i], reinterpret_cast<const char*>(row));
        }
    }
    stats(fq);
    msw_fastq_close(fq);
    return 0;
}

int packed(const char* path, uint64_t max, uint64_t cap) {
    msw_fastq* fq = nullptr;
    if (int rc = msw_fastq_open(path, &fq)) return fail(rc);
    std::vector<uint8_t> buf(std::max<uint64_t>(cap, 1));
    std::vector<uint32_t> lens(std::max<uint64_t>(max, 1));
    for (;;) {
        uint64_t k = 0, nb = 0, need = 0;
        if (int rc = msw_fastq_next_packed(fq, buf.data(), cap, lens.data(), max, &k, &nb, &need)) {
            msw_fastq_close(fq);
            return fail(rc);
        }
        printf("C %llu\n", (unsigned long long)k);
        uint64_t off = 0;
        for (uint64_t i = 0; i < k; ++i) {
            printf("S %u -1 %.*s\n", lens[i], (int)lens[i], reinterpret_cast<const char*>(buf.data() + off));
            off += lens[i];
        }
        if (off != nb || nb > cap) printf("SIZEERR %llu %llu\n", (unsigned long long)off, (unsigned long long)nb);
        if (need) {
            printf("N %llu\n", (unsigned long long)need);
            if (need > cap) {
                cap = need;
                buf.resize(cap);
            }
        } else if (!k) {
            break;
        }
    }
    stats(fq);
    msw_fastq_close(fq);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: fastq_dump concat|slab|packed|count PATH [ARGS]\n");
        return 2;
    }
    const std::string cmd = argv[1];
    const char* path = argv[2];
    if (cmd == "concat" && argc == 4) return concat(path, strtoull(argv[3], nullptr, 10));
    if (cmd == "slab" && argc == 5) return slab(path, strtoull(argv[3], nullptr, 10), (uint32_t)atoi(argv[4]));
    if (cmd == "packed" && argc == 5) return packed(path, strtoull(argv[3], nullptr, 10), strtoull(argv[4], nullptr, 10));
    if (cmd == "count" && argc == 3) {
        uint64_t b = 0, r = 0;
        if (int rc = msw_fastq_count_bases(path, &b, &r)) return fail(rc);
        printf("B %llu %llu\n", (unsigned long long)b, (unsigned long long)r);
        return 0;
    }
    fprintf(stderr, "bad arguments\n");
    return 2;
}
