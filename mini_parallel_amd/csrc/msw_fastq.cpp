// msw_fastq.cpp -- FASTQ(.gz) chunk reader (include/msw_fastq.h).
//
// Semantics of process_fastq_file_in_chunks (aligner.rs:107-178); see the
// header.  One reader per lane file; no per-line allocation: records are
// parsed out of a 4 MiB decompressed block buffer and sequences are copied
// straight into the caller's SoA slab.
#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/msw.h"
#include "../../include/msw_fastq.h"

namespace msw_detail {
// Shared with msw_runtime.cpp: sets the thread-local msw_last_error message.
int set_error(int code, const char* fmt, ...);
}  // namespace msw_detail

using msw_detail::set_error;

struct msw_fastq {
    gzFile gz = nullptr;      // zlib reads plain files transparently too
    FILE* raw = nullptr;      // BGZF files decoded block by block with libdeflate
    std::vector<void*> inflaters;  // libdeflate decompressors, one per inflate thread (BGZF mode)
    std::vector<unsigned char> cblock;  // one compressed BGZF block
    std::string io_msg;       // last BGZF decode error
    std::vector<char> buf;    // decompressed bytes
    size_t head = 0, tail = 0;
    bool eof = false;
    std::string carry;        // partial line across buffer refills
    std::string last;         // final line of a file without a trailing newline
    uint64_t lines = 0, reads = 0, errors = 0;
    int64_t pending_pos = -1; // pos= tag of the current record's header
    std::string held;         // msw_fastq_next_packed: a sequence that did not fit the caller's buffer
    bool has_held = false;
    std::string path;
};

namespace {

constexpr size_t kBlock = 4u << 20;

// ---------------------------------------------------------------------------
// BGZF lane files (multi-member gzip whose members are <= 64 KiB blocks with a
// 'BC' extra field carrying the block size, as written by bgzip) are inflated
// block by block with libdeflate (the image's libdeflate.so.0, loaded at run
// time; ~2-3x zlib's inflate rate).  Any other gzip -- and every file when
// libdeflate is absent or MSW_NO_LIBDEFLATE is set -- streams through zlib.
// Both paths yield the same bytes (tests/test_fastq.py).
// ---------------------------------------------------------------------------
struct Deflate {
    void* (*alloc)() = nullptr;
    int (*decompress)(void*, const void*, size_t, void*, size_t, size_t*) = nullptr;
    void (*free_)(void*) = nullptr;
    uint32_t (*crc32)(uint32_t, const void*, size_t) = nullptr;
    bool ok = false;
};

const Deflate& libdeflate() {
    static Deflate d;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        d.alloc = (void* (*)())dlsym(h, "libdeflate_alloc_decompressor");
        d.decompress = (int (*)(void*, const void*, size_t, void*, size_t, size_t*))dlsym(h, "libdeflate_deflate_decompress");
        d.free_ = (void (*)(void*))dlsym(h, "libdeflate_free_decompressor");
        d.crc32 = (uint32_t(*)(uint32_t, const void*, size_t))dlsym(h, "libdeflate_crc32");
        d.ok = d.alloc && d.decompress && d.free_ && d.crc32;
    });
    return d;
}

// Size of the BGZF block whose 18-byte header is h, or 0 if h is not one.
size_t bgzf_block_size(const unsigned char* h) {
    if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) return 0;
    const unsigned xlen = h[10] | (h[11] << 8);
    if (xlen != 6 || h[12] != 'B' || h[13] != 'C' || (h[14] | (h[15] << 8)) != 2) return 0;
    return (size_t)(h[16] | (h[17] << 8)) + 1;
}

bool is_bgzf(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) return false;
    unsigned char h[18];
    const bool yes = fread(h, 1, 18, f) == 18 && bgzf_block_size(h) >= 26;
    fclose(f);
    return yes;
}

// Inflate whole BGZF blocks into out[0, cap) while another block surely fits
// (a block holds <= 64 KiB); returns bytes produced, 0 at end of file, -1 on
// a read / format / checksum error (fq->io_msg says which).  The compressed
// blocks are read first (each trailer gives its output size, hence its output
// offset), then inflated -- by fq->inflaters.size() threads when the reader
// was opened with MSW_INFLATE_THREADS > 1.
long bgzf_fill(msw_fastq* fq, char* out, size_t cap) {
    const Deflate& d = libdeflate();
    struct Blk {
        size_t coff, clen, ooff;
        uint32_t isize, crc;
    };
    std::vector<Blk> blks;
    fq->cblock.clear();
    size_t n = 0;
    while (n + 65536 <= cap) {
        unsigned char h[18];
        const size_t got = fread(h, 1, 18, fq->raw);
        if (got == 0 && feof(fq->raw)) break;
        const size_t bsize = got == 18 ? bgzf_block_size(h) : 0;
        if (bsize < 26) {
            fq->io_msg = "not a BGZF block (mixed gzip members are not supported in BGZF mode)";
            return -1;
        }
        const size_t at = fq->cblock.size();
        fq->cblock.resize(at + bsize - 18);
        if (fread(fq->cblock.data() + at, 1, bsize - 18, fq->raw) != bsize - 18) {
            fq->io_msg = "unexpected end of file";
            return -1;
        }
        const unsigned char* t = fq->cblock.data() + at + bsize - 26;
        const uint32_t crc = t[0] | (t[1] << 8) | (t[2] << 16) | ((uint32_t)t[3] << 24);
        const uint32_t isize = t[4] | (t[5] << 8) | (t[6] << 16) | ((uint32_t)t[7] << 24);
        if (isize > 65536) {
            fq->io_msg = "BGZF block larger than 64 KiB";
            return -1;
        }
        if (isize) blks.push_back({at, bsize - 26, n, isize, crc});
        n += isize;
    }
    std::atomic<size_t> next{0};
    std::atomic<bool> bad{false};
    auto work = [&](void* inflater) {
        for (size_t k; (k = next.fetch_add(1)) < blks.size();) {
            const Blk& bk = blks[k];
            size_t actual = 0;
            if (d.decompress(inflater, fq->cblock.data() + bk.coff, bk.clen, out + bk.ooff, bk.isize, &actual) != 0 ||
                actual != bk.isize || d.crc32(0, out + bk.ooff, bk.isize) != bk.crc)
                bad = true;
        }
    };
    const size_t nt = std::min(fq->inflaters.size(), blks.size());
    std::vector<std::thread> pool;
    for (size_t t = 1; t < nt; ++t) pool.emplace_back(work, fq->inflaters[t]);
    work(fq->inflaters[0]);
    for (auto& th : pool) th.join();
    if (bad) {
        fq->io_msg = "invalid compressed data";
        return -1;
    }
    return (long)n;
}

// Strict UTF-8 validation (what Rust's String conversion in lines() checks).
bool valid_utf8(const unsigned char* s, size_t n) {
    size_t i = 0;
    // ASCII fast path, 8 bytes at a time (FASTQ lines are ASCII)
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, s + i, 8);
        if (w & 0x8080808080808080ull) break;
    }
    while (i < n) {
        unsigned char c = s[i];
        if (c < 0x80) { ++i; continue; }
        size_t len;
        uint32_t cp;
        if ((c & 0xE0) == 0xC0) { len = 2; cp = c & 0x1F; }
        else if ((c & 0xF0) == 0xE0) { len = 3; cp = c & 0x0F; }
        else if ((c & 0xF8) == 0xF0) { len = 4; cp = c & 0x07; }
        else return false;
        if (i + len > n) return false;
        for (size_t k = 1; k < len; ++k) {
            if ((s[i + k] & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (s[i + k] & 0x3F);
        }
        if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && cp < 0x10000) ||
            cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF))
            return false;
        i += len;
    }
    return true;
}

int64_t parse_pos(const char* s, size_t n) {
    for (size_t i = 0; i + 4 <= n; ++i) {
        if (memcmp(s + i, "pos=", 4) == 0) {
            size_t j = i + 4;
            bool neg = j < n && s[j] == '-';
            if (neg) ++j;
            int64_t v = 0;
            bool any = false;
            while (j < n && s[j] >= '0' && s[j] <= '9') { v = v * 10 + (s[j] - '0'); ++j; any = true; }
            if (any) return neg ? -v : v;
        }
    }
    return -1;
}

// Next raw line (without '\n'); false at end of data or on an I/O error
// (*io_err set).  The pointer stays valid until the next call.
bool next_line(msw_fastq* fq, const char** line, size_t* len, int* io_err) {
    for (;;) {
        if (fq->head < fq->tail) {
            const char* start = fq->buf.data() + fq->head;
            const char* nl = (const char*)memchr(start, '\n', fq->tail - fq->head);
            if (nl) {
                const size_t n = (size_t)(nl - start);
                fq->head += n + 1;
                if (!fq->carry.empty()) {
                    fq->last.assign(fq->carry);
                    fq->last.append(start, n);
                    fq->carry.clear();
                    *line = fq->last.data();
                    *len = fq->last.size();
                } else {
                    *line = start;
                    *len = n;
                }
                return true;
            }
            fq->carry.append(start, fq->tail - fq->head);
            fq->head = fq->tail;
        }
        if (fq->eof) {
            if (fq->carry.empty()) return false;
            fq->last.swap(fq->carry);  // last line without a newline
            fq->carry.clear();
            *line = fq->last.data();
            *len = fq->last.size();
            return true;
        }
        const long got = fq->raw ? bgzf_fill(fq, fq->buf.data(), kBlock)
                                 : (long)gzread(fq->gz, fq->buf.data(), (unsigned)kBlock);
        if (got < 0) {
            *io_err = 1;
            return false;
        }
        if (got == 0) fq->eof = true;
        fq->head = 0;
        fq->tail = (size_t)got;
    }
}

// Next sequence line (1-based line % 4 == 2) with aligner.rs:133-165 rules.
// Returns 1 with the bytes, 0 at end of file, or a negative MSW error.
int next_sequence(msw_fastq* fq, const char** seq, size_t* len, int64_t* pos, bool want_pos) {
    for (;;) {
        const char* line;
        size_t n;
        int io_err = 0;
        if (!next_line(fq, &line, &n, &io_err)) {
            if (!io_err) return 0;
            int zerr = 0;
            const char* msg = fq->raw ? fq->io_msg.c_str() : gzerror(fq->gz, &zerr);
            if (++fq->errors > 10)
                return set_error(MSW_E_INVALID, "Too many read errors (>10), stopping at line %llu",
                                 (unsigned long long)fq->lines);
            return set_error(MSW_E_INVALID, "Error reading %s: %s", fq->path.c_str(), msg ? msg : "");
        }
        if (n && line[n - 1] == '\r') --n;  // CRLF, as BufRead::lines
        if (!valid_utf8((const unsigned char*)line, n)) {
            if (++fq->errors > 10)
                return set_error(MSW_E_INVALID, "Too many read errors (>10), stopping at line %llu",
                                 (unsigned long long)fq->lines);
            continue;  // aligner.rs:155-163: skipped and not counted
        }
        ++fq->lines;
        const uint64_t phase = fq->lines % 4;
        if (phase == 1) {
            fq->pending_pos = want_pos ? parse_pos(line, n) : -1;
        } else if (phase == 2) {
            *seq = line;
            *len = n;
            *pos = fq->pending_pos;
            fq->pending_pos = -1;
            ++fq->reads;
            return 1;
        }
    }
}

}  // namespace

extern "C" {

int msw_fastq_open(const char* path, msw_fastq** out) {
    if (!path || !out) return set_error(MSW_E_INVALID, "path/out is NULL");
    *out = nullptr;
    msw_fastq* fq = new msw_fastq();
    const Deflate& d = libdeflate();
    if (d.ok && !getenv("MSW_NO_LIBDEFLATE") && is_bgzf(path)) {
        fq->raw = fopen(path, "rb");
        const char* nt = getenv("MSW_INFLATE_THREADS");
        const int threads = std::max(1, std::min(64, nt ? atoi(nt) : 1));
        for (int t = 0; fq->raw && t < threads; ++t)
            if (void* inf = d.alloc()) fq->inflaters.push_back(inf);
        if (fq->raw) setvbuf(fq->raw, nullptr, _IOFBF, 1u << 20);
    }
    if (fq->inflaters.empty()) {
        if (fq->raw) fclose(fq->raw);
        fq->raw = nullptr;
        gzFile gz = gzopen(path, "rb");
        if (!gz) {
            delete fq;
            return set_error(MSW_E_INVALID, "Failed to open file %s", path);
        }
        gzbuffer(gz, 1u << 20);
        fq->gz = gz;
    }
    fq->buf.resize(kBlock);
    fq->path = path;
    *out = fq;
    return MSW_OK;
}

void msw_fastq_close(msw_fastq* fq) {
    if (!fq) return;
    if (fq->gz) gzclose(fq->gz);
    if (fq->raw) fclose(fq->raw);
    for (void* inf : fq->inflaters) libdeflate().free_(inf);
    delete fq;
}

int msw_fastq_next(msw_fastq* fq, uint8_t* seqs, uint16_t* lens, uint32_t stride, uint64_t max_reads,
                   uint64_t* n_read, int64_t* pos) {
    if (!fq || !n_read || (max_reads && (!seqs || !lens)))
        return set_error(MSW_E_INVALID, "NULL argument");
    *n_read = 0;
    uint64_t n = 0;
    while (n < max_reads) {
        const char* seq;
        size_t len;
        int64_t p;
        const int rc = next_sequence(fq, &seq, &len, &p, pos != nullptr);
        if (rc < 0) return rc;
        if (rc == 0) break;
        if (len > stride || len > 0xFFFF)
            return set_error(MSW_E_RANGE, "sequence of %zu bases at line %llu exceeds slab stride %u", len,
                             (unsigned long long)fq->lines, stride);
        uint8_t* dst = seqs + n * (uint64_t)stride;
        memcpy(dst, seq, len);
        if (len < stride) memset(dst + len, 0, stride - len);
        lens[n] = (uint16_t)len;
        if (pos) pos[n] = p;
        ++n;
    }
    *n_read = n;
    return MSW_OK;
}

int msw_fastq_next_packed(msw_fastq* fq, uint8_t* buf, uint64_t cap, uint32_t* lens, uint64_t max_reads,
                          uint64_t* n_read, uint64_t* n_bytes, uint64_t* need) {
    if (!fq || !n_read || !n_bytes || (max_reads && (!lens || (cap && !buf))))
        return set_error(MSW_E_INVALID, "NULL argument");
    *n_read = 0;
    *n_bytes = 0;
    if (need) *need = 0;
    uint64_t n = 0, at = 0;
    while (n < max_reads) {
        const char* seq;
        size_t len;
        if (fq->has_held) {
            seq = fq->held.data();
            len = fq->held.size();
        } else {
            int64_t p;
            const int rc = next_sequence(fq, &seq, &len, &p, false);
            if (rc < 0) return rc;
            if (rc == 0) break;
            if (len > 0xFFFFFFFFull)
                return set_error(MSW_E_RANGE, "sequence of %zu bases at line %llu", len,
                                 (unsigned long long)fq->lines);
        }
        if (len > cap - at) {  // delivered by a later call (the caller grows its buffer by *need)
            if (!fq->has_held) {
                fq->held.assign(seq, len);
                fq->has_held = true;
            }
            if (need) *need = len;
            break;
        }
        if (len) memcpy(buf + at, seq, len);
        at += len;
        lens[n++] = (uint32_t)len;
        fq->has_held = false;
    }
    *n_read = n;
    *n_bytes = at;
    return MSW_OK;
}

void msw_fastq_stats(const msw_fastq* fq, uint64_t* lines, uint64_t* reads, uint64_t* errors) {
    if (!fq) return;
    if (lines) *lines = fq->lines;
    if (reads) *reads = fq->reads;
    if (errors) *errors = fq->errors;
}

int msw_fastq_count_bases(const char* path, uint64_t* bases, uint64_t* reads) {
    if (!bases) return set_error(MSW_E_INVALID, "bases is NULL");
    msw_fastq* fq = nullptr;
    int rc = msw_fastq_open(path, &fq);
    if (rc) return rc;
    uint64_t total = 0, nr = 0;
    for (;;) {
        const char* seq;
        size_t len;
        int64_t p;
        rc = next_sequence(fq, &seq, &len, &p, false);
        if (rc < 0) { msw_fastq_close(fq); return rc; }
        if (rc == 0) break;
        total += len;  // Rust String::len = bytes (aligner.rs:540)
        ++nr;
    }
    msw_fastq_close(fq);
    *bases = total;
    if (reads) *reads = nr;
    return MSW_OK;
}

}  // extern "C"
