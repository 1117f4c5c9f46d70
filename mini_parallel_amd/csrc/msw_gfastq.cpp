// msw_gfastq.cpp -- GPU-side BGZF lane reader (include/msw_fastq.h,
// msw_gfastq_* and msw_bgzf_inflate).
//
// Replaces process_fastq_file_in_chunks (smith_waterman/src/aligner.rs:107-178)
// for BGZF lane files: the host only reads compressed bytes and indexes the
// members from their 18-byte headers; everything that touches decompressed
// bytes runs on the GPU (msw_inflate.hip, msw_parse.hip).
//
// One reader = one lane file on one context.  Per span (a few hundred MiB of
// output, thousands of members):
//   host    fread compressed bytes into pinned memory, index whole members
//           (output offsets = running sum of the trailers' ISIZE)
//   stream  H2D of the bytes + member table; inflate (one wave per member);
//           CRC-32 check; the previous span's unfinished line copied in front;
//           parse phase A (line counts) -> host sizes the line arrays ->
//           phase B (line ends, UTF-8 pass if needed, lengths, carried state)
//   emit    per batch of max_reads: sequences into a device slab (two slabs
//           alternate), enqueued on the caller's stream after the parse
// The reader has its own stream, so the next span inflates while the caller's
// scoring of the current batch runs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/msw.h"
#include "../../include/msw_fastq.h"
#include "msw_gz.h"

namespace msw_detail {
int set_error(int code, const char* fmt, ...);
int ctx_device(const msw_ctx* c);
hipStream_t ctx_compute_stream(const msw_ctx* c);
uint64_t ctx_gz_group_bytes(const msw_ctx* c);
}  // namespace msw_detail

using msw_detail::set_error;

namespace {

#define GZ_TRY(expr)                                                                                     \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess)                                                                            \
            return set_error(MSW_E_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                             __LINE__);                                                                  \
    } while (0)

constexpr uint64_t kCarry = 64u << 10;     // room in front of a span for the previous span's last line
constexpr uint64_t kPad = 256;             // device buffers: slack past the end for wide loads
constexpr uint64_t kReadPiece = 8u << 20;  // compressed bytes per fread
constexpr uint64_t kInPad = 1024;          // past the compressed bytes: the inflate input window reads <= 520 B
constexpr uint64_t kDefaultSpan = 1024u << 20;  // ~16k members: two rounds of 8 inflate waves per SIMD

const char* status_text(uint32_t s) {
    switch (s) {
        case msw::GZ_E_BTYPE: return "invalid block type";
        case msw::GZ_E_STORED: return "invalid stored block lengths";
        case msw::GZ_E_HEADER: return "invalid dynamic block header";
        case msw::GZ_E_CODES: return "invalid code lengths set";
        case msw::GZ_E_SYMBOL: return "invalid literal/length or distance code";
        case msw::GZ_E_DIST: return "invalid distance too far back";
        case msw::GZ_E_OVERRUN: return "more data than the member's ISIZE";
        case msw::GZ_E_TRUNC: return "truncated deflate data";
        case msw::GZ_E_SIZE: return "less data than the member's ISIZE";
        case msw::GZ_E_CRC: return "incorrect data check";
        default: return "invalid compressed data";
    }
}

// --- CRC-32 combine constants (zlib crc32.c multmodp / x2nmodp) -------------
uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (uint32_t m = 1u << 31; m; m >>= 1) {
        if (a & m) p ^= b;
        b = b & 1 ? (b >> 1) ^ 0xEDB88320u : b >> 1;
    }
    return p;
}

msw::GzCrcConsts crc_consts() {
    msw::GzCrcConsts c;
    uint32_t p = 1u << 30;  // x^1
    c.x2n[0] = p;
    for (int n = 1; n < 32; ++n) c.x2n[n] = p = multmodp(p, p);
    for (int i = 0; i < 4; ++i)
        for (uint32_t v = 0; v < 256; ++v) c.adv[i][v] = multmodp(c.x2n[11], v << (8 * i));  // x^2048
    return c;
}

// Size of the BGZF member whose 18-byte header is h, or 0 if h is not one.
size_t member_size(const uint8_t* h) {
    if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) return 0;
    const unsigned xlen = h[10] | (h[11] << 8);
    if (xlen != 6 || h[12] != 'B' || h[13] != 'C' || (h[14] | (h[15] << 8)) != 2) return 0;
    return (size_t)(h[16] | (h[17] << 8)) + 1;
}

uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }

// Whole members of buf[0, n) whose output fits in out_cap more bytes and
// whose compressed bytes fit in in_cap: appended to mem (coff relative to buf,
// ooff from out_base).  *used = bytes of those members (<= in_cap: members of
// ISIZE 0, e.g. runs of BGZF EOF blocks, add compressed bytes but no output,
// so the output cap alone does not bound the staging copy).  Returns MSW_OK,
// or MSW_E_INVALID for data that is not BGZF.
int index_members(const uint8_t* buf, size_t n, uint64_t out_base, uint64_t out_cap, size_t in_cap,
                  std::vector<msw::GzMember>& mem, size_t* used, uint64_t* out_bytes) {
    size_t p = 0;
    uint64_t ob = 0;
    while (p + 18 <= n) {
        const size_t sz = member_size(buf + p);
        if (sz < 26) return set_error(MSW_E_INVALID, "not a BGZF block (mixed gzip members are not supported)");
        if (p + sz > n || p + sz > in_cap) break;
        const uint32_t isize = le32(buf + p + sz - 4), crc = le32(buf + p + sz - 8);
        if (isize > 65536) return set_error(MSW_E_INVALID, "BGZF block larger than 64 KiB");
        if (ob + isize > out_cap) break;
        msw::GzMember m;
        m.coff = p + 18;
        m.ooff = out_base + ob;
        m.clen = (uint32_t)(sz - 26);
        m.isize = isize;
        m.crc = crc;
        m.pad = 0;
        mem.push_back(m);
        p += sz;
        ob += isize;
    }
    *used = p;
    *out_bytes = ob;
    return MSW_OK;
}

template <typename T>
int grow(T** p, size_t* cap, size_t n) {
    if (n <= *cap && *p) return MSW_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t want = std::max<size_t>(n, 1) + n / 4;  // headroom against regrowth
    if (hipMalloc((void**)p, want * sizeof(T) + kPad) != hipSuccess)
        return set_error(MSW_E_NOMEM, "hipMalloc(%zu) failed (GPU lane reader)", want * sizeof(T) + kPad);
    *cap = want;
    return MSW_OK;
}

// Device side of inflating one group of members (shared by the reader and msw_bgzf_inflate).
struct Inflater {
    uint8_t* dc = nullptr;                  // compressed bytes
    size_t dc_cap = 0;
    msw::GzMember* d_mem = nullptr;
    size_t mem_cap = 0;
    uint32_t* d_status = nullptr;
    size_t status_cap = 0;
    uint32_t* d_flag = nullptr;             // [0] any error
    msw::GzCrcConsts* d_crc = nullptr;
    uint32_t* h_flag = nullptr;             // pinned
    msw::GzMember* h_mem = nullptr;         // pinned copy of the member table (an async upload)
    size_t h_mem_cap = 0;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};  // MSW_GZ_TIMING

    int init() {
        GZ_TRY(hipMalloc((void**)&d_flag, 64));
        GZ_TRY(hipMalloc((void**)&d_crc, sizeof(msw::GzCrcConsts)));
        const msw::GzCrcConsts c = crc_consts();
        GZ_TRY(hipMemcpy(d_crc, &c, sizeof(c), hipMemcpyHostToDevice));
        GZ_TRY(hipHostMalloc((void**)&h_flag, 64, hipHostMallocDefault));
        return MSW_OK;
    }
    void release() {
        if (dc) (void)hipFree(dc);
        if (d_mem) (void)hipFree(d_mem);
        if (d_status) (void)hipFree(d_status);
        if (d_flag) (void)hipFree(d_flag);
        if (d_crc) (void)hipFree(d_crc);
        if (h_flag) (void)hipHostFree(h_flag);
        if (h_mem) (void)hipHostFree(h_mem);
        h_mem = nullptr;
        h_mem_cap = 0;
        dc = nullptr;
        d_mem = nullptr;
        d_status = nullptr;
        d_flag = nullptr;
        d_crc = nullptr;
        h_flag = nullptr;
    }
    // upload cbytes of compressed data + the member table, inflate into out,
    // check CRCs.  in_place: the device address of h_comp's pinned pages --
    // the kernel then reads the compressed bytes over PCIe as it decodes
    // instead of waiting for a DMA of the whole span first.  pre: a device
    // buffer that already holds h_comp's cbytes (uploaded ahead on s) and
    // kInPad bytes of room after them.
    int run(const uint8_t* h_comp, size_t cbytes, const std::vector<msw::GzMember>& mem, uint8_t* out,
            hipStream_t s, const uint8_t* in_place = nullptr, uint8_t* pre = nullptr) {
        int rc;
        if ((rc = grow(&d_mem, &mem_cap, mem.size()))) return rc;
        if ((rc = grow(&d_status, &status_cap, mem.size()))) return rc;
        if (mem.size() > h_mem_cap) {
            // the previous upload from it finished (callers synchronise s after each run)
            if (h_mem) (void)hipHostFree(h_mem);
            h_mem = nullptr;
            h_mem_cap = 0;
            const size_t want = mem.size() + mem.size() / 4;
            if (hipHostMalloc((void**)&h_mem, want * sizeof(msw::GzMember), hipHostMallocDefault) != hipSuccess) {
                h_mem = nullptr;
                return set_error(MSW_E_NOMEM, "hipHostMalloc failed (GPU inflate member table)");
            }
            h_mem_cap = want;
        }
        const uint8_t* src = in_place;
        size_t src_bytes = cbytes;
        if (!src && pre) {
            GZ_TRY(hipMemsetAsync(pre + cbytes, 0, kInPad, s));
            src = pre;
            src_bytes = cbytes + kInPad;
        }
        if (!src) {
            if ((rc = grow(&dc, &dc_cap, cbytes + kInPad))) return rc;
            if (cbytes) GZ_TRY(hipMemcpyAsync(dc, h_comp, cbytes, hipMemcpyHostToDevice, s));
            GZ_TRY(hipMemsetAsync(dc + cbytes, 0, kInPad, s));
            src = dc;
            src_bytes = cbytes + kInPad;
        }
        if (!mem.empty()) {
            memcpy(h_mem, mem.data(), mem.size() * sizeof(msw::GzMember));
            GZ_TRY(hipMemcpyAsync(d_mem, h_mem, mem.size() * sizeof(msw::GzMember), hipMemcpyHostToDevice, s));
        }
        GZ_TRY(hipMemsetAsync(d_flag, 0, 4, s));
        const uint32_t n = (uint32_t)mem.size();
        static const bool timing = getenv("MSW_GZ_TIMING") != nullptr;  // kernel times to stderr (tools)
        if (timing) {
            if (!ev[0]) {
                GZ_TRY(hipEventCreate(&ev[0]));
                GZ_TRY(hipEventCreate(&ev[1]));
                GZ_TRY(hipEventCreate(&ev[2]));
            }
            GZ_TRY(hipEventRecord(ev[0], s));
        }
        static const bool prof_on = getenv("MSW_GZ_PROFILE") != nullptr;  // MSW_GZ_PROFILE builds: counters
        uint32_t* d_prof = nullptr;
        if (prof_on && n) GZ_TRY(hipMalloc((void**)&d_prof, (size_t)n * 64));
        if (d_prof) GZ_TRY(hipMemsetAsync(d_prof, 0, (size_t)n * 64, s));
        GZ_TRY(msw::launch_gz_inflate(src, src_bytes, d_mem, n, out, d_status, d_flag, s, d_prof));
        if (timing) GZ_TRY(hipEventRecord(ev[1], s));
        if (d_prof) {
            std::vector<uint32_t> h((size_t)n * 16);
            GZ_TRY(hipMemcpyAsync(h.data(), d_prof, h.size() * 4, hipMemcpyDeviceToHost, s));
            GZ_TRY(hipStreamSynchronize(s));
            double sum[12] = {0};
            for (uint32_t m = 0; m < n; ++m)
                for (int i = 0; i < 12; ++i) sum[i] += h[(size_t)m * 16 + i];
            const char* names[12] = {"cycles", "hdr_cycles", "walk_lits", "win_decode_cycles", "scalar_steps",
                                     "windows_emitted", "far_copies", "windows", "near_cycles", "blocks",
                                     "far_cycles", "win_emit_cycles"};
            fprintf(stderr, "[gzprof] per member:");
            for (int i = 0; i < 12; ++i) fprintf(stderr, " %s=%.0f", names[i], sum[i] / n);
            fprintf(stderr, "\n");
            (void)hipFree(d_prof);
        }
        GZ_TRY(msw::launch_gz_crc(out, d_mem, n, d_crc, d_status, d_flag, s));
        if (timing) {
            GZ_TRY(hipEventRecord(ev[2], s));
            GZ_TRY(hipEventSynchronize(ev[2]));
            float a = 0, c = 0;
            (void)hipEventElapsedTime(&a, ev[0], ev[1]);
            (void)hipEventElapsedTime(&c, ev[1], ev[2]);
            uint64_t ob = 0;
            for (const auto& m : mem) ob += m.isize;
            fprintf(stderr, "[gz] %u members, %zu B in, %llu B out: inflate %.3f ms (%.2f GB/s out), crc %.3f ms\n", n,
                    cbytes, (unsigned long long)ob, a, ob / (a * 1e6), c);
        }
        GZ_TRY(hipMemcpyAsync(h_flag, d_flag, 4, hipMemcpyDeviceToHost, s));
        return MSW_OK;
    }
    // after the stream synchronised: error message for the first failing member
    int check(const std::vector<msw::GzMember>& mem, const char* what) {
        if (!h_flag[0]) return MSW_OK;
        std::vector<uint32_t> st(mem.size());
        GZ_TRY(hipMemcpy(st.data(), d_status, st.size() * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < st.size(); ++i)
            if (st[i]) return set_error(MSW_E_INVALID, "Error reading %s: %s (BGZF member %zu of the span)", what,
                                        status_text(st[i]), i);
        return set_error(MSW_E_INVALID, "Error reading %s: invalid compressed data", what);
    }
};

}  // namespace

struct msw_gfastq {
    msw_ctx* ctx = nullptr;
    int device = 0;
    // the reader's switches, read once at msw_gfastq_open (tests set them per reader)
    int read_threads = 4;              // MSW_GZ_READ_THREADS (1..8): threads of a large compressed top-up
    uint64_t in_place_max = 64ull << 20;  // MSW_GZ_IN_PLACE_MB: first spans up to this are inflated in place
    bool no_map = false;               // MSW_GZ_NO_MAP=1: copied mode (preads into pinned staging)
    hipStream_t rs = nullptr;          // the reader's own stream (inflate + parse)
    hipEvent_t parsed = nullptr;       // phase B of the current span done
    // per span buffer i (dout[i] and its line arrays pb[i]): the last emit
    // that read it, on the caller's stream.  A span only waits for the emits
    // of the span two before it, so inflating and parsing the next span (or
    // the next file) runs beside the current span's emits and scoring.
    // The last two emits of each buffer (a caller may alternate two
    // streams: each stream's last emit covers its earlier ones).
    hipEvent_t emitted[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
    bool emitted_valid[2][2] = {{false, false}, {false, false}};
    int emit_slot[2] = {0, 0};
    int last_buf = 1;                  // buffer of the latest span (any file); the next takes the other
    FILE* f = nullptr;
    std::string path;
    uint64_t fsize = 0, fread_off = 0;
    uint32_t stride = 0;
    uint64_t max_reads = 0;
    bool want_pos = false;
    uint64_t span = kDefaultSpan;

    // compressed bytes read but not yet inflated: hc[0, hc_len).  Two ways
    // to get them (msw_fastq.h):
    //  mapped (default): hc points into the file's read-only mapping; the
    //    whole mapping is pinned in place once per file (hipHostRegister) and
    //    each window [reg_lo, fread_off) DMA'd to the GPU from it -- no host
    //    copy, no pinned staging allocation.  A finished file stays pinned
    //    and mapped (retired) until the reader closes or its retired files
    //    pass retire_cap bytes: hipHostUnregister waits for every stream of
    //    the device and, for a lane file's 2.3 GB, holds the other threads'
    //    HIP calls ~24 ms (a pin per window, unpinned per span, held each
    //    worker until the other's scoring drained: DESIGN 5.1);
    //  copied (MSW_GZ_NO_MAP=1, or when mapping / registering fails): preads
    //    into hc_buf, a hipHostMalloc'ed staging buffer allocated on first use.
    uint8_t* hc = nullptr;
    size_t hc_cap = 0, hc_len = 0;
    size_t in_cap = 0;                 // compressed bytes per span, either way
    uint8_t* hc_buf = nullptr;         // copied mode's pinned staging (in_cap bytes)
    bool mapped = false;
    uint8_t* map = nullptr;            // whole-file mapping (mapped mode)
    uint64_t map_off = 0;              // first byte not yet inflated
    uint64_t reg_lo = 0, reg_len = 0;  // the current window of the mapping
    bool reg_all = false;              // the whole mapping is pinned
    // finished files' mappings, pinned (reg) or not, oldest first; unpinned
    // and unmapped on the retire thread once retired_bytes > retire_cap
    struct Retired {
        uint8_t* map;
        size_t len;
        bool reg;
    };
    std::deque<Retired> retired;
    uint64_t retired_bytes = 0, retire_cap = 0;
    std::thread retire;
    // mapped mode: the next span's compressed window [ahead_lo, + ahead_len)
    // of mapping ahead_map, DMA'd into d_ahead on the reader stream as soon
    // as the current span is parsed (upload_ahead), so it crosses PCIe while
    // the current span is scored instead of in front of the next inflate
    uint8_t* d_ahead = nullptr;
    size_t d_ahead_cap = 0;
    // false from a file's open until its first span is in: the prefetch
    // thread pins the next file only then (a 2.3 GB pin beside the first
    // span's upload and inflate stretched that span from ~15 to ~130 ms)
    std::atomic<bool> first_span_in{true};
    const uint8_t* ahead_map = nullptr;
    uint64_t ahead_lo = 0, ahead_len = 0;
    bool reg_failed = false;
    // msw_gfastq_prefetch: the next lane file opened, mapped and its first
    // window pinned by a host thread while this file's spans run; open_file
    // adopts it when the caller resets to that path
    struct Prefetch {
        std::string path;
        FILE* f = nullptr;
        uint64_t fsize = 0, reg_len = 0;  // reg_len: the first window
        uint8_t* map = nullptr;
        bool reg = false;  // the whole mapping pinned
        bool ok = false;
        std::atomic<bool> done{false};  // the thread has finished (ok or not)
        std::atomic<bool> cancel{false};  // drop_prefetch: stop waiting
        // the first span's member index, built on the same thread (the host
        // walk over the window's member headers; its page touches stalled the
        // reader up to ~20 ms beside other threads' pinning)
        std::vector<msw::GzMember> mem;
        size_t used = 0;
        uint64_t obytes = 0;
        bool indexed = false;
        std::thread th;
    } pf;
    // a prefetched file's first span, indexed ahead (open_file adopts it)
    std::vector<msw::GzMember> pre_mem;
    size_t pre_used = 0;
    uint64_t pre_obytes = 0;
    bool pre_indexed = false;
    // read-ahead: while the GPU inflates / the caller scores, a host thread
    // reads the next span's compressed bytes into hc after hc_len
    std::thread filler;
    int fill_rc = 0;
    std::string fill_msg;
    size_t last_used = 0;
    Inflater inf;
    std::vector<msw::GzMember> mem;

    // span buffers: [kCarry | span + kPad]; cur = the parsed one (-1: none yet in this file)
    uint8_t* dout[2] = {nullptr, nullptr};
    int cur = -1;
    uint64_t cur_off = 0, cur_len = 0, tail_start = 0;  // parse window [cur_off, cur_off + cur_len) of dout[cur]
    bool started = false, at_eof = false;

    // parse arrays: tile counts shared (only the reader stream uses them), line
    // arrays per span buffer (the emits read them)
    uint32_t* tile_nl = nullptr;
    uint32_t* tile_hi = nullptr;
    size_t tile_cap = 0, tile_hi_cap = 0;
    msw::ParseBufs pb[2]{};
    size_t line_cap[2] = {0, 0}, vidx_cap[2] = {0, 0}, v_cap[2] = {0, 0}, blk_cap[2] = {0, 0};
    msw::ParseState* d_state = nullptr;
    msw::ParseState* d_state0 = nullptr;  // a file's initial state (copied on the reader stream)
    msw::ParseOut* d_out = nullptr;
    msw::ParseOut* h_out = nullptr;  // pinned
    msw::ParseState* h_state = nullptr;  // pinned
    msw::EmitSpan sp{};

    // batch slabs
    uint8_t* s_reads[2] = {nullptr, nullptr};
    uint16_t* s_rlen[2] = {nullptr, nullptr};
    int64_t* s_pos[2] = {nullptr, nullptr};
    int slot = 0;

    uint64_t span_reads = 0, span_done = 0, next_first = 0;
    uint32_t span_min = 0, span_max = 0;
    uint64_t spans = 0;                     // spans parsed over the reader's life (all files)
    uint64_t bucket_reads = 1;              // reads per span_bmax entry
    uint32_t span_bmax[msw::kLenBuckets] = {};
    int failed = 0;  // sticky error code

    // stats
    uint64_t lines = 0, reads = 0, errors = 0, bases = 0, bytes_in = 0, bytes_out = 0;
};

namespace {

void join_filler(msw_gfastq* g) {
    if (g->filler.joinable()) g->filler.join();
}

// Drop a prefetched file that was not adopted (or join it before adopting).
void join_prefetch(msw_gfastq* g) {
    if (g->pf.th.joinable()) g->pf.th.join();
}

void drop_prefetch(msw_gfastq* g) {
    g->pf.cancel.store(true, std::memory_order_release);
    join_prefetch(g);
    g->pf.cancel.store(false, std::memory_order_relaxed);
    msw_gfastq::Prefetch& p = g->pf;
    if (p.map && g->ahead_map == p.map) {  // its first window may still be uploading
        (void)hipSetDevice(g->device);
        (void)hipStreamSynchronize(g->rs);
        g->ahead_map = nullptr;
        g->ahead_len = 0;
    }
    if (p.reg) (void)hipHostUnregister(p.map);
    if (p.map) munmap(p.map, (size_t)p.fsize);
    if (p.f) fclose(p.f);
    p.f = nullptr;
    p.map = nullptr;
    p.fsize = p.reg_len = 0;
    p.reg = false;
    p.ok = false;
    p.indexed = false;
    p.mem.clear();
    p.path.clear();
}

void unmap_file(msw_gfastq* g);

void join_retire(msw_gfastq* g) {
    if (g->retire.joinable()) g->retire.join();
}

void free_retired(const std::vector<msw_gfastq::Retired>& v, int dev) {
    for (const msw_gfastq::Retired& r : v) {
        if (r.reg && hipSetDevice(dev) == hipSuccess) (void)hipHostUnregister(r.map);
        munmap(r.map, r.len);
    }
}

// every retired file unpinned and unmapped (the reader closes)
void drain_retired(msw_gfastq* g) {
    join_retire(g);
    free_retired(std::vector<msw_gfastq::Retired>(g->retired.begin(), g->retired.end()), g->device);
    g->retired.clear();
    g->retired_bytes = 0;
}

void release(msw_gfastq* g) {
    join_filler(g);
    drop_prefetch(g);
    (void)hipSetDevice(g->device);
    if (g->rs) (void)hipStreamSynchronize(g->rs);
    unmap_file(g);
    drain_retired(g);
    if (g->f) fclose(g->f);
    for (int i = 0; i < 2; ++i) {
        if (g->dout[i]) (void)hipFree(g->dout[i]);
        if (i == 0 && g->d_ahead) (void)hipFree(g->d_ahead);
        if (g->s_reads[i]) (void)hipFree(g->s_reads[i]);
        if (g->s_rlen[i]) (void)hipFree(g->s_rlen[i]);
        if (g->s_pos[i]) (void)hipFree(g->s_pos[i]);
    }
    if (g->tile_nl) (void)hipFree(g->tile_nl);
    if (g->tile_hi) (void)hipFree(g->tile_hi);
    for (msw::ParseBufs& b : g->pb) {
        if (b.line_end) (void)hipFree(b.line_end);
        if (b.vidx) (void)hipFree(b.vidx);
        if (b.vline) (void)hipFree(b.vline);
        if (b.blk) (void)hipFree(b.blk);
    }
    if (g->d_state) (void)hipFree(g->d_state);
    if (g->d_state0) (void)hipFree(g->d_state0);
    if (g->d_out) (void)hipFree(g->d_out);
    if (g->h_out) (void)hipHostFree(g->h_out);
    if (g->h_state) (void)hipHostFree(g->h_state);
    if (g->hc_buf) (void)hipHostFree(g->hc_buf);
    g->inf.release();
    if (g->parsed) (void)hipEventDestroy(g->parsed);
    for (hipEvent_t e : {g->emitted[0][0], g->emitted[0][1], g->emitted[1][0], g->emitted[1][1]})
        if (e) (void)hipEventDestroy(e);
    if (g->rs) (void)hipStreamDestroy(g->rs);
    delete g;
}

// Top up hc with compressed bytes from the file (up to want, within cap).
// Positioned reads (pread at fread_off); a large top-up -- a new file's
// first span, ~180 MB at the config-4 shape -- of 32 MiB or more is split
// over 4 threads (MSW_GZ_READ_THREADS, 1..8): one
// thread copies page-cache data into pinned memory at ~11 GB/s, and 16 ms of
// it per file left the GPU idle between files (MSW_GFASTQ_TRACE).
int fill_compressed(msw_gfastq* g, size_t want) {
    want = std::min(want, g->hc_cap);
    if (want <= g->hc_len || g->fread_off >= g->fsize) return MSW_OK;
    const uint64_t todo = std::min<uint64_t>(want - g->hc_len, g->fsize - g->fread_off);
    const int fd = fileno(g->f);
    auto piece = [fd](uint8_t* dst, uint64_t off, uint64_t len) {
        while (len) {
            const ssize_t r = pread(fd, dst, (size_t)std::min<uint64_t>(len, kReadPiece), (off_t)off);
            if (r <= 0) return false;
            dst += r;
            off += (uint64_t)r;
            len -= (uint64_t)r;
        }
        return true;
    };
    const int threads = g->read_threads;
    const int parts = todo >= (32ull << 20) ? threads : 1;
    const uint64_t per = (todo + parts - 1) / parts;
    bool ok[8] = {true, true, true, true, true, true, true, true};
    std::vector<std::thread> th;
    for (int k = 1; k < parts; ++k) {
        const uint64_t b = per * k, e = std::min<uint64_t>(todo, b + per);
        if (b >= e) continue;
        try {
            th.emplace_back([&, k, b, e]() { ok[k] = piece(g->hc + g->hc_len + b, g->fread_off + b, e - b); });
        } catch (const std::exception&) {  // no thread to spare: read this part here
            ok[k] = piece(g->hc + g->hc_len + b, g->fread_off + b, e - b);
        }
    }
    ok[0] = piece(g->hc + g->hc_len, g->fread_off, std::min<uint64_t>(todo, per));
    for (std::thread& t : th) t.join();
    if (!std::all_of(ok, ok + 8, [](bool b) { return b; }))
        return set_error(MSW_E_INVALID, "Error reading %s: short read", g->path.c_str());
    g->hc_len += (size_t)todo;
    g->fread_off += todo;
    return MSW_OK;
}

// Inflate and parse the next span into dout[next]; sets span_reads (0 is
// possible: a span without a complete sequence line).  Returns MSW_OK with
// at_eof set when the file has no more data.
int fill_compressed(msw_gfastq* g, size_t want);

// Start reading ahead ~one span's compressed bytes (the last span's size; a
// whole staging buffer at the start of a file) in the background; next_span
// joins before it touches hc.
// Mapped mode: the next window of the mapping, [map_off rounded down to a
// page, + in_cap); the first call of a file pins the whole mapping, in the
// background (cached pages register at ~200 GB/s, tools/host_feed.cpp; cold
// ones are read from disk here).
void register_window(msw_gfastq* g) {
    const uint64_t lo = g->map_off & ~(uint64_t)4095;
    const uint64_t hi = std::min<uint64_t>(g->fsize, lo + g->in_cap);
    if (!g->reg_all) {
        if (hipSetDevice(g->device) != hipSuccess ||
            hipHostRegister(g->map, (size_t)g->fsize, hipHostRegisterReadOnly) != hipSuccess) {
            (void)hipGetLastError();
            g->reg_failed = true;  // next_span falls back to copies
            return;
        }
        g->reg_all = true;
    }
    g->reg_lo = lo;
    g->reg_len = hi - lo;
    g->hc = g->map + g->map_off;
    g->hc_len = g->hc_cap = (size_t)(hi - g->map_off);
    g->fread_off = hi;
}

void start_filler(msw_gfastq* g) {
    join_filler(g);
    if (g->mapped) {
        if (g->map_off >= g->fsize || g->reg_len) return;
        try {
            g->filler = std::thread([g]() { register_window(g); });
        } catch (const std::exception&) {
            register_window(g);
        }
        return;
    }
    if (g->fread_off >= g->fsize || g->hc_len >= g->hc_cap) return;
    const size_t want = g->cur < 0 ? g->hc_cap : std::min(g->hc_cap, g->hc_len + g->last_used + kReadPiece);
    g->fill_rc = 0;
    try {
        g->filler = std::thread([g, want]() {
            g->fill_rc = fill_compressed(g, want);
            if (g->fill_rc) g->fill_msg = msw_last_error();  // thread-local: carried to the caller's thread
        });
    } catch (const std::exception&) {
        // no thread to spare: no read-ahead; next_span tops hc up inline
        // (its own fill_compressed loop), so nothing escapes the C ABI
    }
}

// copied mode's pinned staging, allocated on first use
int ensure_stage(msw_gfastq* g) {
    if (!g->hc_buf && hipHostMalloc((void**)&g->hc_buf, g->in_cap, hipHostMallocDefault) != hipSuccess) {
        g->hc_buf = nullptr;
        return set_error(MSW_E_NOMEM, "hipHostMalloc failed (GPU lane reader staging)");
    }
    return MSW_OK;
}

// after the stream drained: retire the file's mapping (see `retired`); the
// oldest retired files past retire_cap are unpinned and unmapped on a thread
// of their own, the caller going on with the next file
void unmap_file(msw_gfastq* g) {
    uint8_t* map = g->map;
    const size_t len = (size_t)g->fsize;
    const bool reg = g->reg_all;
    g->map = nullptr;
    g->mapped = false;
    g->reg_all = false;
    g->reg_lo = g->reg_len = 0;
    if (!map) return;
    g->retired.push_back({map, len, reg});
    g->retired_bytes += len;
    std::vector<msw_gfastq::Retired> out;
    while (g->retired_bytes > g->retire_cap && !g->retired.empty()) {
        out.push_back(g->retired.front());
        g->retired_bytes -= g->retired.front().len;
        g->retired.pop_front();
    }
    if (out.empty()) return;
    join_retire(g);
    const int dev = g->device;
    try {
        g->retire = std::thread([out, dev]() { free_retired(out, dev); });
    } catch (const std::exception&) {
        free_retired(out, dev);
    }
}

// A window could not be pinned: the rest of the file goes through copies.
int to_copied(msw_gfastq* g) {
    const uint64_t off = g->map_off;
    unmap_file(g);
    int rc;
    if ((rc = ensure_stage(g))) return rc;
    g->hc = g->hc_buf;
    g->hc_cap = g->in_cap;
    g->hc_len = 0;
    g->fread_off = off;
    return fill_compressed(g, g->hc_cap);
}

// Mapped mode, after a span is parsed: DMA the next span's window -- this
// file's next window, or after the file's last span the prefetched next
// file's first window -- into d_ahead on the reader stream (see d_ahead).
// Anything not ready (a window still pinning, a prefetch still running)
// is left to next_span's own upload.
void upload_ahead(msw_gfastq* g) {
    g->ahead_map = nullptr;
    g->ahead_len = 0;
    if (!g->d_ahead) return;
    const uint8_t* map = nullptr;
    uint64_t lo = 0, len = 0;
    if (g->mapped && !g->at_eof) {
        join_filler(g);
        if (g->fill_rc || g->reg_failed || !g->reg_all) return;
        if (!g->reg_len && g->map_off < g->fsize) register_window(g);
        if (!g->reg_len || g->reg_failed) return;
        map = g->map;
        lo = g->reg_lo;
        len = g->reg_len;
    } else if (g->at_eof && g->pf.done.load(std::memory_order_acquire)) {
        join_prefetch(g);  // finished: no wait
        if (!g->pf.ok || !g->pf.reg) return;
        map = g->pf.map;
        len = g->pf.reg_len;
    } else {
        return;
    }
    if (len + kInPad > g->d_ahead_cap) return;
    if (hipMemcpyAsync(g->d_ahead, map + lo, len, hipMemcpyHostToDevice, g->rs) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    g->ahead_map = map;
    g->ahead_lo = lo;
    g->ahead_len = len;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int next_span(msw_gfastq* g) {
    int rc;
    static const bool trace = getenv("MSW_GFASTQ_TRACE") != nullptr;
    const double t0 = trace ? now_ms() : 0.0;
    const int nx = 1 - g->last_buf;
    join_filler(g);
    const double t_join = trace ? now_ms() : 0.0;
    if (g->fill_rc) return set_error(g->fill_rc, "%s", g->fill_msg.c_str());
    if (g->mapped && g->reg_failed && (rc = to_copied(g))) return rc;
    if (g->mapped && !g->reg_len && g->map_off < g->fsize) register_window(g);  // no read-ahead ran
    if (g->mapped && g->reg_failed && (rc = to_copied(g))) return rc;
    const double t_reg = trace ? now_ms() : 0.0;
    // A lane file must not change while it is read (the mapping is
    // MAP_SHARED: touching pages past a truncation raises SIGBUS).  Checked
    // before the host parses this span's member headers, so a file truncated
    // between spans is an error instead of a signal.
    if (g->mapped) {
        struct stat sb;
        if (fstat(fileno(g->f), &sb) != 0 || (uint64_t)sb.st_size < g->fsize)
            return set_error(MSW_E_INVALID, "Error reading %s: the file shrank while it was being read",
                             g->path.c_str());
    }
    // 1. whole members whose output fits the span (compressed <= span bytes + 1 MiB)
    g->mem.clear();
    size_t used = 0;
    uint64_t obytes = 0;
    // Every span is full size: a shorter first span (scoring starts sooner)
    // measured slower -- 256 MB first spans 99-102 vs 104-105 M reads/s over
    // 16 files, 67-69 vs 76 M over 2 files (profiles/r03/e2e/first_span_ab.jsonl):
    // fewer members per inflate launch cost more than the earlier start wins.
    const uint64_t cap = g->span;
    if (g->pre_indexed) {  // a prefetched file's first span: indexed on the prefetch thread
        g->mem.swap(g->pre_mem);
        used = g->pre_used;
        obytes = g->pre_obytes;
        g->pre_indexed = false;
    } else {
        for (;;) {
            if ((rc = index_members(g->hc, g->hc_len, kCarry, cap, g->in_cap, g->mem, &used, &obytes))) return rc;
            const bool full = obytes + 65536 > cap || g->fread_off >= g->fsize || g->hc_len == g->hc_cap;
            if (full) break;
            g->mem.clear();
            if ((rc = fill_compressed(g, g->hc_len + kReadPiece))) return rc;
        }
    }
    const bool last = g->fread_off >= g->fsize && used == g->hc_len;
    if (g->mem.empty() && !last) {
        if (g->hc_len - used >= 18 && member_size(g->hc + used) > g->hc_cap)
            return set_error(MSW_E_INVALID, "Error reading %s: BGZF member larger than the staging buffer",
                             g->path.c_str());
    }
    if (g->fread_off >= g->fsize && used < g->hc_len && g->mem.empty())
        return set_error(MSW_E_INVALID, "Error reading %s: unexpected end of file", g->path.c_str());

    const double t_read = trace ? now_ms() : 0.0;
    hipStream_t s = g->rs;
    // dout[nx] and its line arrays were last read by the emits of the span
    // before the current one (long finished, normally); the current span's
    // emits and the caller's scoring keep running
    for (int j = 0; j < 2; ++j)
        if (g->emitted_valid[nx][j]) GZ_TRY(hipStreamWaitEvent(s, g->emitted[nx][j], 0));
    // 2. inflate + CRC into dout[nx] at kCarry (mapped: the upload starts at
    // the page boundary below hc, inside the registered window)
    const size_t lead = g->mapped ? (size_t)(g->map_off - g->reg_lo) : 0;
    if (lead)
        for (msw::GzMember& m : g->mem) m.coff += lead;
    // A file's first span, when small (<= MSW_GZ_IN_PLACE_MB compressed, 64 by
    // default: config 3's 46 MB lane files), is read by the inflate kernel in
    // place from the pinned window: nothing of this file is in flight yet to
    // hide its upload behind, and the DMA of the whole span (~0.8 ms per
    // 46 MB, two lanes sharing the link) would come first.  Later spans and
    // large ones are uploaded (their DMA overlaps the previous span's work,
    // and PCIe reads at decode time would slow inflate on a saturated link).
    uint8_t* pre = nullptr;
    if (g->mapped && g->ahead_map && g->ahead_map == g->map && g->ahead_lo == g->reg_lo &&
        used + lead <= g->ahead_len)
        pre = g->d_ahead;
    g->ahead_map = nullptr;  // used now, or stale
    const uint8_t* in_place = nullptr;
    if (!pre && g->mapped && g->reg_len && g->cur < 0 && used + lead <= g->in_place_max) {
        void* dp = nullptr;
        if (hipHostGetDevicePointer(&dp, (void*)(g->hc - lead), 0) == hipSuccess && dp)
            in_place = (const uint8_t*)dp;
        else
            (void)hipGetLastError();
    }
    if ((rc = g->inf.run(g->hc - lead, used + lead, g->mem, g->dout[nx], s, in_place, pre))) return rc;
    const double t_run = trace ? now_ms() : 0.0;
    // 3. the previous span's unfinished line goes right in front
    const uint64_t carry = g->cur < 0 ? 0 : g->cur_len - g->tail_start;
    if (carry > kCarry)
        return set_error(MSW_E_RANGE, "Error reading %s: a line longer than %llu bytes", g->path.c_str(),
                         (unsigned long long)kCarry);
    if (carry)
        GZ_TRY(hipMemcpyAsync(g->dout[nx] + kCarry - carry, g->dout[g->cur] + g->cur_off + g->tail_start, carry,
                              hipMemcpyDeviceToDevice, s));
    // 4. parse phase A over [kCarry - carry, kCarry + obytes), from a 16-byte aligned base
    msw::ParseBufs& b = g->pb[nx];
    const uint64_t base = (kCarry - carry) & ~(uint64_t)15;
    b.buf = g->dout[nx] + base;
    b.begin = (uint32_t)(kCarry - carry - base);
    b.len = kCarry + obytes - base;
    b.eof = last ? 1u : 0u;
    b.want_pos = g->want_pos ? 1u : 0u;
    b.ntiles = (uint32_t)((b.len + msw::kParseTile - 1) / msw::kParseTile);
    if ((rc = grow(&g->tile_nl, &g->tile_cap, (size_t)b.ntiles + 1))) return rc;
    if ((rc = grow(&g->tile_hi, &g->tile_hi_cap, (size_t)b.ntiles + 1))) return rc;
    b.tile_nl = g->tile_nl;
    b.tile_hi = g->tile_hi;
    b.line_cap = ~0ull;
    b.state = g->d_state;
    b.out = g->d_out;
    b.stride = g->stride;
    GZ_TRY(msw::launch_parse_a(b, s));
    GZ_TRY(hipMemcpyAsync(g->h_out, g->d_out, sizeof(msw::ParseOut), hipMemcpyDeviceToHost, s));
    GZ_TRY(hipStreamSynchronize(s));
    const double t_a = trace ? now_ms() : 0.0;
    if (lead)  // uploads done: the member table holds offsets into hc again
        for (msw::GzMember& m : g->mem) m.coff -= lead;
    if ((rc = g->inf.check(g->mem, g->path.c_str()))) return rc;
    // the upload of hc has completed: drop the consumed bytes and read ahead
    if (g->mapped) {
        // the window's upload is done (the mapping stays pinned until the file closes)
        g->reg_len = 0;
        g->map_off += used;
        g->hc_len = 0;
    } else if (used) {
        memmove(g->hc, g->hc + used, g->hc_len - used);
        g->hc_len -= used;
    }
    g->last_used = used;
    start_filler(g);
    const double t_unpin = trace ? now_ms() : 0.0;
    const uint64_t nlines = g->h_out->lines;
    const bool any_high = g->h_out->any_high != 0;
    // 5. size the line arrays, phase B
    if ((rc = grow(&b.line_end, &g->line_cap[nx], (size_t)nlines + 1))) return rc;
    b.line_cap = g->line_cap[nx];
    if (any_high) {
        if ((rc = grow(&b.vidx, &g->vidx_cap[nx], (size_t)nlines + 1))) return rc;
        if ((rc = grow(&b.vline, &g->v_cap[nx], (size_t)nlines + 1))) return rc;
        if ((rc = grow(&b.blk, &g->blk_cap[nx], (size_t)(nlines / 1024 + 2)))) return rc;
    }
    // read-length maxima per run of whole batches (<= kLenBuckets runs)
    {
        const uint64_t batches = (nlines / 4 + 1 + g->max_reads - 1) / g->max_reads;
        b.bucket_reads = g->max_reads * ((batches + msw::kLenBuckets - 1) / msw::kLenBuckets);
    }
    GZ_TRY(msw::launch_parse_b(b, nlines, any_high, s));
    GZ_TRY(hipMemcpyAsync(g->h_out, g->d_out, sizeof(msw::ParseOut), hipMemcpyDeviceToHost, s));
    GZ_TRY(hipEventRecord(g->parsed, s));
    GZ_TRY(hipStreamSynchronize(s));
    const msw::ParseOut& o = *g->h_out;
    if (trace)
        fprintf(stderr, "[gfastq] %s span: %zu members, %.1f MB in, %.1f MB out: read+index %.2f ms "
                        "(read-ahead join %.2f, window pin %.2f, index %.2f), "
                        "inflate+parse A %.2f ms (host calls %.2f, %s), parse B %.2f ms (read-ahead start %.2f), "
                        "%llu reads\n",
                g->path.c_str(), g->mem.size(), used / 1e6, obytes / 1e6, t_read - t0, t_join - t0, t_reg - t_join,
                t_read - t_reg, t_a - t_read, t_run - t_read, pre ? "uploaded ahead" : (in_place ? "in place" : "upload"),
                now_ms() - t_a, t_unpin - t_a, (unsigned long long)o.reads);
    if (o.err_over)
        return set_error(MSW_E_INVALID, "Too many read errors (>10), stopping at line %llu",
                         (unsigned long long)o.err_line);
    if (o.too_long)
        return set_error(MSW_E_RANGE, "sequence longer than the slab stride %u at line %llu", g->stride,
                         (unsigned long long)o.too_long_line);
    g->bytes_in += used;
    g->bytes_out += obytes;
    g->cur = nx;
    g->last_buf = nx;
    g->cur_off = base;
    g->cur_len = b.len;
    g->tail_start = o.tail_start;
    g->started = true;
    g->at_eof = last;
    g->span_reads = o.reads;
    g->span_done = 0;
    ++g->spans;
    g->span_min = o.min_len;
    g->span_max = o.max_len;
    g->bucket_reads = b.bucket_reads;
    memcpy(g->span_bmax, o.bmax, sizeof(g->span_bmax));
    g->sp.v0 = o.v0;
    g->sp.pending_in = o.pending_in;
    g->sp.any_high = o.any_high;
    g->lines += o.valid;
    g->errors += o.lines - o.valid;
    g->reads += o.reads;
    g->bases += o.bases;
    upload_ahead(g);
    g->first_span_in.store(true, std::memory_order_release);
    return MSW_OK;
}

// Point the reader at a (new) lane file: per-file state back to the start,
// buffers kept.  The parse state goes back to line 0 on the reader stream.
int open_file(msw_gfastq* g, const char* path) {
    join_filler(g);
    join_prefetch(g);
    if (g->mapped || g->map) {
        // the previous file's last window may still be uploading
        GZ_TRY(hipSetDevice(g->device));
        GZ_TRY(hipStreamSynchronize(g->rs));
        unmap_file(g);
    }
    if (g->f) fclose(g->f);
    g->f = nullptr;
    g->path = path;
    g->fsize = g->fread_off = 0;
    g->hc_len = 0;
    g->hc = g->hc_buf;
    g->hc_cap = g->hc_buf ? g->in_cap : 0;
    g->map_off = g->reg_lo = g->reg_len = 0;
    g->reg_failed = false;
    g->cur = -1;
    g->cur_off = g->cur_len = g->tail_start = 0;
    g->started = g->at_eof = false;
    g->span_reads = g->span_done = g->next_first = 0;
    g->failed = 0;
    g->fill_rc = 0;
    g->last_used = 0;
    g->lines = g->reads = g->errors = g->bases = g->bytes_in = g->bytes_out = 0;
    g->pre_indexed = false;
    g->first_span_in.store(false, std::memory_order_release);
    if (g->pf.ok && g->pf.path == path) {
        // prefetched (msw_gfastq_prefetch): file open, mapped and pinned, the
        // first window [0, reg_len) -- the state register_window leaves behind
        msw_gfastq::Prefetch& p = g->pf;
        g->f = p.f;
        g->fsize = p.fsize;
        g->map = p.map;
        g->mapped = true;
        g->reg_all = p.reg;
        g->map_off = g->reg_lo = 0;
        g->reg_len = p.reg_len;
        g->hc = g->map;
        g->hc_len = g->hc_cap = (size_t)p.reg_len;
        g->fread_off = p.reg_len;
        if (p.indexed) {
            g->pre_mem.swap(p.mem);
            g->pre_used = p.used;
            g->pre_obytes = p.obytes;
            g->pre_indexed = true;
        }
        p.f = nullptr;
        p.map = nullptr;
        p.fsize = p.reg_len = 0;
        p.reg = false;
        p.ok = false;
        p.indexed = false;
        p.mem.clear();
        p.path.clear();
        if (g->d_state) {
            GZ_TRY(hipSetDevice(g->device));
            GZ_TRY(hipMemcpyAsync(g->d_state, g->d_state0, sizeof(msw::ParseState), hipMemcpyDeviceToDevice, g->rs));
        }
        return MSW_OK;
    }
    drop_prefetch(g);  // prefetched another path: not needed
    g->f = fopen(path, "rb");
    if (!g->f) return set_error(MSW_E_INVALID, "Failed to open file %s", path);
    fseeko(g->f, 0, SEEK_END);
    g->fsize = (uint64_t)ftello(g->f);
    fseeko(g->f, 0, SEEK_SET);
    setvbuf(g->f, nullptr, _IONBF, 0);
    if (g->fsize >= 18) {
        uint8_t h[18];
        if (fread(h, 1, 18, g->f) != 18 || member_size(h) < 26)
            return set_error(MSW_E_INVALID, "%s is not a BGZF file", path);
        fseeko(g->f, 0, SEEK_SET);
    } else if (g->fsize > 0) {
        return set_error(MSW_E_INVALID, "%s is not a BGZF file", path);
    }
    if (g->d_state) {
        // back to line 0, in order on the reader stream (the emits never read
        // the state); the previous file's batches stay valid on the caller's stream
        GZ_TRY(hipSetDevice(g->device));
        GZ_TRY(hipMemcpyAsync(g->d_state, g->d_state0, sizeof(msw::ParseState), hipMemcpyDeviceToDevice, g->rs));
    }
    if (!g->no_map && g->fsize > 0) {
        void* m = mmap(nullptr, (size_t)g->fsize, PROT_READ, MAP_SHARED, fileno(g->f), 0);
        if (m != MAP_FAILED) {
            g->map = (uint8_t*)m;
            g->mapped = true;
            (void)madvise(m, (size_t)g->fsize, MADV_SEQUENTIAL);
        }
    }
    if (!g->mapped && g->fsize > 0) {
        int rc;
        if ((rc = ensure_stage(g))) return rc;
        g->hc = g->hc_buf;
        g->hc_cap = g->in_cap;
    }
    start_filler(g);  // the first span's compressed bytes, read while the caller finishes the last file
    return MSW_OK;
}

}  // namespace

extern "C" {

int msw_is_bgzf(const char* path) {
    FILE* f = path ? fopen(path, "rb") : nullptr;
    if (!f) return 0;
    uint8_t h[18];
    const bool yes = fread(h, 1, 18, f) == 18 && member_size(h) >= 26;
    fclose(f);
    return yes ? 1 : 0;
}

int msw_gfastq_open(msw_ctx* ctx, const char* path, uint32_t read_stride, uint64_t max_reads, int want_pos,
                    uint64_t span_bytes, msw_gfastq** out) {
    if (!ctx || !out) return set_error(MSW_E_INVALID, "ctx/out is NULL");
    *out = nullptr;
    if (read_stride == 0 || read_stride % 16 || read_stride > 32768)
        return set_error(MSW_E_INVALID, "read_stride %u must be a multiple of 16 in [16, 32768]", read_stride);
    if (max_reads == 0) return set_error(MSW_E_INVALID, "max_reads is 0");
    msw_gfastq* g = new msw_gfastq();
    g->ctx = ctx;
    g->device = msw_detail::ctx_device(ctx);
    g->path = path ? path : "";
    g->stride = read_stride;
    g->max_reads = max_reads;
    g->want_pos = want_pos != 0;
    {
        const char* et = getenv("MSW_GZ_READ_THREADS");
        g->read_threads = std::max(1, std::min(8, et ? atoi(et) : 4));
        const char* eip = getenv("MSW_GZ_IN_PLACE_MB");
        if (eip) g->in_place_max = strtoull(eip, nullptr, 10) << 20;
        const char* nm = getenv("MSW_GZ_NO_MAP");
        g->no_map = nm && atoi(nm) != 0;
        // finished files kept pinned: MSW_GZ_RETIRE_MB, default min(32 GiB, RAM / 8)
        const char* er = getenv("MSW_GZ_RETIRE_MB");
        const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
        const uint64_t ram = pages > 0 && psz > 0 ? (uint64_t)pages * (uint64_t)psz : (64ull << 30);
        g->retire_cap = er ? strtoull(er, nullptr, 10) << 20 : std::min<uint64_t>(32ull << 30, ram / 8);
    }
    if (span_bytes == 0) {
        const char* e = getenv("MSW_GFASTQ_SPAN_MB");
        span_bytes = e && atoll(e) > 0 ? (uint64_t)atoll(e) << 20 : kDefaultSpan;
    }
    g->span = std::max<uint64_t>(span_bytes, 1u << 20);
    if (g->span > (2ull << 30)) g->span = 2ull << 30;  // 32-bit line offsets
    auto bail = [&](int rc) {
        release(g);
        return rc;
    };
    if (hipSetDevice(g->device) != hipSuccess) return bail(set_error(MSW_E_DEVICE, "hipSetDevice failed"));
    int rc;
    if ((rc = g->inf.init())) return bail(rc);
    // The reader's stream gets a hardware queue of its own: a stream with a
    // CU mask (here all CUs) is not placed on one of the GPU_MAX_HW_QUEUES
    // queues that plain streams share, where the --full-wgs traces showed one
    // worker's inflate and parse kernels queued with a scoring stream
    // (DESIGN.md 6.2).  A CU-masked stream is a blocking stream (ordered with
    // the null stream); the fallback, when the masked one cannot be made, is
    // a blocking stream too, so the reader's ordering is the same either way:
    // work a caller puts on the null stream (hipMemcpy, PyTorch's default
    // stream) serialises with inflate and parse -- score on a stream of your
    // own to overlap them (fastq.GpuFastqReader).
    {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, g->device) != hipSuccess || ncu <= 0)
            ncu = 256;
        std::vector<uint32_t> mask(((size_t)ncu + 31) / 32, 0xFFFFFFFFu);
        if (ncu % 32) mask.back() = (1u << (ncu % 32)) - 1u;
        if (hipExtStreamCreateWithCUMask(&g->rs, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
            (void)hipGetLastError();
            g->rs = nullptr;
        }
    }
    if ((!g->rs && hipStreamCreateWithFlags(&g->rs, hipStreamDefault) != hipSuccess) ||
        hipEventCreateWithFlags(&g->parsed, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->emitted[0][0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->emitted[0][1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->emitted[1][0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->emitted[1][1], hipEventDisableTiming) != hipSuccess)
        return bail(set_error(MSW_E_DEVICE, "stream/event creation failed"));
    // the reader's kernels' code objects, loaded with the reader instead of
    // at the first span (two workers' first launches each waited ~80 ms there)
    if (msw::gz_preload() != hipSuccess || msw::parse_preload() != hipSuccess)
        return bail(set_error(MSW_E_DEVICE, "GPU lane reader: kernel load failed"));
    // compressed staging: half a span (FASTQ compresses ~3-4x; less
    // compressible data just makes shorter spans) + room for one fread piece
    g->in_cap = (size_t)(std::max<uint64_t>(g->span / 2, 16u << 20) + kReadPiece + (1u << 20));
    if (hipHostMalloc((void**)&g->h_out, sizeof(msw::ParseOut), hipHostMallocDefault) != hipSuccess)
        return bail(set_error(MSW_E_NOMEM, "hipHostMalloc failed (GPU lane reader staging)"));
    {
        // copied mode asked for up front: its pinned staging now, with the
        // other buffers (~85 ms per 512 MB), not at the first file's read
        if (g->no_map && (rc = ensure_stage(g))) return bail(rc);
    }
    const size_t ob = (size_t)(kCarry + g->span + kPad);
    for (int i = 0; i < 2; ++i) {
        if (hipMalloc((void**)&g->dout[i], ob) != hipSuccess ||
            hipMalloc((void**)&g->s_reads[i], (size_t)max_reads * read_stride + kPad) != hipSuccess ||
            hipMalloc((void**)&g->s_rlen[i], (size_t)max_reads * 2 + kPad) != hipSuccess ||
            (g->want_pos && hipMalloc((void**)&g->s_pos[i], (size_t)max_reads * 8 + kPad) != hipSuccess))
            return bail(set_error(MSW_E_NOMEM, "hipMalloc failed (GPU lane reader buffers, span %llu MiB)",
                                  (unsigned long long)(g->span >> 20)));
    }
    // Every device buffer a span needs, sized for a full span now (setup), so
    // no hipMalloc runs between a file's first inflate and its first batch:
    // in a short run (config 3 from FASTQ: one file per worker) those
    // first-use allocations sat on the critical path, 2-4 ms each, and the
    // workers' allocations serialised (profiles/r05/c3f/).  Line arrays
    // assume lines of >= 32 bytes on average (FASTQ of 150 bp reads: ~90);
    // a span with more lines still grows them.
    {
        const size_t lines = (size_t)(g->span / 32) + 1024;
        const size_t members = (size_t)(g->span / 32768) + 1024;  // BGZF members hold <= 64 KiB
        const size_t tiles = (size_t)((kCarry + g->span + 16 + msw::kParseTile - 1) / msw::kParseTile) + 1;
        if (!g->no_map) {
            g->d_ahead_cap = g->in_cap + 4096 + kInPad;
            if (hipMalloc((void**)&g->d_ahead, g->d_ahead_cap) != hipSuccess) {
                (void)hipGetLastError();
                g->d_ahead = nullptr;  // no upload ahead: each span uploads in front of its inflate
                g->d_ahead_cap = 0;
            }
        }
        if (hipHostMalloc((void**)&g->inf.h_mem, members * sizeof(msw::GzMember), hipHostMallocDefault) != hipSuccess)
            return bail(set_error(MSW_E_NOMEM, "hipHostMalloc failed (GPU lane reader member table)"));
        g->inf.h_mem_cap = members;
        if ((rc = grow(&g->inf.dc, &g->inf.dc_cap, g->in_cap + 4096 + kInPad)) ||
            (rc = grow(&g->inf.d_mem, &g->inf.mem_cap, members)) ||
            (rc = grow(&g->inf.d_status, &g->inf.status_cap, members)) ||
            (rc = grow(&g->tile_nl, &g->tile_cap, tiles)) || (rc = grow(&g->tile_hi, &g->tile_hi_cap, tiles)) ||
            (rc = grow(&g->pb[0].line_end, &g->line_cap[0], lines)) ||
            (rc = grow(&g->pb[1].line_end, &g->line_cap[1], lines)))
            return bail(rc);
    }
    if (hipMalloc((void**)&g->d_state, sizeof(msw::ParseState)) != hipSuccess ||
        hipMalloc((void**)&g->d_state0, sizeof(msw::ParseState)) != hipSuccess ||
        hipMalloc((void**)&g->d_out, sizeof(msw::ParseOut)) != hipSuccess ||
        hipHostMalloc((void**)&g->h_state, sizeof(msw::ParseState), hipHostMallocDefault) != hipSuccess)
        return bail(set_error(MSW_E_NOMEM, "hipMalloc failed (GPU lane reader state)"));
    *g->h_state = msw::ParseState{0, 0, -1, 0};
    if (hipMemcpy(g->d_state0, g->h_state, sizeof(msw::ParseState), hipMemcpyHostToDevice) != hipSuccess)
        return bail(set_error(MSW_E_DEVICE, "hipMemcpy failed (GPU lane reader state)"));
    if (path && (rc = open_file(g, path))) return bail(rc);
    if (!path) g->failed = MSW_E_INVALID;  // buffers only: msw_gfastq_reset names the first file
    *out = g;
    return MSW_OK;
}

int msw_gfastq_reset(msw_gfastq* g, const char* path) {
    if (!g || !path) return set_error(MSW_E_INVALID, "reader/path is NULL");
    const int rc = open_file(g, path);
    if (rc) g->failed = rc;
    return rc;
}

int msw_gfastq_prefetch(msw_gfastq* g, const char* path) {
    if (!g || !path) return set_error(MSW_E_INVALID, "reader/path is NULL");
    drop_prefetch(g);
    if (g->no_map) return MSW_OK;  // copied mode: nothing to pin ahead
    g->pf.path = path;
    g->pf.done.store(false, std::memory_order_relaxed);
    const size_t cap = g->in_cap;
    const uint64_t span = g->span;
    const int device = g->device;
    msw_gfastq::Prefetch* p = &g->pf;
    std::atomic<bool>* gate = &g->first_span_in;
    try {
        p->th = std::thread([p, cap, span, device, gate]() {
            struct Done {
                std::atomic<bool>& d;
                ~Done() { d.store(true, std::memory_order_release); }
            } done{p->done};
            // any failure leaves ok = false: reset then opens the file the usual way
            p->f = fopen(p->path.c_str(), "rb");
            if (!p->f) return;
            if (fseeko(p->f, 0, SEEK_END) != 0) return;
            p->fsize = (uint64_t)ftello(p->f);
            fseeko(p->f, 0, SEEK_SET);
            setvbuf(p->f, nullptr, _IONBF, 0);
            uint8_t h[18];
            if (p->fsize < 18 || fread(h, 1, 18, p->f) != 18 || member_size(h) < 26) return;
            fseeko(p->f, 0, SEEK_SET);
            void* m = mmap(nullptr, (size_t)p->fsize, PROT_READ, MAP_SHARED, fileno(p->f), 0);
            if (m == MAP_FAILED) return;
            p->map = (uint8_t*)m;
            (void)madvise(m, (size_t)p->fsize, MADV_SEQUENTIAL);
            const uint64_t hi = std::min<uint64_t>(p->fsize, cap);
            // pin once the current file's first span is in (bounded wait)
            for (int i = 0; i < 20000 && !gate->load(std::memory_order_acquire); ++i) {
                if (p->cancel.load(std::memory_order_acquire)) return;
                usleep(250);
            }
            if (p->cancel.load(std::memory_order_acquire)) return;
            if (hipSetDevice(device) != hipSuccess ||
                hipHostRegister(p->map, (size_t)p->fsize, hipHostRegisterReadOnly) != hipSuccess) {
                (void)hipGetLastError();
                return;
            }
            p->reg = true;
            p->reg_len = hi;
            p->ok = true;
            // the first span's members, as next_span would index them for a
            // fresh file (hc = the window, full on the first pass); an error
            // leaves it to next_span, which reports it
            p->mem.clear();
            p->indexed = index_members(p->map, (size_t)hi, kCarry, span, cap, p->mem, &p->used, &p->obytes) == 0;
        });
    } catch (const std::exception&) {
        g->pf.path.clear();  // no thread to spare: reset opens it then
    }
    return MSW_OK;
}

int msw_gfastq_next(msw_gfastq* g, void* stream, msw_dev_reads_t* out) {
    if (!g || !out) return set_error(MSW_E_INVALID, "reader/out is NULL");
    memset(out, 0, sizeof(*out));
    out->read_stride = g->stride;
    if (g->failed)
        return set_error(g->failed, g->path.empty() ? "GPU lane reader: no file (msw_gfastq_reset first)"
                                                    : "Error reading %s: the reader failed earlier",
                         g->path.c_str());
    if (hipSetDevice(g->device) != hipSuccess) return set_error(MSW_E_DEVICE, "hipSetDevice failed");
    hipStream_t cs = stream ? (hipStream_t)stream : msw_detail::ctx_compute_stream(g->ctx);
    while (g->span_done == g->span_reads) {
        if (g->started && g->at_eof) {
            out->first_read = g->next_first;
            return MSW_OK;  // n = 0: end of file
        }
        const int rc = next_span(g);
        if (rc) {
            g->failed = rc;
            return rc;
        }
    }
    const uint64_t n = std::min<uint64_t>(g->max_reads, g->span_reads - g->span_done);
    const int k = g->slot;
    g->slot ^= 1;
    GZ_TRY(hipStreamWaitEvent(cs, g->parsed, 0));
    GZ_TRY(msw::launch_emit_reads(g->pb[g->cur], g->sp, g->span_done, n, g->s_reads[k], g->s_rlen[k],
                                  g->want_pos ? g->s_pos[k] : nullptr, cs));
    {
        const int j = g->emit_slot[g->cur];
        g->emit_slot[g->cur] ^= 1;
        GZ_TRY(hipEventRecord(g->emitted[g->cur][j], cs));
        g->emitted_valid[g->cur][j] = true;
    }
    out->reads = g->s_reads[k];
    out->read_len = g->s_rlen[k];
    out->pos = g->want_pos ? g->s_pos[k] : nullptr;
    out->n = n;
    out->first_read = g->next_first;
    out->min_len = g->span_min;
    // the batch's own longest read (its run of the span), not the span's
    out->max_len = g->span_bmax[std::min<uint64_t>(g->span_done / g->bucket_reads, msw::kLenBuckets - 1)];
    g->span_done += n;
    g->next_first += n;
    return MSW_OK;
}

void msw_gfastq_stats(const msw_gfastq* g, uint64_t* lines, uint64_t* reads, uint64_t* errors, uint64_t* bases,
                      uint64_t* bytes_in, uint64_t* bytes_out) {
    if (!g) return;
    if (lines) *lines = g->lines;
    if (reads) *reads = g->reads;
    if (errors) *errors = g->errors;
    if (bases) *bases = g->bases;
    if (bytes_in) *bytes_in = g->bytes_in;
    if (bytes_out) *bytes_out = g->bytes_out;
}

void msw_gfastq_close(msw_gfastq* g) {
    if (g) release(g);
}

int msw_bgzf_inflate(msw_ctx* ctx, const uint8_t* data, uint64_t len, uint8_t* out, uint64_t cap,
                     uint64_t* out_len) {
    if (!ctx || (!data && len) || !out_len) return set_error(MSW_E_INVALID, "ctx/data/out_len is NULL");
    *out_len = 0;
    GZ_TRY(hipSetDevice(msw_detail::ctx_device(ctx)));
    hipStream_t s = msw_detail::ctx_compute_stream(ctx);
    Inflater inf;
    int rc = inf.init();
    uint8_t* dout = nullptr;
    uint8_t* hstage = nullptr;
    // output bytes per launch, MSW_GZ_GROUP_MB (default 1024: ~16k members,
    // two waves per SIMD slot), read at context creation
    const uint64_t kGroup = msw_detail::ctx_gz_group_bytes(ctx);
    const size_t kStage = (size_t)(kGroup + kGroup / 8 + (4u << 20));  // pinned staging: a group's compressed bytes
    uint64_t p = 0, total = 0;
    std::vector<msw::GzMember> mem;
    while (!rc && p < len) {
        mem.clear();
        size_t used = 0;
        uint64_t ob = 0;
        rc = index_members(data + p, (size_t)(len - p), 0, kGroup, kStage, mem, &used, &ob);
        if (rc) break;
        if (mem.empty()) {
            rc = set_error(MSW_E_INVALID, "unexpected end of file");
            break;
        }
        if (total + ob > cap) {
            rc = set_error(MSW_E_RANGE, "output buffer of %llu bytes is too small", (unsigned long long)cap);
            break;
        }
        if (!dout && hipMalloc((void**)&dout, kGroup + kPad) != hipSuccess) {
            rc = set_error(MSW_E_NOMEM, "hipMalloc failed");
            break;
        }
        if (!hstage && hipHostMalloc((void**)&hstage, kStage) != hipSuccess) {
            rc = set_error(MSW_E_NOMEM, "hipHostMalloc failed");
            break;
        }
        memcpy(hstage, data + p, used);
        if ((rc = inf.run(hstage, used, mem, dout, s))) break;
        if (hipStreamSynchronize(s) != hipSuccess) {
            rc = set_error(MSW_E_DEVICE, "inflate launch failed");
            break;
        }
        if ((rc = inf.check(mem, "BGZF data"))) break;
        if (ob && hipMemcpy(out + total, dout, ob, hipMemcpyDeviceToHost) != hipSuccess) {
            rc = set_error(MSW_E_DEVICE, "D2H failed");
            break;
        }
        total += ob;
        p += used;
    }
    if (dout) (void)hipFree(dout);
    if (hstage) (void)hipHostFree(hstage);
    inf.release();
    if (!rc) *out_len = total;
    return rc;
}

}  // extern "C"
