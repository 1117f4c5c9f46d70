// msw_runtime.cpp -- device runtime and C ABI (include/msw.h) for the
// MI355X-native batched Smith-Waterman scorer.
//
// Replaces (smith_waterman/src/):
//   gpu.rs:33-132        OpenCL discovery + Mutex'd context singleton
//                        -> msw_device_count/info, one msw_ctx per device
//   aligner.rs:410-532   gpu_align: per-call JIT, buffer build, blocking finish
//                        -> msw_align_compat (kernels compiled ahead of time)
//   aligner.rs:269-289   per-chunk concat + gpu_align loop
//                        -> msw_align_batch: pinned double-buffered staging, H2D
//                           on a copy stream overlapped with the kernels
//   system_info.rs:236-243  80 % memory cap -> hipMemGetInfo
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <deque>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/msw.h"
#include "msw_kernels.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

}  // namespace

namespace msw_detail {
int set_error(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}
}  // namespace msw_detail

namespace {

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(MSW_E_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),   \
                        __FILE__, __LINE__);                                                   \
    } while (0)

inline uint32_t dup16(uint32_t v) { return (v & 0xFFFFu) | ((v & 0xFFFFu) << 16); }

// The library's run-time switches, read ONCE when a context is created
// (msw_ctx_create -> read_options) and kept in the context: no call or launch
// path reads the environment.  Every one forces a code path the tests cover
// (INTEGRATION.md section 4), or turns a diagnostic trace on.
struct Options {
    bool no_f16 = false;          // MSW_NO_F16: the integer path for every launch
    bool force_long = false;      // MSW_FORCE_LONG=1: every pair on the long-pair kernel
    uint64_t long_blocks = 0;     // MSW_LONG_BLOCKS: a fixed long-pair block count (work-queue grids)
    bool layout_set = false;      // MSW_LAYOUT given (per-bucket launches then)
    bool force_pairs = false, force_split = false, force_mixed = false;  // its value
    bool group_set = false;       // MSW_GROUP_LANES given
    uint32_t group_lanes = 0;     // its value (8..16)
    bool no_multi = false;        // MSW_NO_MULTI: one launch per bucket
    bool host_trace = false;      // MSW_HOST_TRACE: per-call host phase times on stderr
    std::string wave_trace;       // MSW_WAVE_TRACE=file: per-block placement records
    uint64_t chunk = 65536;       // GPU_CHUNK_SIZE_READS: default pairs per staged chunk (aligner.rs:9-15)
    uint64_t gz_group_bytes = 1024ull << 20;  // MSW_GZ_GROUP_MB: output bytes per msw_bgzf_inflate launch
};

Options read_options() {
    Options o;
    auto has = [](const char* k) { return getenv(k) != nullptr; };
    o.no_f16 = has("MSW_NO_F16");
    const char* fl = getenv("MSW_FORCE_LONG");
    o.force_long = fl && *fl == '1';
    const char* lb = getenv("MSW_LONG_BLOCKS");
    o.long_blocks = lb && atoll(lb) > 0 ? (uint64_t)atoll(lb) : 0;
    const char* lay = getenv("MSW_LAYOUT");
    o.layout_set = lay != nullptr;
    o.force_pairs = lay && !strcmp(lay, "pairs");
    o.force_split = lay && !strcmp(lay, "split");
    o.force_mixed = lay && !strcmp(lay, "mixed");
    const char* g = getenv("MSW_GROUP_LANES");
    o.group_set = g != nullptr;
    o.group_lanes = g ? (uint32_t)atoi(g) : 0u;
    o.no_multi = has("MSW_NO_MULTI");
    o.host_trace = has("MSW_HOST_TRACE");
    const char* wt = getenv("MSW_WAVE_TRACE");
    o.wave_trace = wt ? wt : "";
    const char* v = getenv("GPU_CHUNK_SIZE_READS");
    if (v && *v) {
        char* end = nullptr;
        const unsigned long long n = strtoull(v, &end, 10);
        if (end && *end == '\0' && n > 0) o.chunk = n;
    }
    const char* gz = getenv("MSW_GZ_GROUP_MB");
    if (gz && atoll(gz) > 0) o.gz_group_bytes = (uint64_t)atoll(gz) << 20;
    return o;
}

const Options kDefaultOptions{};

// Validated kernel constants for one scoring scheme.
struct Scheme {
    const Options* opt = &kDefaultOptions;  // the context's switches
    bool affine, coords;
    uint32_t match2, delta2, gap2, open_ext2, bias2, code_shift;
    int32_t match;
    uint32_t bias;  // affine value bias K (0 for linear)
    // f16 fast path: match and mismatch are f16 values with a zero low byte
    // (the v_perm tables hold high bytes only); per-launch bound in f16_fits.
    bool f16_scheme;
    uint32_t f16_hi, f16_ngap2, f16_noe2;
};

int make_scheme(const msw_scoring_t* sc, const Options& opt, Scheme* s) {
    if (!sc) return fail(MSW_E_INVALID, "scoring is NULL");
    s->opt = &opt;
    if (sc->match < 1 || sc->match > 64)
        return fail(MSW_E_RANGE, "match=%d outside [1, 64]", sc->match);
    if (sc->mismatch > 0 || sc->match - sc->mismatch > 64)
        return fail(MSW_E_RANGE, "mismatch=%d outside [match-64, 0]", sc->mismatch);
    if (sc->gap_extend < 0 || sc->gap_open < 0)
        return fail(MSW_E_RANGE, "negative gap penalty (open=%d extend=%d)", sc->gap_open,
                    sc->gap_extend);
    if (sc->gap_extend > 1024 || sc->gap_open > 30000)
        return fail(MSW_E_RANGE, "gap penalty too large (gap_extend <= 1024, gap_open <= 30000)");
    s->affine = sc->affine != 0;
    s->coords = sc->want_coords != 0;
    s->match = sc->match;
    const uint32_t delta = (uint32_t)(sc->match - sc->mismatch);
    uint32_t shift = 0;
    while ((1u << shift) < delta) ++shift;
    s->code_shift = shift;
    s->match2 = dup16((uint32_t)sc->match);
    s->delta2 = dup16(delta);
    s->gap2 = dup16((uint32_t)sc->gap_extend);
    // Affine kernels keep H/E/F biased by K = 256 + gap_extend (msw_kernels.hip):
    // K > 0xFF, the largest substitution penalty (fast-path padding columns).
    s->bias = s->affine ? 256u + (uint32_t)sc->gap_extend : 0u;
    s->bias2 = dup16(s->bias);
    s->open_ext2 = dup16((uint32_t)(sc->gap_open + sc->gap_extend) + s->bias);
    // f16 domain (cells H * 2^-11, exact below 2048): gaps of 2048 or more
    // zero any cell, exactly as 2047 does, so they are capped there.
    const uint32_t mb = msw::f16_cell_bits(sc->match), xb = msw::f16_cell_bits(sc->mismatch);
    s->f16_scheme = (mb & 0xFFu) == 0 && (xb & 0xFFu) == 0;
    s->f16_hi = (mb >> 8) | ((xb >> 8) << 8);
    const int32_t ge = std::min(sc->gap_extend, 2047);
    const int32_t oe = std::min(sc->affine ? sc->gap_open + sc->gap_extend : sc->gap_extend, 2047);
    s->f16_ngap2 = dup16(msw::f16_cell_bits(-ge));
    s->f16_noe2 = dup16(msw::f16_cell_bits(-oe));
    return MSW_OK;
}

// The f16 path holds every cell value (<= match * min(m, n)) below 2048.
bool f16_fits(const Scheme& s, uint32_t max_m, uint32_t max_n) {
    if (s.opt->no_f16) return false;  // tests: force the integer path
    return s.f16_scheme && (uint64_t)s.match * (std::min(max_m, max_n) + 2u) < 2048u;
}

// Length limits: pairs up to kMaxReadLen x kMaxWinLen run on the packed
// 16-bit kernels (every cell value, <= match * (257 + 1) + bias < 0x7C00, is
// a finite non-negative f16 bit pattern for v_pk_maximum3_f16); longer reads
// or windows, up to kMaxLongLen (the i16 coordinates), on the i32 long-pair
// kernel (msw_long.hip).
int check_bounds(const Scheme& s, uint32_t max_m, uint32_t max_n) {
    (void)s;
    if (max_m > (uint32_t)msw::kMaxLongLen)
        return fail(MSW_E_RANGE, "read length %u > %d", max_m, msw::kMaxLongLen);
    if (max_n > (uint32_t)msw::kMaxLongLen)
        return fail(MSW_E_RANGE, "window length %u > %d", max_n, msw::kMaxLongLen);
    return MSW_OK;
}

// A pair (or a bound) beyond the packed kernels' limits.
inline bool is_long(uint32_t m, uint32_t n) {
    return m > (uint32_t)msw::kMaxReadLen || n > (uint32_t)msw::kMaxWinLen;
}
// MSW_FORCE_LONG=1 (Options::force_long) sends every pair to the long-pair
// kernel (tests and tools/long_bench.py run it on the packed kernels' shapes).

// Long-pair launch (p's pointers, order and output fields set by the caller):
// one wave per pair, one block per slot: the dispatcher fills every wave slot
// the kernel's registers and LDS allow and refills freed ones in slot order,
// so with the slots of spread lengths sorted heaviest first (`spread`,
// bucket_chunk) that is longest-job-first over the SIMDs (tools/long_bench.py
// mixed 257-2000: 2.4 -> 3.9 TCUPS).  Equal pairs whose last round would be a
// short tail (<= 1/8 of the resident waves, running almost alone) are spread
// evenly over the fewest rounds instead (150 x 5000: 3.0 -> 3.6 TCUPS; with
// larger tails keeping full occupancy measured faster).  Past a block cap
// (boundary-row scratch <= 1 GiB), finished blocks take the next slot from a
// work queue.  Scratch and queue counter are allocated stream-ordered on
// `st`, so calls on any stream stay independent.
int launch_long(const Scheme& sch, msw::SwParams p, uint64_t n, uint32_t max_m, uint32_t max_n, bool spread,
                int cu_count, hipStream_t st) {
    if (n == 0) return MSW_OK;
    p.n_slots = (uint32_t)n;
    const bool strips = max_m > 64u * (uint32_t)msw::long_rows_per_lane(max_m);
    const size_t per_block = strips ? (size_t)msw::long_scratch_cols(max_n) * (sch.affine ? 2u : 1u) * sizeof(int32_t) : 0;
    const uint64_t resident =
        (uint64_t)(cu_count > 0 ? cu_count : 256) * (uint64_t)msw::long_blocks_per_cu(sch.affine, sch.coords, max_m, max_n);
    uint64_t blocks = n;
    if (!spread && n > resident && n % resident != 0 && (n % resident) * 8 <= resident) {
        const uint64_t rounds = (n + resident - 1) / resident;
        blocks = (n + rounds - 1) / rounds;
    }
    blocks = std::min<uint64_t>(blocks, per_block ? std::max<uint64_t>(resident, (1ull << 30) / per_block) : 1ull << 20);
    if (sch.opt->long_blocks) blocks = std::min<uint64_t>(n, sch.opt->long_blocks);  // tests: a fixed block count
    const bool queue = n > blocks;
    const size_t scratch_bytes = (size_t)blocks * per_block;
    uint8_t* mem = nullptr;
    if (strips || queue) {
        HIP_TRY(hipMallocAsync((void**)&mem, scratch_bytes + 256, st));
        p.long_scratch = strips ? reinterpret_cast<int32_t*>(mem) : nullptr;
        p.long_cols = strips ? msw::long_scratch_cols(max_n) : 0u;
        if (queue) {
            p.long_next = reinterpret_cast<uint32_t*>(mem + scratch_bytes);
            HIP_TRY(hipMemsetAsync(p.long_next, 0, sizeof(uint32_t), st));
        }
    }
    const hipError_t e = msw::launch_sw_long(p, sch.affine, sch.coords, max_m, max_n, (uint32_t)blocks, st);
    if (mem) HIP_TRY(hipFreeAsync(mem, st));
    HIP_TRY(e);
    return MSW_OK;
}

msw::SwParams base_params(const Scheme& s) {
    msw::SwParams p;
    memset(&p, 0, sizeof(p));
    p.code_shift = s.code_shift;
    p.match2 = s.match2;
    p.delta2 = s.delta2;
    p.gap2 = s.gap2;
    p.open_ext2 = s.open_ext2;
    p.bias2 = s.bias2;
    p.f16_hi = s.f16_hi;
    p.f16_ngap2 = s.f16_ngap2;
    p.f16_noe2 = s.f16_noe2;
    return p;
}

// Device + pinned buffers for one in-flight chunk.  The per-pair metadata of a
// chunk (window positions, read and window lengths, slot order) is one block,
// [pos i64 | rlen u16 | wlen u16 | order u32] x n, uploaded by ONE copy of the
// part the chunk uses (pairs mode skips the positions, a chunk in input order
// the order); the results [score i32 | end_i i16 | end_j i16] come back by one
// copy, or are written by the kernels straight into the pinned block (a
// one-chunk call: no copy and no event between the kernel and the host).
struct Slot {
    size_t cap_pairs = 0, cap_read = 0, cap_win = 0;
    uint8_t *d_reads = nullptr, *d_wins = nullptr, *d_meta = nullptr, *d_res = nullptr;
    uint8_t *h_reads = nullptr, *h_wins = nullptr, *h_meta = nullptr, *h_res = nullptr;
    // device addresses of the pinned staging blocks (one-chunk calls pull from them)
    const uint8_t *g_reads = nullptr, *g_wins = nullptr, *g_meta = nullptr;
    // views into d_meta / h_meta and d_res / h_res
    int64_t *d_pos = nullptr, *h_pos = nullptr;
    uint32_t *d_order = nullptr, *h_order = nullptr;
    uint16_t *d_rlen = nullptr, *d_wlen = nullptr, *h_rlen = nullptr, *h_wlen = nullptr;
    int32_t *d_score = nullptr, *h_score = nullptr;
    int16_t *d_ei = nullptr, *d_ej = nullptr, *h_ei = nullptr, *h_ej = nullptr;
    // where this chunk's kernels store results: the device block or the host one
    int32_t* k_score = nullptr;
    int16_t *k_ei = nullptr, *k_ej = nullptr;
    hipEvent_t uploaded = nullptr, computed = nullptr, done = nullptr;
    // timing events around the chunk's scoring launches; a chunk whose kernels
    // write the host block directly ends on k_end (done is not recorded)
    hipEvent_t k_start = nullptr, k_end = nullptr;
    bool busy = false;
    bool by_slot = false;  // results in slot order: the drain scatters them through h_order
    bool direct_out = false;  // the kernels wrote h_res themselves; k_end marks completion
    uint64_t ticket = 0;  // msw_align_*_async call that owns the chunk in flight
    uint64_t seq = 0;     // submission order of the chunk (drains go in this order)
    // Pending readback bookkeeping.
    uint64_t first = 0, count = 0;
    msw_out_t out{};
};

constexpr size_t kMetaBytesPerPair = 8 + 2 + 2 + 4;
constexpr size_t kResBytesPerPair = 4 + 2 + 2;

// Views of the metadata / result blocks for a chunk of n pairs (each array
// packed at n entries, so one copy moves exactly the chunk's bytes).
void set_views(Slot& s, uint64_t n) {
    auto views = [n](uint8_t* meta, uint8_t* res, int64_t*& pos, uint32_t*& order, uint16_t*& rlen, uint16_t*& wlen,
                     int32_t*& score, int16_t*& ei, int16_t*& ej) {
        pos = reinterpret_cast<int64_t*>(meta);
        rlen = reinterpret_cast<uint16_t*>(meta + 8 * n);
        wlen = reinterpret_cast<uint16_t*>(meta + 10 * n);
        order = reinterpret_cast<uint32_t*>(meta + 12 * n);
        score = reinterpret_cast<int32_t*>(res);
        ei = reinterpret_cast<int16_t*>(res + 4 * n);
        ej = reinterpret_cast<int16_t*>(res + 6 * n);
    };
    views(s.d_meta, s.d_res, s.d_pos, s.d_order, s.d_rlen, s.d_wlen, s.d_score, s.d_ei, s.d_ej);
    views(s.h_meta, s.h_res, s.h_pos, s.h_order, s.h_rlen, s.h_wlen, s.h_score, s.h_ei, s.h_ej);
}

void free_slot(Slot& s) {
    for (void* p : {(void*)s.d_reads, (void*)s.d_wins, (void*)s.d_meta, (void*)s.d_res})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)s.h_reads, (void*)s.h_wins, (void*)s.h_meta, (void*)s.h_res})
        if (p) (void)hipHostFree(p);
    s = Slot{};
}

}  // namespace

struct msw_ctx {
    int device = 0;
    int cu_count = 256;
    Options opt;  // the environment's switches, read at creation
    // compute: created with the context; the others too, unless the context
    // is lean (MSW_CTX_LEAN: made by the first call that uses them,
    // aux_streams): a stream costs 3-30 ms to create (the first few each make
    // a hardware queue) and as much to destroy, and the --full-wgs GPU-reader
    // workers never use them (profiles/r06/c3f/)
    hipStream_t compute = nullptr, copy = nullptr, d2h = nullptr;
    // multi-chunk calls alternate their chunks' kernels over compute and
    // compute2, so chunk k+1's waves start under chunk k's tail (one stream
    // would idle the CUs the tail leaves)
    hipStream_t compute2 = nullptr;
    hipStream_t side = nullptr;  // long-pair launches beside packed ones (fork_side)
    // Staging slots, used round robin by successive chunks (and calls): with
    // three, the host stages chunk k+1 while k runs and k-1 drains, so the
    // uploads of k+1 finish under kernel k.
    static constexpr int kSlots = 3;
    Slot slots[kSlots];
    uint64_t next_ticket = 1, done_ticket = 0;
    uint64_t slot_seq = 0;  // chunks submitted (slot = slot_seq % kSlots)
    msw_stats_t stats{};    // msw_ctx_stats: host-batch calls since creation / the last reset
    // Origin of the kernel-time interval union (recorded at creation, moved
    // forward every ~second of GPU time so float ms offsets stay fine-grained:
    // epoch_next is recorded, and once it has completed becomes the epoch)
    hipEvent_t epoch = nullptr, epoch_next = nullptr;
    double busy_until = 0.0;     // ms after epoch at which the counted scoring intervals end
    // pinned_cached: the most recently used (address, bytes) ranges asked
    // about, most recent first (move to front on a hit).  16: a --full-wgs
    // worker's two result sets x five copies per batch, plus a call's reads /
    // windows, stay cached (the 8-entry FIFO missed every one).
    struct PinnedRange {
        const void* p = nullptr;
        size_t bytes = 0;
        bool pinned = false;
        const uint8_t* dev = nullptr;  // its device address (pinned ranges)
    };
    static constexpr unsigned kPinnedRanges = 16;
    PinnedRange pinned_ranges[kPinnedRanges];
    unsigned pinned_used = 0;
    uint64_t pinned_epoch = 0;           // g_host_free_epoch when the cache was last valid
    uint64_t pinned_hits = 0, pinned_misses = 0;  // MSW_HOST_TRACE
    // compat buffers
    uint8_t *c_s1 = nullptr, *c_s2 = nullptr;
    int32_t* c_res = nullptr;
    size_t c_cap = 0;
    hipEvent_t c_k0 = nullptr, c_k1 = nullptr;  // timing of the compat launch (msw_ctx_stats)
    // msw_align_reads_device scratch: the cut windows and their clipped lengths
    // msw_align_reads_device's window slab and lengths, one set per stream
    // it is called on (calls on two streams run concurrently)
    struct ReadsScratch {
        hipStream_t st = nullptr;
        uint8_t* wins = nullptr;
        uint16_t* wlen = nullptr;
        size_t wins_cap = 0, wlen_cap = 0;
    };
    std::vector<ReadsScratch> rscratch;
    // streams made by msw_stream_create (synchronised by msw_synchronize,
    // destroyed with the context if the caller has not)
    std::vector<hipStream_t> user_streams;
    // timing events of msw_align_reads_device launches not yet harvested
    struct DevTiming {
        hipEvent_t k0, k1;
        uint64_t pairs;
    };
    std::deque<DevTiming> dev_timings;
    std::vector<hipEvent_t> free_events;
    // free_events and fences: msw_fence_wait may run on several threads at
    // once (--full-wgs settles its last two batches on two)
    std::mutex ev_mu;
    msw::Layout last_layout = msw::Layout::kPairs;  // the last packed launch's plan (MSW_HOST_TRACE)
    uint32_t last_group_lanes = 0, last_kr = 0;
    std::unordered_map<uint64_t, hipEvent_t> fences;  // msw_fence_record, not yet waited on
    uint64_t next_fence = 1;
};

struct msw_genome {
    const msw_ctx* ctx = nullptr;  // identity only
    int device = 0;
    uint8_t* d_seq = nullptr;      // len + kGenomePad bytes (cut kernel over-reads <= 20)
    uint64_t len = 0;
};

// Internal accessors for the other units of the library (msw_gfastq.cpp).
namespace msw_detail {
int ctx_device(const msw_ctx* c) { return c->device; }
hipStream_t ctx_compute_stream(const msw_ctx* c) { return c->compute; }
uint64_t ctx_gz_group_bytes(const msw_ctx* c) { return c->opt.gz_group_bytes; }
}  // namespace msw_detail

namespace {

int set_device(msw_ctx* ctx) {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur == ctx->device) return MSW_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    return MSW_OK;
}

// The streams a context creates on first use (compute is made with it).
int aux_streams(msw_ctx* ctx) {
    for (hipStream_t* st : {&ctx->compute2, &ctx->copy, &ctx->d2h, &ctx->side})
        if (!*st) HIP_TRY(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
    return MSW_OK;
}

hipEvent_t take_event(msw_ctx* ctx) {
    {
        std::lock_guard<std::mutex> lk(ctx->ev_mu);
        if (!ctx->free_events.empty()) {
            hipEvent_t e = ctx->free_events.back();
            ctx->free_events.pop_back();
            return e;
        }
    }
    hipEvent_t e = nullptr;
    return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}

// A finished scoring interval [k0, k1] into ctx->stats.kernel_ms as part of
// the union of all of them: chunks alternate over two compute streams and
// overlap, so each interval adds only its part after everything counted so
// far ends.  Durations come from elapsed(k0, k1) (exact), the overlap from
// offsets against the context's epoch event.  Intervals arrive in
// submission order, i.e. in start order but for a chunk that starts before
// its predecessor, which is then undercounted, never counted twice.
// Callers hand intervals over oldest chunk first (drain_through), so each
// starts no earlier than the previous one save for the two compute streams'
// overlap, which is exactly what the union removes.
void add_kernel_interval(msw_ctx* ctx, hipEvent_t k0, hipEvent_t k1) {
    float dur = 0.f, start = 0.f;
    if (hipEventElapsedTime(&dur, k0, k1) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    if (!ctx->epoch || hipEventElapsedTime(&start, ctx->epoch, k0) != hipSuccess) {
        (void)hipGetLastError();
        ctx->stats.kernel_ms += dur;
        return;
    }
    const double covered = std::min<double>(dur, std::max(0.0, ctx->busy_until - start));
    ctx->stats.kernel_ms += dur - covered;
    ctx->busy_until = std::max<double>(ctx->busy_until, (double)start + dur);
    // Re-base: a float offset of T ms resolves T / 2^24 -- 0.25 ms after an
    // hour -- so the epoch moves up once it is a second behind.  The new one
    // is an event on the compute stream; it takes over once it has completed
    // and its distance from the old one is known (both offsets then move by
    // it; an interval starting before it gets a negative offset, which the
    // union handles the same way).
    if (ctx->epoch_next) {
        float delta = 0.f;
        if (hipEventQuery(ctx->epoch_next) == hipSuccess &&
            hipEventElapsedTime(&delta, ctx->epoch, ctx->epoch_next) == hipSuccess) {
            ctx->busy_until -= delta;
            std::swap(ctx->epoch, ctx->epoch_next);
            (void)hipEventDestroy(ctx->epoch_next);
            ctx->epoch_next = nullptr;
        }
        (void)hipGetLastError();
    } else if (start > 1000.f) {
        if (hipEventCreate(&ctx->epoch_next) != hipSuccess || hipEventRecord(ctx->epoch_next, ctx->compute) != hipSuccess) {
            if (ctx->epoch_next) (void)hipEventDestroy(ctx->epoch_next);
            ctx->epoch_next = nullptr;
            (void)hipGetLastError();
        }
    }
}

// Kernel time of finished msw_align_reads_device launches into ctx->stats
// (wait = true: all of them, after synchronising).
void harvest_dev_timings(msw_ctx* ctx, bool wait) {
    while (!ctx->dev_timings.empty()) {
        msw_ctx::DevTiming& t = ctx->dev_timings.front();
        if (wait) (void)hipEventSynchronize(t.k1);
        else if (hipEventQuery(t.k1) != hipSuccess) break;
        add_kernel_interval(ctx, t.k0, t.k1);
        ctx->stats.launches += 1;
        ctx->stats.pairs += t.pairs;
        {
            std::lock_guard<std::mutex> lk(ctx->ev_mu);
            ctx->free_events.push_back(t.k0);
            ctx->free_events.push_back(t.k1);
        }
        ctx->dev_timings.pop_front();
    }
}

template <typename T>
int grow_dev(T** p, size_t n) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    if (n == 0) return MSW_OK;
    hipError_t e = hipMalloc((void**)p, n * sizeof(T));
    if (e != hipSuccess) return fail(MSW_E_NOMEM, "hipMalloc(%zu B): %s", n * sizeof(T), hipGetErrorString(e));
    return MSW_OK;
}
template <typename T>
int grow_host(T** p, size_t n, unsigned flags = hipHostMallocDefault) {
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    if (n == 0) return MSW_OK;
    hipError_t e = hipHostMalloc((void**)p, n * sizeof(T), flags);
    if (e != hipSuccess) return fail(MSW_E_NOMEM, "hipHostMalloc(%zu B): %s", n * sizeof(T), hipGetErrorString(e));
    return MSW_OK;
}

// The device address of a pinned host block (the pull copy reads it there).
int dev_addr(const uint8_t* h, const uint8_t** out) {
    void* d = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&d, (void*)h, 0));
    *out = (const uint8_t*)d;
    return MSW_OK;
}

int ensure_slot(Slot& s, size_t pairs, size_t read_bytes, size_t win_bytes) {
    int rc;
    if (!s.uploaded) {
        HIP_TRY(hipEventCreateWithFlags(&s.uploaded, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&s.computed, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        HIP_TRY(hipEventCreate(&s.k_start));
        HIP_TRY(hipEventCreate(&s.k_end));
    }
    if (pairs > s.cap_pairs) {
        // the result block is mapped and coherent: one-chunk calls have the
        // kernels store into it directly (its device address is the host one)
        if ((rc = grow_dev(&s.d_meta, pairs * kMetaBytesPerPair)) ||
            (rc = grow_host(&s.h_meta, pairs * kMetaBytesPerPair)) ||
            (rc = grow_dev(&s.d_res, pairs * kResBytesPerPair)) ||
            (rc = grow_host(&s.h_res, pairs * kResBytesPerPair, hipHostMallocMapped | hipHostMallocCoherent)) ||
            (rc = dev_addr(s.h_meta, &s.g_meta)))
            return rc;
        s.cap_pairs = pairs;
    }
    if (read_bytes > s.cap_read) {
        if ((rc = grow_dev(&s.d_reads, read_bytes)) || (rc = grow_host(&s.h_reads, read_bytes)) ||
            (rc = dev_addr(s.h_reads, &s.g_reads)))
            return rc;
        s.cap_read = read_bytes;
    }
    if (win_bytes > s.cap_win) {
        if ((rc = grow_dev(&s.d_wins, win_bytes)) || (rc = grow_host(&s.h_wins, win_bytes)) ||
            (rc = dev_addr(s.h_wins, &s.g_wins)))
            return rc;
        s.cap_win = win_bytes;
    }
    return MSW_OK;
}

// Lane-group layout of one launch.  "pairs" scores 2 pairs per G-lane group,
// "split" 1 pair per group (rows split over the two halves; half the work per
// wave), "mixed" (G = 16) runs up to one pairs-wave per SIMD and the rest as
// split-waves.  G (8..16 lanes per group, 64 / G groups per wave) sets how many
// pairs one wave holds, so a small batch can be cut into about one wave per
// SIMD.  The choice minimises a makespan model:
//  - a wave issues steps x (a * KR + b) instructions (a, b fitted to the
//    compiled loops: tools/issue_sim.py);
//  - waves are dealt round-robin over the 4 x CU SIMDs in block order (what
//    tools/wave_trace.py observes), and a SIMD holding k waves issues one
//    instruction per r(k) cycles (measured: 5.27 alone, 4.6 for two, 3.94 at
//    eight -- a lone wave cannot issue back to back).
// MSW_LAYOUT=pairs|split|mixed and MSW_GROUP_LANES=8..16 override (tests use
// them to cover every path).
struct LaunchPlan {
    msw::Layout layout;
    uint32_t pairs_blocks;
    uint32_t group_lanes;
    uint32_t groups;
};

static double simd_cycles_per_instr(uint64_t k) {
    static const double r[] = {0.0, 5.27, 4.6, 4.3, 4.15, 4.05, 4.0, 3.97, 3.94};
    return r[k > 8 ? 8 : k];
}

LaunchPlan choose_layout(uint64_t n_pairs, uint32_t max_m, uint32_t max_n, const Scheme& sch, int cu_count) {
    const uint64_t simds = 4ull * (uint64_t)(cu_count > 0 ? cu_count : 256);
    // VALU instructions per packed row of the compiled loops:
    // f16 path 4.8 (+4.1 affine, +2.6 coordinates); integer path 5.5 (+5.2, +2.8).
    const bool f16 = f16_fits(sch, max_m, max_n);
    const double per_row = f16 ? 4.8 + (sch.affine ? 4.1 : 0.0) + (sch.coords ? 2.6 : 0.0)
                               : 5.5 + (sch.affine ? 5.2 : 0.0) + (sch.coords ? 2.8 : 0.0);
    auto wave_instr = [&](bool split, uint32_t G) {
        const int kr = msw::rows_per_lane(max_m, split, G);
        const double steps = (double)max_n + (split ? 2.0 * G : (double)G);
        const double over = (split ? 5.5 : 3.0) + (sch.affine ? 2.0 : 0.0);
        return steps * (per_row * kr + over) + 300.0;
    };
    // Round-robin dealing: SIMD i holds waves i, i + S, ...; time = its
    // instructions x r(its wave count).
    auto makespan = [&](uint64_t w1, double c1, uint64_t w2, double c2) {
        const uint64_t w = w1 + w2;
        if (w == 0) return 0.0;
        if (w2 == 0 || w1 == 0) {
            const double c = w1 ? c1 : c2;
            const uint64_t k = (w + simds - 1) / simds;
            return (double)k * c * simd_cycles_per_instr(k);
        }
        // SIMD i holds w1 / S + (i < w1 % S) first-kind waves of w / S + (i <
        // w % S): constant between the two breakpoints, so three SIMDs cover
        // every case (closed form: a loop over the waves cost ~1 ms of host
        // time per 2M-pair launch, stalling the GPU between kernels)
        const uint64_t b1 = w1 % simds, b = w % simds;
        double t = 0.0;
        for (uint64_t i : {(uint64_t)0, std::min(b1, b), std::max(b1, b)}) {
            if (i >= simds) continue;
            const uint64_t n1 = w1 / simds + (i < b1 ? 1 : 0), n = w / simds + (i < b ? 1 : 0);
            if (n == 0) continue;
            t = std::max(t, ((double)n1 * c1 + (double)(n - n1) * c2) * simd_cycles_per_instr(n));
        }
        return t;
    };
    const uint32_t stride = msw::stream_stride(max_n);
    const uint32_t force_g = sch.opt->group_lanes;
    const bool force_pairs = sch.opt->force_pairs, force_split = sch.opt->force_split;
    const bool force_mixed = sch.opt->force_mixed;

    LaunchPlan best{msw::Layout::kPairs, 0, 16, 4};
    double best_t = 1e300;
    for (int split = 0; split <= 1; ++split) {
        if ((force_pairs && split) || (force_split && !split) || force_mixed) continue;
        for (uint32_t G = 16; G >= 8; --G) {
            if (force_g ? G != force_g : ((force_pairs || force_split) && G != 16)) continue;
            const int kr = msw::rows_per_lane(max_m, split, G);
            if (kr > (split ? 8 : msw::kMaxRowsPerLane)) continue;
            const uint32_t groups = 64 / G;
            if (G != 16 && msw::lds_bytes(stride, groups) > 65536) continue;
            const uint64_t per = msw::pairs_per_wave(split, groups);
            // 17..19 rows in narrower groups (150 bp reads: G = 8 / KR = 19 or
            // G = 9 / KR = 17) fit only 2-3 waves per SIMD (VGPRs; the LDS of 7-8
            // window streams), and the makespan model does not predict where
            // they start to win (an occupancy-rounds model puts
            // them ahead at every size).  So the gate is the measured crossover
            // per instance family (tools/group_lanes_probe.py, alternating A/B
            // against G = 16, profiles/r05/ab/group_9v16.jsonl and
            // profiles/r04/ab/group_lanes_probe_sizes.jsonl):
            //  KR 17 (G = 9): 2-3 % slower at 9 waves per SIMD (131k pairs),
            //    2.4-3.5 % faster at 18, 3.5-5 % at 37, 5-6 % at 55: >= 16;
            //  KR 18..19 (G = 8): 4 % faster to 13 % slower at 16 waves per
            //    SIMD (262k), 5-6 % faster at 64 (1M): >= 48.
            // Larger rows-per-lane counts were never measured: not taken.
            const uint64_t min_waves = kr <= 17 ? 16 : 48;
            if (!split && G != 16 && kr > 16 && !force_g &&
                (kr > 19 || (n_pairs + per - 1) / per < min_waves * simds))
                continue;
            const double t = makespan((n_pairs + per - 1) / per, wave_instr(split, G), 0, 0.0);
            if (t < best_t * 0.995) {
                best_t = t;
                best = {split ? msw::Layout::kSplit : msw::Layout::kPairs, 0, G, groups};
            }
        }
    }
    // Mixed grid (G = 16, even KR): up to one pairs-wave per SIMD, then split waves.
    const int krp = msw::rows_per_lane(max_m, false);
    const bool mixed_ok = (krp % 2) == 0 && krp <= 16 && (!force_g || force_g == 16) && !force_pairs && !force_split;
    if (mixed_ok) {
        const double cp = wave_instr(false, 16), cs = wave_instr(true, 16);
        for (uint64_t k = 1; k <= 4; ++k) {
            const uint64_t pw = std::min<uint64_t>(n_pairs / 8, k * simds / 4);
            if (pw == 0) continue;
            const uint64_t rest = n_pairs - pw * 8;
            const double t = makespan(pw, cp, (rest + 3) / 4, cs);
            if (t < best_t * 0.995 || (force_mixed && best.layout != msw::Layout::kMixed)) {
                best_t = t;
                best = {msw::Layout::kMixed, (uint32_t)pw, 16, 4};
            }
        }
        if (force_mixed && best.layout != msw::Layout::kMixed)
            best = {msw::Layout::kMixed, (uint32_t)std::min<uint64_t>(n_pairs / 8, simds), 16, 4};
    } else if (force_mixed) {
        best = {msw::Layout::kSplit, 0, 16, 4};
    }
    return best;
}

// Whether one launch of n pairs under these bounds can read its windows from
// the resident genome: the GEN instances exist for the pairs layout with up
// to 16 rows per lane (the shapes of short-read chunks), not for long pairs.
bool genome_windows_ok(uint64_t n, uint32_t max_m, uint32_t max_n, const Scheme& sch, int cu_count) {
    if (is_long(max_m, max_n)) return false;
    const LaunchPlan plan = choose_layout(n, max_m, max_n, sch, cu_count);
    return plan.layout == msw::Layout::kPairs && msw::rows_per_lane(max_m, false, plan.group_lanes) <= 16;
}

// Buckets of one chunk: pairs grouped by rows-per-lane (read length / 16), and
// inside a bucket by window length, so every wave runs with tight bounds.
struct Bucket {
    uint32_t begin, count, max_m, max_n;
    bool long_pairs = false;  // beyond the packed kernels: sw_long_kernel
    bool spread = false;      // long pairs of spread lengths, sorted heaviest first
};

// lengths: the chunk's {min read, max read, min window, max window}.
// all_long: Options::force_long.
void bucket_chunk(const uint16_t* rlen, const uint16_t* wlen, uint64_t n, uint32_t* order,
                  std::vector<Bucket>& buckets, uint32_t lengths[4], bool all_long) {
    buckets.clear();
    // key = KR (1..24) * 257 + ceil(n / 16) (<= 256): counting sort; pairs
    // beyond the packed kernels' limits share the last key.
    constexpr int kLongKey = (msw::kMaxRowsPerLane + 1) * 257, kKeys = kLongKey + 1;
    auto key_of = [&](uint64_t i) {
        if (all_long || is_long(rlen[i], wlen[i])) return kLongKey;
        const int kr = msw::rows_per_lane(rlen[i], false);
        const int nb = (wlen[i] + 15) / 16;
        return kr * 257 + nb;
    };
    // One key (fixed-length reads and windows, the common case): one bucket in
    // input order, no sort -- unless they are long pairs of spread lengths,
    // which the work queue wants heaviest first.
    int kmin = kKeys, kmax = -1;
    uint32_t gm = 0, gn = 0, lm = 0xFFFF, ln = 0xFFFF;
    for (uint64_t i = 0; i < n; ++i) {
        const int k = key_of(i);
        kmin = std::min(kmin, k);
        kmax = std::max(kmax, k);
        gm = std::max<uint32_t>(gm, rlen[i]);
        gn = std::max<uint32_t>(gn, wlen[i]);
        lm = std::min<uint32_t>(lm, rlen[i]);
        ln = std::min<uint32_t>(ln, wlen[i]);
    }
    lengths[0] = lm, lengths[1] = gm, lengths[2] = ln, lengths[3] = gn;
    const bool spread_long = kmin == kLongKey && (gm - lm >= 64 || gn - ln >= 64);
    if (n && kmin == kmax && !spread_long) {
        for (uint64_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
        buckets.push_back({0, (uint32_t)n, gm, gn, kmin == kLongKey});
        return;
    }
    std::vector<uint32_t> hist(kKeys + 1, 0);
    for (uint64_t i = 0; i < n; ++i) hist[key_of(i) + 1]++;
    for (int k = 0; k < kKeys; ++k) hist[k + 1] += hist[k];
    std::vector<uint32_t> pos(hist.begin(), hist.end() - 1);
    for (uint64_t i = 0; i < n; ++i) order[pos[key_of(i)]++] = (uint32_t)i;
    // One bucket per KR value; the window bound is the bucket's max.
    for (int kr = 1; kr <= msw::kMaxRowsPerLane; ++kr) {
        const uint32_t b = hist[kr * 257], e = hist[kr * 257 + 257];
        if (e <= b) continue;
        uint32_t mm = 0, mn = 0;
        for (uint32_t s = b; s < e; ++s) {
            mm = std::max<uint32_t>(mm, rlen[order[s]]);
            mn = std::max<uint32_t>(mn, wlen[order[s]]);
        }
        buckets.push_back({b, e - b, mm, mn});
    }
    if (hist[kLongKey + 1] > hist[kLongKey]) {  // the long pairs: last in slot order
        const uint32_t b = hist[kLongKey], e = hist[kLongKey + 1];
        uint32_t mm = 0, mn = 0;
        for (uint32_t s = b; s < e; ++s) {
            mm = std::max<uint32_t>(mm, rlen[order[s]]);
            mn = std::max<uint32_t>(mn, wlen[order[s]]);
        }
        // heaviest first (strips x steps at the launch's rows per lane): the
        // kernel's work queue then schedules longest-job-first
        const uint32_t strip_rows = 64u * (uint32_t)msw::long_rows_per_lane(mm);
        auto cost = [&](uint32_t i) {
            return (uint64_t)((rlen[i] + strip_rows - 1) / strip_rows) * (uint64_t)(wlen[i] + 63u);
        };
        std::stable_sort(order + b, order + e, [&](uint32_t x, uint32_t y) { return cost(x) > cost(y); });
        buckets.push_back({b, e - b, mm, mn, true, cost(order[b]) != cost(order[e - 1])});
    }
}

// The packed-kernel buckets of a list (all but a trailing long bucket).
size_t short_buckets(const std::vector<Bucket>& buckets) {
    return !buckets.empty() && buckets.back().long_pairs ? buckets.size() - 1 : buckets.size();
}

// The leading buckets sw_multi_kernel takes (KR <= 16; buckets come in KR
// order); the rest of the packed buckets (KR 17..24) launch on their own.
size_t multi_buckets(const std::vector<Bucket>& buckets) {
    const size_t n = short_buckets(buckets);
    size_t k = 0;
    while (k < n && msw::rows_per_lane(buckets[k].max_m, false) <= msw::kMaxMultiKR) ++k;
    return k;
}

// One-launch table of a bucket list (msw::MultiTable): heaviest waves first
// (rows per lane x window steps), so the tail of the grid is short waves.
// [lo, hi): the KR <= 16 buckets (sw_multi_kernel) or the KR 17..24 ones (its
// wide instance).
void fill_multi(const std::vector<Bucket>& buckets, size_t lo, size_t hi, const Scheme& sch, msw::MultiTable& t) {
    std::vector<Bucket> bs(buckets.begin() + lo, buckets.begin() + hi);
    auto cost = [](const Bucket& b) { return (uint64_t)msw::rows_per_lane(b.max_m, false) * (b.max_n + 16u); };
    std::stable_sort(bs.begin(), bs.end(), [&](const Bucket& a, const Bucket& b) { return cost(a) > cost(b); });
    memset(&t, 0, sizeof(t));
    uint32_t blocks = 0;
    for (const Bucket& b : bs) {
        const uint32_t i = t.n_buckets++;
        blocks += (b.count + msw::kPairsPerWave - 1) / msw::kPairsPerWave;
        t.block_end[i] = blocks;
        t.slot_begin[i] = b.begin;
        t.count[i] = b.count;
        t.kr[i] = (uint32_t)msw::rows_per_lane(b.max_m, false);
        t.lds_stride[i] = msw::stream_stride(b.max_n);
        t.f16_ok[i] = f16_fits(sch, b.max_m, b.max_n) ? 1u : 0u;
    }
}

// Several buckets run as one sw_multi_kernel launch, unless MSW_NO_MULTI is
// set or a layout / group width is forced (MSW_LAYOUT, MSW_GROUP_LANES): then
// each bucket gets its own launch with that layout (tests cover both).
bool use_multi(size_t n_buckets, const Options& o) {
    return n_buckets > 1 && !o.no_multi && !o.layout_set && !o.group_set;
}

// A long-pair launch next to packed launches runs on the context's side
// stream, forked from `st` and joined back after the packed launches: the
// long kernel's tail and the packed buckets' short launches (a few lone waves
// each for KR 17..24) share the CUs instead of queueing behind each other.
struct SideFork {
    hipEvent_t ev = nullptr;
    SideFork() = default;
    SideFork(const SideFork&) = delete;
    SideFork& operator=(const SideFork&) = delete;
    ~SideFork() {
        if (ev) (void)hipEventDestroy(ev);
    }
};

int fork_side(msw_ctx* ctx, hipStream_t st, SideFork& f) {
    if (!ctx->side) {
        const int rc = aux_streams(ctx);
        if (rc) return rc;
    }
    HIP_TRY(hipEventCreateWithFlags(&f.ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(f.ev, st));
    HIP_TRY(hipStreamWaitEvent(ctx->side, f.ev, 0));
    return MSW_OK;
}

int join_side(msw_ctx* ctx, hipStream_t st, SideFork& f) {
    HIP_TRY(hipEventRecord(f.ev, ctx->side));
    HIP_TRY(hipStreamWaitEvent(st, f.ev, 0));
    return MSW_OK;
}

// The KR 17..24 buckets as one launch (one launch per bucket measured slower:
// 8.5 vs 12.7 TCUPS linear).
bool use_wide_multi(size_t n_wide, const Options& o) { return use_multi(n_wide, o); }

// Where a launch's windows come from: the slot's cut slab (win_stride), or,
// with a genome, straight from the resident genome at the slot's positions
// (the packed kernels only; long pairs need the slab).
void set_windows(msw::SwParams& p, const Slot& s, uint32_t win_stride, const msw_genome* g) {
    if (g) {
        p.wins = nullptr;
        p.win_stride = 0;
        p.win_src = g->d_seq;
        p.win_pos = s.d_pos;
        p.win_vec = 1;
    } else {
        p.wins = s.d_wins;
        p.win_stride = win_stride;
        p.win_vec = msw::vec_ok(p.wins, p.win_stride);
    }
}

int launch_buckets(msw_ctx* ctx, const Scheme& sch, Slot& s, uint64_t n, const std::vector<Bucket>& buckets,
                   bool use_order, uint32_t read_stride, uint32_t win_stride, hipStream_t cs,
                   const msw_genome* g = nullptr) {
    const size_t n_short = short_buckets(buckets);
    SideFork side;
    if (n_short < buckets.size()) {  // long pairs: their own launch, beside any packed ones
        const Bucket& b = buckets.back();
        msw::SwParams p = base_params(sch);
        if (g) return fail(MSW_E_INVALID, "internal: long pairs need the window slab");
        p.reads = s.d_reads;
        p.wins = s.d_wins;
        p.read_len = s.d_rlen;
        p.win_len = s.d_wlen;
        p.order = use_order ? s.d_order + b.begin : nullptr;
        p.out_by_slot = use_order ? 1u : 0u;
        p.out_slot_base = b.begin;
        p.slot_base = use_order ? 0u : b.begin;
        p.score = s.k_score;
        p.end_i = sch.coords ? s.k_ei : nullptr;
        p.end_j = sch.coords ? s.k_ej : nullptr;
        p.read_stride = read_stride;
        p.win_stride = win_stride;
        int rc = n_short ? fork_side(ctx, cs, side) : MSW_OK;
        if (!rc)
            rc = launch_long(sch, p, b.count, b.max_m, b.max_n, use_order && b.spread, ctx->cu_count,
                             n_short ? ctx->side : cs);
        if (rc) return rc;
        if (n_short == 0) return MSW_OK;
    }
    if (g && (use_order || buckets.size() != 1)) return fail(MSW_E_INVALID, "internal: genome windows need one bucket");
    const size_t n_multi = multi_buckets(buckets);
    size_t first_single = 0;
    if (use_order && use_multi(n_multi, *sch.opt)) {
        msw::SwParams p = base_params(sch);
        p.reads = s.d_reads;
        p.wins = s.d_wins;
        p.read_len = s.d_rlen;
        p.win_len = s.d_wlen;
        p.order = s.d_order;
        p.score = s.k_score;
        p.end_i = sch.coords ? s.k_ei : nullptr;
        p.end_j = sch.coords ? s.k_ej : nullptr;
        p.read_stride = read_stride;
        set_windows(p, s, win_stride, g);
        p.group_lanes = 16;
        p.groups = 4;
        p.out_by_slot = 1;
        p.out_slot_base = 0;
        msw::MultiTable t;
        fill_multi(buckets, 0, n_multi, sch, t);
        HIP_TRY(msw::launch_sw_multi(p, t, sch.affine, sch.coords, cs));
        first_single = n_multi;
    }
    // the KR 17..24 buckets: one launch of the wide instance when there are
    // several (one launch each left each bucket's few waves running alone)
    size_t single_end = n_short;
    if (use_order && use_wide_multi(n_short - n_multi, *sch.opt)) {
        msw::SwParams p = base_params(sch);
        p.reads = s.d_reads;
        p.wins = s.d_wins;
        p.read_len = s.d_rlen;
        p.win_len = s.d_wlen;
        p.order = s.d_order;
        p.score = s.k_score;
        p.end_i = sch.coords ? s.k_ei : nullptr;
        p.end_j = sch.coords ? s.k_ej : nullptr;
        p.read_stride = read_stride;
        set_windows(p, s, win_stride, g);
        p.group_lanes = 16;
        p.groups = 4;
        p.out_by_slot = 1;
        p.out_slot_base = 0;
        msw::MultiTable t;
        fill_multi(buckets, n_multi, n_short, sch, t);
        HIP_TRY(msw::launch_sw_multi(p, t, sch.affine, sch.coords, cs));
        single_end = n_multi;
    }
    for (size_t bi = first_single; bi < single_end; ++bi) {
        const Bucket& b = buckets[bi];
        msw::SwParams p = base_params(sch);
        p.reads = s.d_reads;
        p.wins = s.d_wins;
        p.read_len = s.d_rlen;
        p.win_len = s.d_wlen;
        p.order = use_order ? s.d_order + b.begin : nullptr;
        p.out_by_slot = use_order ? 1u : 0u;
        p.out_slot_base = b.begin;
        p.score = s.k_score;
        p.end_i = sch.coords ? s.k_ei : nullptr;
        p.end_j = sch.coords ? s.k_ej : nullptr;
        p.read_stride = read_stride;
        set_windows(p, s, win_stride, g);
        p.n_slots = b.count;
        p.lds_stride = msw::stream_stride(b.max_n);
        p.f16_ok = f16_fits(sch, b.max_m, b.max_n) ? 1u : 0u;
        const LaunchPlan plan = choose_layout(b.count, b.max_m, b.max_n, sch, ctx->cu_count);
        p.pairs_blocks = plan.pairs_blocks;
        p.group_lanes = plan.group_lanes;
        p.groups = plan.groups;
        ctx->last_layout = plan.layout;
        ctx->last_group_lanes = plan.group_lanes;
        ctx->last_kr = (uint32_t)msw::rows_per_lane(b.max_m, plan.layout == msw::Layout::kSplit, plan.group_lanes);
        HIP_TRY(msw::launch_sw(p, sch.affine, sch.coords, b.max_m, plan.layout, cs));
    }
    if (side.ev) return join_side(ctx, cs, side);
    (void)n;
    return MSW_OK;
}

// Copy finished results of a slot into the caller's arrays; the chunk's
// kernel time goes into the context's counters.
int drain_slot(msw_ctx* ctx, Slot& s) {
    if (!s.busy) return MSW_OK;
    s.busy = false;
    HIP_TRY(hipEventSynchronize(s.direct_out ? s.k_end : s.done));
    add_kernel_interval(ctx, s.k_start, s.k_end);
    if (s.by_slot) {  // length-bucketed chunk: slot k holds pair h_order[k]
        int32_t* sc = s.out.score + s.first;
        for (uint64_t k = 0; k < s.count; ++k) sc[s.h_order[k]] = s.h_score[k];
        if (s.out.end_i) {
            int16_t *ei = s.out.end_i + s.first, *ej = s.out.end_j + s.first;
            for (uint64_t k = 0; k < s.count; ++k) {
                ei[s.h_order[k]] = s.h_ei[k];
                ej[s.h_order[k]] = s.h_ej[k];
            }
        }
        return MSW_OK;
    }
    memcpy(s.out.score + s.first, s.h_score, s.count * sizeof(int32_t));
    if (s.out.end_i) memcpy(s.out.end_i + s.first, s.h_ei, s.count * sizeof(int16_t));
    if (s.out.end_j) memcpy(s.out.end_j + s.first, s.h_ej, s.count * sizeof(int16_t));
    return MSW_OK;
}

// Drain the busy slots whose ticket is <= `ticket` (all: UINT64_MAX) oldest
// chunk first, so the kernel-time union sees its intervals in start order.
int drain_through(msw_ctx* ctx, uint64_t ticket) {
    for (;;) {
        Slot* next = nullptr;
        for (Slot& s : ctx->slots)
            if (s.busy && s.ticket <= ticket && (!next || s.seq < next->seq)) next = &s;
        if (!next) return MSW_OK;
        const int rc = drain_slot(ctx, *next);
        if (rc) return rc;
    }
}

int validate_batch(const msw_batch_t* b, const msw_out_t* out, const Scheme& sch) {
    if (!b || !out) return fail(MSW_E_INVALID, "batch/out is NULL");
    if (b->n_pairs == 0) return MSW_OK;
    if (!b->reads || !b->wins || !b->read_len || !b->win_len || !out->score)
        return fail(MSW_E_INVALID, "NULL array in batch/out");
    if (sch.coords && (!out->end_i || !out->end_j))
        return fail(MSW_E_INVALID, "want_coords set but end_i/end_j is NULL");
    if (b->n_pairs > 0xFFFFFFFFull) return fail(MSW_E_RANGE, "n_pairs > 2^32-1");
    return MSW_OK;
}

// Host-memory batch of either form: pairs (reads + windows) or reads against
// a genome-resident window source (wins == nullptr, genome + win_pos set).
struct HostBatch {
    const uint8_t* reads = nullptr;
    const uint16_t* read_len = nullptr;
    uint32_t read_stride = 0;
    const uint8_t* wins = nullptr;
    const uint16_t* win_len = nullptr;
    uint32_t win_stride = 0;
    const msw_genome* genome = nullptr;
    const int64_t* win_pos = nullptr;
    uint64_t n = 0;
};

// True when [p, p + bytes) lies in page-locked host memory (hipHostMalloc /
// hipHostRegister): such arrays are DMA'd directly, without staging.
// dev: the device address of p when pinned.
bool is_pinned(const void* p, size_t bytes, const uint8_t** dev) {
    *dev = nullptr;
    if (!p || !bytes) return false;
    for (const void* q : {p, (const void*)((const uint8_t*)p + bytes - 1)}) {
        hipPointerAttribute_t a;
        memset(&a, 0, sizeof(a));
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (a.type != hipMemoryTypeHost) return false;
        if (q == p) *dev = (const uint8_t*)a.devicePointer;
    }
    return true;
}

inline uint32_t round16(uint32_t v) { return (v + 15u) & ~15u; }

// Window length actually scored in genome mode: clipped at the genome end,
// empty for positions outside it.
inline uint16_t genome_window(int64_t pos, uint16_t want, uint64_t glen) {
    const uint64_t p = (uint64_t)pos;  // negative positions wrap past glen
    const uint64_t room = p < glen ? glen - p : 0;
    return (uint16_t)std::min<uint64_t>(want, room);
}

// Copy `n` rows of `len` bytes from stride `src_stride` to `dst_stride`.
void repack_rows(uint8_t* dst, uint32_t dst_stride, const uint8_t* src, uint32_t src_stride, uint64_t n) {
    if (dst_stride == src_stride) {
        memcpy(dst, src, n * src_stride);
        return;
    }
    for (uint64_t i = 0; i < n; ++i) memcpy(dst + i * dst_stride, src + i * src_stride, dst_stride);
}

// MSW_HOST_TRACE=1 (Options::host_trace): per-call host phase times on
// stderr (tools / DESIGN.md 5).
struct HostTrace {
    bool on;
    explicit HostTrace(bool enabled) : on(enabled) {}
    double scan = 0, stage = 0, submit = 0, wait = 0;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    double lap() {
        const auto n = std::chrono::steady_clock::now();
        const double d = std::chrono::duration<double, std::micro>(n - t).count();
        t = n;
        return d;
    }
};

// Host loops compiled twice, AVX2 and baseline x86-64, picked at load time
// (the attribute means nothing to the gfx950 pass of this file).
#if defined(__HIP_DEVICE_COMPILE__)
#define MSW_HOST_SIMD
#else
#define MSW_HOST_SIMD __attribute__((target_clones("avx2", "default")))
#endif

// One pass over a chunk's per-pair arrays: the read lengths, the window
// lengths (genome mode: clipped at the genome end) and the positions into the
// slot's metadata block, and what the dispatch needs -- the length bounds and
// the cells and bytes.  Plain loops over the arrays (the compiler vectorises
// them; AVX2 where the host has it): ~10k pairs per microsecond.
struct ChunkScan {
    uint32_t lm = 0xFFFF, gm = 0, ln = 0xFFFF, gn = 0;
    uint64_t cells = 0, bytes = 0;
};

MSW_HOST_SIMD
void scan_lengths(const uint16_t* __restrict rl, const uint16_t* __restrict wl, uint64_t n, ChunkScan& c) {
    uint32_t lm = 0xFFFF, gm = 0, ln = 0xFFFF, gn = 0;
    uint64_t cells = 0, bytes = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t r = rl[i], w = wl[i];
        lm = std::min(lm, r);
        gm = std::max(gm, r);
        ln = std::min(ln, w);
        gn = std::max(gn, w);
        cells += r * w;
        bytes += r + w;
    }
    c.lm = lm, c.gm = gm, c.ln = ln, c.gn = gn, c.cells = cells, c.bytes = bytes;
}

MSW_HOST_SIMD
void clip_windows(const int64_t* __restrict pos, const uint16_t* __restrict want, uint64_t n, uint64_t glen,
                  uint16_t* __restrict out) {
    for (uint64_t i = 0; i < n; ++i) out[i] = genome_window(pos[i], want[i], glen);
}

MSW_HOST_SIMD
void max_u16(const uint16_t* __restrict a, uint64_t n, uint32_t& m) {
    uint32_t v = 0;
    for (uint64_t i = 0; i < n; ++i) v = std::max<uint32_t>(v, a[i]);
    m = v;
}

ChunkScan stage_meta(Slot& s, const HostBatch& b, uint64_t first, uint64_t cnt) {
    memcpy(s.h_rlen, b.read_len + first, cnt * sizeof(uint16_t));
    if (b.genome) {
        memcpy(s.h_pos, b.win_pos + first, cnt * sizeof(int64_t));
        clip_windows(b.win_pos + first, b.win_len + first, cnt, b.genome->len, s.h_wlen);
    } else {
        memcpy(s.h_wlen, b.win_len + first, cnt * sizeof(uint16_t));
    }
    ChunkScan c;
    scan_lengths(s.h_rlen, s.h_wlen, cnt, c);
    return c;
}

// True when every pair of the chunk has one bucket key (bucket_chunk's: rows
// per lane of its read, 16-column blocks of its window, not long) -- decided
// from the bounds alone, both keys being monotone in the lengths.
bool single_key(const ChunkScan& c, bool all_long) {
    return !all_long && !is_long(c.gm, c.gn) &&
           msw::rows_per_lane(c.lm, false) == msw::rows_per_lane(c.gm, false) &&
           (c.ln + 15) / 16 == (c.gn + 15) / 16;
}

// Pinned-ness of the caller's arrays, remembered for the most recently used
// ranges (hipPointerGetAttributes twice per array and call is a visible share
// of a small call).  msw_host_free bumps g_host_free_epoch, which empties
// every context's cache at its next lookup, so a freed msw_host_alloc block
// whose address comes back as pageable memory is never taken for pinned
// (ADVICE r05).  Memory the caller pins or unpins itself must stay as it was
// while a call uses it, as for any DMA API; a stale verdict then only changes
// how a copy is made, never what it copies (hipMemcpyAsync accepts pageable
// and pinned sources alike, and the d2h copy kernel needs a device pointer
// for the block, which an unpinned one no longer has).
std::atomic<uint64_t> g_host_free_epoch{0};

bool pinned_cached(msw_ctx* ctx, const void* p, size_t bytes, const uint8_t** dev = nullptr) {
    const uint64_t ep = g_host_free_epoch.load(std::memory_order_acquire);
    if (ep != ctx->pinned_epoch) {
        ctx->pinned_used = 0;
        ctx->pinned_epoch = ep;
    }
    msw_ctx::PinnedRange* r = ctx->pinned_ranges;
    for (unsigned k = 0; k < ctx->pinned_used; ++k)
        if (r[k].p == p && r[k].bytes == bytes && p) {
            const msw_ctx::PinnedRange hit = r[k];
            for (unsigned q = k; q > 0; --q) r[q] = r[q - 1];  // move to front
            r[0] = hit;
            ++ctx->pinned_hits;
            if (dev) *dev = hit.dev;
            return hit.pinned;
        }
    ++ctx->pinned_misses;
    const uint8_t* d = nullptr;
    const bool pinned = is_pinned(p, bytes, &d);
    const unsigned n = std::min(ctx->pinned_used + 1, msw_ctx::kPinnedRanges);  // the least recent falls off
    for (unsigned q = n - 1; q > 0; --q) r[q] = r[q - 1];
    r[0] = {p, bytes, pinned, d};
    ctx->pinned_used = n;
    if (dev) *dev = d;
    return pinned;
}


int run_batch_impl(msw_ctx* ctx, const msw_scoring_t* sc, const HostBatch& b, msw_out_t* out,
                   uint64_t chunk_pairs, bool sync) {
    Scheme sch;
    int rc;
    if ((rc = make_scheme(sc, ctx->opt, &sch))) return rc;
    if (!out) return fail(MSW_E_INVALID, "out is NULL");
    const bool gmode = b.genome != nullptr;
    const uint64_t n = b.n;
    if (n == 0) return MSW_OK;
    if (!b.reads || !b.read_len || !b.win_len || !out->score || (gmode ? !b.win_pos : !b.wins))
        return fail(MSW_E_INVALID, "NULL array in batch/out");
    if (sch.coords && (!out->end_i || !out->end_j))
        return fail(MSW_E_INVALID, "want_coords set but end_i/end_j is NULL");
    if (n > 0xFFFFFFFFull) return fail(MSW_E_RANGE, "n_pairs > 2^32-1");
    if (gmode && (b.genome->ctx != ctx)) return fail(MSW_E_INVALID, "genome belongs to another context");
    if ((rc = set_device(ctx))) return rc;
    HostTrace tr(ctx->opt.host_trace);
    // Host-side range checks over the whole batch first: fail before any launch.
    // (genome mode bounds the requested window lengths: a clipped window is
    // never longer, and the positions need not be read here)
    uint32_t gm = 0, gn = 0;
    max_u16(b.read_len, n, gm);
    max_u16(b.win_len, n, gn);
    if (gm > b.read_stride || (!gmode && gn > b.win_stride))
        return fail(MSW_E_INVALID, "length exceeds stride (max read %u / stride %u, max window %u / stride %u)",
                    gm, b.read_stride, gn, b.win_stride);
    if ((rc = check_bounds(sch, gm, gn))) return rc;

    // Direct DMA from pinned caller arrays; otherwise stage through the slot's
    // pinned buffers with rows repacked to 16-byte-rounded strides.
    const uint8_t *g_reads = nullptr, *g_wins = nullptr;  // their device addresses
    const bool d_reads = pinned_cached(ctx, b.reads, n * b.read_stride, &g_reads);
    const bool d_wins = !gmode && pinned_cached(ctx, b.wins, n * b.win_stride, &g_wins);
    const uint32_t rs = d_reads ? b.read_stride : std::min(b.read_stride, std::max(16u, round16(gm)));
    const uint32_t ws = gmode ? std::max(16u, round16(gn))
                              : (d_wins ? b.win_stride : std::min(b.win_stride, std::max(16u, round16(gn))));
    if (tr.on) tr.scan += tr.lap();

    const uint64_t chunk = chunk_pairs ? chunk_pairs : ctx->opt.chunk;
    // A multi-chunk call pipelines its own chunks: copies on the copy stream,
    // kernels alternating between the two compute streams, results back on
    // the d2h stream.  A one-chunk call keeps its kernels and results on one
    // compute stream (async calls alternate it, so consecutive calls
    // overlap; a synchronous call uploads there too) and its kernels store
    // the results straight into the slot's mapped host block (no copy, no
    // event after the kernels but the timing one).
    const bool multi_chunk = n > chunk;
    const bool alternate = multi_chunk || !sync;
    const bool direct_out = !multi_chunk;
    // the copy / second compute / d2h streams: created by the first call that uses them
    if (alternate && !ctx->copy && (rc = aux_streams(ctx))) return rc;
    // Genome mode: a chunk of one bucket that the model puts in the pairs
    // layout with <= 16 rows per lane reads its windows straight from the
    // resident genome (GEN kernel instances: no cut launch, one dependent
    // step fewer per chunk); other chunks (several buckets, long pairs, other
    // layouts) cut a window slab first.
    const bool all_long = ctx->opt.force_long;
    const bool genome_ok = gmode && !all_long;
    uint64_t fused_chunks = 0;
    std::vector<Bucket> buckets;
    uint64_t c = 0;
    // A short first chunk starts the GPU early; with chunks of more than 64k
    // pairs the chunks after it double up to `chunk`, so each chunk's upload
    // hides under the kernel of the one before (a large chunk straight after
    // a small one left the GPU idle while it uploaded) and the large ones
    // still reach the narrow lane groups.  1M config-3 pairs
    // from pinned memory, genome form (tools/h2h_sweep.py,
    // profiles/r05/h2h/chunk_ramp.jsonl): 131k / 262k / 524k chunks 8.29 /
    // 8.49 / 9.41-9.49 ms -> 7.99 / 7.97-8.02 / 8.26-8.56; at 32k the ramp's
    // extra chunk cost 1 % (7.92 -> 8.01), so smaller chunks keep the old
    // schedule.
    const bool ramp = chunk > 65536;
    uint64_t next_chunk = n > chunk ? std::max<uint64_t>(std::min<uint64_t>(chunk, 8192), chunk / 8) : chunk;
    for (uint64_t first = 0, cnt = 0; first < n; first += cnt, ++c) {
        const uint64_t this_chunk = next_chunk;
        next_chunk = ramp ? std::min<uint64_t>(chunk, 2 * next_chunk) : chunk;
        cnt = std::min(this_chunk, n - first);
        // Slots alternate across calls too, so consecutive async calls overlap.
        const uint64_t seq = ctx->slot_seq++;
        Slot& s = ctx->slots[seq % msw_ctx::kSlots];
        hipStream_t cs = (alternate && (seq & 1)) ? ctx->compute2 : ctx->compute;
        if (tr.on) tr.submit += tr.lap();
        if ((rc = drain_slot(ctx, s))) return rc;  // the slot's previous chunk must be out before reuse
        if (tr.on) tr.wait += tr.lap();
        if ((rc = ensure_slot(s, cnt, (size_t)cnt * rs, (size_t)cnt * ws))) return rc;
        set_views(s, cnt);
        // Bulk rows: DMA'd from the caller's memory when pinned, else staged.
        const uint8_t* src_reads = b.reads + first * b.read_stride;
        if (!d_reads) {
            repack_rows(s.h_reads, rs, src_reads, b.read_stride, cnt);
            src_reads = s.h_reads;
        }
        const uint8_t* src_wins = nullptr;
        if (!gmode) {
            src_wins = b.wins + first * b.win_stride;
            if (!d_wins) {
                repack_rows(s.h_wins, ws, src_wins, b.win_stride, cnt);
                src_wins = s.h_wins;
            }
        }
        // Metadata block: lengths (effective window lengths in genome mode),
        // positions; the slot order only for a chunk of several buckets.
        const ChunkScan cs_ = stage_meta(s, b, first, cnt);
        bool uniform;
        if (single_key(cs_, all_long)) {  // fixed-length reads and windows, the common case: no sort
            buckets.assign(1, Bucket{0, (uint32_t)cnt, cs_.gm, cs_.gn});
            uniform = true;
        } else {
            uint32_t lens[4];
            bucket_chunk(s.h_rlen, s.h_wlen, cnt, s.h_order, buckets, lens, all_long);
            // One read-length bucket: order only matters if windows vary a lot;
            // long pairs of spread read lengths keep their heaviest-first order.
            uniform = buckets.size() == 1 && lens[3] - lens[2] < 16 &&
                      (!buckets[0].long_pairs || lens[1] - lens[0] < 64);
        }
        const bool fused = genome_ok && uniform && genome_windows_ok(cnt, cs_.gm, cs_.gn, sch, ctx->cu_count);
        fused_chunks += fused ? 1 : 0;
        if (tr.on) tr.stage += tr.lap();
        // [pos | rlen | wlen | order]: the contiguous part this chunk uses
        const size_t meta_lo = gmode ? 0 : 8 * cnt, meta_hi = (uniform ? 12 : 16) * cnt;
        // A one-chunk call pulls its rows and metadata from pinned host
        // memory into the slot with one copy kernel on its compute stream,
        // ahead of its scoring launch: no DMA engine and no event between
        // them.  (The DMA form -- uploads on the copy stream, the kernel
        // behind an event -- ran the 10k-pair stream at 57 us per batch:
        // reads and metadata copies 33.6 + 8.0 us back to back on the DMA
        // engine and ~22 us from an upload's end to its kernel's start,
        // kernels never overlapping; profiles/r06/host/stream_trace/.)
        // Sources must share the slot buffers' alignment mod 16.
        const uint8_t* g_src_reads = d_reads ? g_reads + first * b.read_stride : s.g_reads;
        const uint8_t* g_src_wins = gmode ? nullptr : (d_wins ? g_wins + first * b.win_stride : s.g_wins);
        const bool pull = !multi_chunk && g_src_reads && (gmode || g_src_wins) &&
                          (((uintptr_t)g_src_reads ^ (uintptr_t)s.d_reads) & 15u) == 0 &&
                          (gmode || (((uintptr_t)g_src_wins ^ (uintptr_t)s.d_wins) & 15u) == 0);
        if (pull) {
            msw::PullRanges pr{};
            pr.dst[0] = s.d_reads;
            pr.src[0] = g_src_reads;
            pr.bytes[0] = cnt * rs;
            if (!gmode) {
                pr.dst[1] = s.d_wins;
                pr.src[1] = g_src_wins;
                pr.bytes[1] = cnt * ws;
            }
            pr.dst[2] = s.d_meta + meta_lo;
            pr.src[2] = s.g_meta + meta_lo;
            pr.bytes[2] = meta_hi - meta_lo;
            // (The copy on the copy stream running ahead, the kernels on one
            // compute stream behind an event: 58.3 vs 55.1 us per batch,
            // profiles/r06/host/pull_ahead_ab.jsonl.)
            HIP_TRY(msw::launch_pull_copy(pr, cs));
            if (gmode && !fused)
                HIP_TRY(msw::launch_cut_windows(b.genome->d_seq, b.genome->len, s.d_pos, s.d_wlen, s.d_wins, nullptr,
                                                ws, cnt, cs));
        } else {
            // Multi-chunk calls: H2D on the copy stream, kernels on the
            // compute streams (an event orders each kernel after its chunk's
            // upload), results back on the d2h stream -- chunk k+1's uploads
            // and chunk k-1's readback overlap chunk k's kernel.  (One-chunk
            // calls whose sources are misaligned: DMA'd on the call's own
            // stream.)
            hipStream_t up = multi_chunk ? ctx->copy : cs;
            HIP_TRY(hipMemcpyAsync(s.d_reads, src_reads, cnt * rs, hipMemcpyHostToDevice, up));
            if (!gmode) HIP_TRY(hipMemcpyAsync(s.d_wins, src_wins, cnt * ws, hipMemcpyHostToDevice, up));
            HIP_TRY(hipMemcpyAsync(s.d_meta + meta_lo, s.h_meta + meta_lo, meta_hi - meta_lo, hipMemcpyHostToDevice,
                                   up));
            if (gmode && !fused)
                HIP_TRY(msw::launch_cut_windows(b.genome->d_seq, b.genome->len, s.d_pos, s.d_wlen, s.d_wins, nullptr,
                                                ws, cnt, up));
            if (multi_chunk) {
                HIP_TRY(hipEventRecord(s.uploaded, ctx->copy));
                HIP_TRY(hipStreamWaitEvent(cs, s.uploaded, 0));
            }
        }
        if (uniform) {
            buckets.resize(1);
            buckets[0].begin = 0;
        }
        s.k_score = direct_out ? s.h_score : s.d_score;
        s.k_ei = direct_out ? s.h_ei : s.d_ei;
        s.k_ej = direct_out ? s.h_ej : s.d_ej;
        HIP_TRY(hipEventRecord(s.k_start, cs));
        if ((rc = launch_buckets(ctx, sch, s, cnt, buckets, !uniform, rs, ws, cs, fused ? b.genome : nullptr)))
            return rc;
        HIP_TRY(hipEventRecord(s.k_end, cs));
        ctx->stats.launches += 1;
        ctx->stats.pairs += cnt;
        ctx->stats.cells += cs_.cells;
        ctx->stats.alg_bytes += cs_.bytes + cnt * (sch.coords ? 8u : 4u);
        if (!direct_out) {
            hipStream_t down = cs;
            if (multi_chunk) {
                HIP_TRY(hipEventRecord(s.computed, cs));
                HIP_TRY(hipStreamWaitEvent(ctx->d2h, s.computed, 0));
                down = ctx->d2h;
            }
            HIP_TRY(hipMemcpyAsync(s.h_res, s.d_res, (sch.coords ? kResBytesPerPair : 4) * cnt,
                                   hipMemcpyDeviceToHost, down));
            HIP_TRY(hipEventRecord(s.done, down));
        }
        s.busy = true;
        s.direct_out = direct_out;
        s.by_slot = !uniform;
        s.ticket = ctx->next_ticket;  // the ticket an async call returns
        s.seq = seq;
        s.first = first;
        s.count = cnt;
        s.out = *out;
        if (!sch.coords) { s.out.end_i = nullptr; s.out.end_j = nullptr; }
    }
    if (tr.on) tr.submit += tr.lap();  // the last chunk's HIP calls
    if (sync) {
        if ((rc = drain_through(ctx, UINT64_MAX))) return rc;
        if (tr.on) tr.wait += tr.lap();
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return fail(MSW_E_DEVICE, "kernel failure: %s", hipGetErrorString(e));
    }
    if (tr.on)
        fprintf(stderr,
                "[msw host] pairs=%llu chunks=%llu direct(reads=%d wins=%d out=%d) genome_chunks=%llu rs=%u ws=%u "
                "last_launch(layout=%s G=%u KR=%u) scan=%.1fus stage=%.1fus submit=%.1fus wait=%.1fus "
                "pinned_cache(hits=%llu misses=%llu)\n",
                (unsigned long long)n, (unsigned long long)c, (int)d_reads, (int)d_wins, (int)direct_out,
                (unsigned long long)fused_chunks, rs, ws,
                ctx->last_layout == msw::Layout::kSplit ? "split" : (ctx->last_layout == msw::Layout::kMixed ? "mixed" : "pairs"),
                ctx->last_group_lanes, ctx->last_kr,
                tr.scan, tr.stage, tr.submit, tr.wait, (unsigned long long)ctx->pinned_hits,
                (unsigned long long)ctx->pinned_misses);
    return MSW_OK;
}


// A call that fails after submitting some of its chunks must not leave them
// behind: they point at the caller's output arrays, and a later msw_wait or
// slot reuse would drain them there (the caller may have freed them by then).
// The streams are synchronised, the call's chunks dropped, and its ticket
// number consumed so no later call shares it.
int run_batch(msw_ctx* ctx, const msw_scoring_t* sc, const HostBatch& b, msw_out_t* out, uint64_t chunk_pairs,
              bool sync) {
    if (!ctx) return fail(MSW_E_INVALID, "ctx is NULL");
    const uint64_t ticket = ctx->next_ticket;
    const int rc = run_batch_impl(ctx, sc, b, out, chunk_pairs, sync);
    if (rc == MSW_OK) return rc;
    bool dropped = false;
    for (Slot& s : ctx->slots) dropped = dropped || (s.busy && s.ticket == ticket);
    if (dropped) {
        const std::string msg = g_last_error;
        for (hipStream_t st : {ctx->copy, ctx->compute, ctx->compute2, ctx->d2h, ctx->side})
            if (st) (void)hipStreamSynchronize(st);
        for (Slot& s : ctx->slots)
            if (s.busy && s.ticket == ticket) s.busy = false;
        ctx->next_ticket++;
        g_last_error = msg;
    }
    return rc;
}

HostBatch pairs_batch(const msw_batch_t& b) {
    HostBatch h;
    h.reads = b.reads;
    h.read_len = b.read_len;
    h.read_stride = b.read_stride;
    h.wins = b.wins;
    h.win_len = b.win_len;
    h.win_stride = b.win_stride;
    h.n = b.n_pairs;
    return h;
}

HostBatch reads_batch(const msw_read_batch_t& b, const msw_genome* g) {
    HostBatch h;
    h.reads = b.reads;
    h.read_len = b.read_len;
    h.read_stride = b.read_stride;
    h.win_len = b.win_len;
    h.genome = g;
    h.win_pos = b.win_pos;
    h.n = b.n_pairs;
    return h;
}

}  // namespace

extern "C" {

const char* msw_last_error(void) { return g_last_error.c_str(); }

const char* msw_version(void) { return "msw 0.1.0 (gfx950, HIP)"; }

int msw_device_count(int* n) {
    if (!n) return fail(MSW_E_INVALID, "n is NULL");
    *n = 0;
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess || c == 0) return fail(MSW_E_NODEVICE, "no GPU: %s", hipGetErrorString(e));
    *n = c;
    return MSW_OK;
}

int msw_device_info(int ordinal, msw_device_info_t* out) {
    if (!out) return fail(MSW_E_INVALID, "out is NULL");
    int n = 0;
    int rc = msw_device_count(&n);
    if (rc) return rc;
    if (ordinal < 0 || ordinal >= n) return fail(MSW_E_INVALID, "device %d out of range [0,%d)", ordinal, n);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, ordinal));
    memset(out, 0, sizeof(*out));
    snprintf(out->name, sizeof(out->name), "%s", prop.name);
    if (!out->name[0])  // the marketing name can be empty under ROCm: name the target instead
        snprintf(out->name, sizeof(out->name), "AMD Instinct GPU (%s, %d CUs)", prop.gcnArchName,
                 prop.multiProcessorCount);
    snprintf(out->arch, sizeof(out->arch), "%s", prop.gcnArchName);
    out->mem_bytes = prop.totalGlobalMem;
    out->max_wg = (uint32_t)prop.maxThreadsPerBlock;
    out->cu_count = (uint32_t)prop.multiProcessorCount;
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (hipSetDevice(ordinal) == hipSuccess) {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess) out->mem_free_bytes = fr;
        (void)hipSetDevice(cur);
    }
    return MSW_OK;
}

int msw_ctx_create(int ordinal, msw_ctx** out) { return msw_ctx_create_ex(ordinal, 0u, out); }

int msw_ctx_create_ex(int ordinal, unsigned flags, msw_ctx** out) {
    if (!out) return fail(MSW_E_INVALID, "out is NULL");
    if (flags & ~MSW_CTX_LEAN) return fail(MSW_E_INVALID, "unknown context flags 0x%x", flags);
    *out = nullptr;
    int n = 0;
    int rc = msw_device_count(&n);
    if (rc) return rc;
    if (ordinal < 0 || ordinal >= n) return fail(MSW_E_INVALID, "device %d out of range [0,%d)", ordinal, n);
    msw_ctx* c = new msw_ctx();
    c->device = ordinal;
    c->opt = read_options();
    hipError_t e = hipSetDevice(ordinal);
    hipDeviceProp_t prop;
    if (e == hipSuccess && hipGetDeviceProperties(&prop, ordinal) == hipSuccess && prop.multiProcessorCount > 0)
        c->cu_count = prop.multiProcessorCount;
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->compute, hipStreamNonBlocking);
    if (e == hipSuccess && !(flags & MSW_CTX_LEAN) && aux_streams(c) != MSW_OK) e = hipErrorOutOfMemory;
    if (e == hipSuccess) e = hipEventCreate(&c->epoch);
    if (e == hipSuccess) e = hipEventRecord(c->epoch, c->compute);
    if (e != hipSuccess) {
        delete c;
        return fail(MSW_E_DEVICE, "context creation on device %d failed: %s", ordinal, hipGetErrorString(e));
    }
    *out = c;
    return MSW_OK;
}

void msw_ctx_destroy(msw_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->compute) (void)hipStreamSynchronize(ctx->compute);
    if (ctx->compute2) (void)hipStreamSynchronize(ctx->compute2);
    if (ctx->copy) (void)hipStreamSynchronize(ctx->copy);
    if (ctx->d2h) (void)hipStreamSynchronize(ctx->d2h);
    if (ctx->side) (void)hipStreamSynchronize(ctx->side);
    for (Slot& s : ctx->slots) {
        if (s.uploaded) (void)hipEventDestroy(s.uploaded);
        if (s.computed) (void)hipEventDestroy(s.computed);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.k_start) (void)hipEventDestroy(s.k_start);
        if (s.k_end) (void)hipEventDestroy(s.k_end);
        free_slot(s);
    }
    if (ctx->c_k0) (void)hipEventDestroy(ctx->c_k0);
    if (ctx->c_k1) (void)hipEventDestroy(ctx->c_k1);
    (void)hipFree(ctx->c_s1);
    (void)hipFree(ctx->c_s2);
    (void)hipFree(ctx->c_res);
    for (auto& r : ctx->rscratch) {
        (void)hipFree(r.wins);
        (void)hipFree(r.wlen);
    }
    for (hipStream_t st : ctx->user_streams) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
    }
    for (auto& t : ctx->dev_timings) {
        (void)hipEventDestroy(t.k0);
        (void)hipEventDestroy(t.k1);
    }
    for (hipEvent_t e : ctx->free_events) (void)hipEventDestroy(e);
    for (auto& kv : ctx->fences) (void)hipEventDestroy(kv.second);
    if (ctx->epoch) (void)hipEventDestroy(ctx->epoch);
    if (ctx->epoch_next) (void)hipEventDestroy(ctx->epoch_next);
    if (ctx->compute) (void)hipStreamDestroy(ctx->compute);
    if (ctx->compute2) (void)hipStreamDestroy(ctx->compute2);
    if (ctx->copy) (void)hipStreamDestroy(ctx->copy);
    if (ctx->d2h) (void)hipStreamDestroy(ctx->d2h);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    delete ctx;
}

int msw_align_batch(msw_ctx* ctx, const msw_scoring_t* sc, const msw_batch_t* batch, msw_out_t* out,
                    uint64_t chunk_pairs) {
    if (!batch) return fail(MSW_E_INVALID, "batch is NULL");
    return run_batch(ctx, sc, pairs_batch(*batch), out, chunk_pairs, true);
}

int msw_align_batch_async(msw_ctx* ctx, const msw_scoring_t* sc, const msw_batch_t* batch, msw_out_t* out,
                          uint64_t chunk_pairs, uint64_t* ticket) {
    if (!ticket) return fail(MSW_E_INVALID, "ticket is NULL");
    if (!batch) return fail(MSW_E_INVALID, "batch is NULL");
    int rc = run_batch(ctx, sc, pairs_batch(*batch), out, chunk_pairs, false);
    if (rc) return rc;
    *ticket = ctx->next_ticket++;
    return MSW_OK;
}

int msw_wait(msw_ctx* ctx, uint64_t ticket) {
    if (!ctx) return fail(MSW_E_INVALID, "ctx is NULL");
    if (ticket == 0 || ticket >= ctx->next_ticket) return fail(MSW_E_INVALID, "unknown ticket %llu", (unsigned long long)ticket);
    int rc = set_device(ctx);
    if (rc) return rc;
    // Drain the chunks of this ticket and of every earlier one (tickets are
    // enqueued in order on the same streams); later calls stay in flight.
    if ((rc = drain_through(ctx, ticket))) return rc;
    ctx->done_ticket = std::max(ctx->done_ticket, ticket);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MSW_E_DEVICE, "kernel failure: %s", hipGetErrorString(e));
    return MSW_OK;
}

// Diagnostics only (MSW_WAVE_TRACE=file, read by tools/wave_trace.py): the
// launch records per-block clocks and placement and appends one record
// {u64 n_blocks, u64 layout | G << 8 | pairs_blocks << 16, n_blocks x 4 u64}
// to the file.  Synchronous.
static int traced_launch(msw::SwParams p, const Scheme& sch, uint32_t max_read_len, const LaunchPlan& plan,
                         hipStream_t st, const char* path) {
    const uint64_t n_blocks = p.n_slots / 4 + 2;  // the split layout's count bounds every grid
    uint64_t* d = nullptr;
    HIP_TRY(hipMalloc(&d, n_blocks * 4 * sizeof(uint64_t)));
    (void)hipMemsetAsync(d, 0, n_blocks * 4 * sizeof(uint64_t), st);
    p.trace = d;
    hipError_t e = msw::launch_sw(p, sch.affine, sch.coords, max_read_len, plan.layout, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    std::vector<uint64_t> h(n_blocks * 4);
    if (e == hipSuccess) e = hipMemcpy(h.data(), d, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(MSW_E_DEVICE, "traced launch: %s", hipGetErrorString(e));
    FILE* f = fopen(path, "ab");
    if (!f) return fail(MSW_E_INVALID, "cannot open MSW_WAVE_TRACE file %s", path);
    const uint64_t hdr[2] = {n_blocks, (uint64_t)plan.layout | ((uint64_t)plan.group_lanes << 8) |
                                           ((uint64_t)plan.pairs_blocks << 16)};
    fwrite(hdr, sizeof(hdr), 1, f);
    fwrite(h.data(), sizeof(uint64_t), h.size(), f);
    fclose(f);
    return MSW_OK;
}

// One packed-kernel launch of p (pointers, strides / window source and
// n_slots set) under the given length bounds: layout from the makespan model.
static int launch_packed(msw_ctx* ctx, const Scheme& sch, msw::SwParams& p, uint32_t max_read_len,
                         uint32_t max_win_len, hipStream_t st) {
    p.lds_stride = msw::stream_stride(max_win_len);
    p.f16_ok = f16_fits(sch, max_read_len, max_win_len) ? 1u : 0u;
    const LaunchPlan plan = choose_layout(p.n_slots, max_read_len, max_win_len, sch, ctx->cu_count);
    p.pairs_blocks = plan.pairs_blocks;
    p.group_lanes = plan.group_lanes;
    p.groups = plan.groups;
    if (!ctx->opt.wave_trace.empty()) return traced_launch(p, sch, max_read_len, plan, st, ctx->opt.wave_trace.c_str());
    HIP_TRY(msw::launch_sw(p, sch.affine, sch.coords, max_read_len, plan.layout, st));
    return MSW_OK;
}

int msw_align_batch_device(msw_ctx* ctx, const msw_scoring_t* sc, const msw_batch_t* b, msw_out_t* out,
                           uint32_t max_read_len, uint32_t max_win_len, void* stream) {
    if (!ctx) return fail(MSW_E_INVALID, "ctx is NULL");
    Scheme sch;
    int rc;
    if ((rc = make_scheme(sc, ctx->opt, &sch))) return rc;
    if ((rc = validate_batch(b, out, sch))) return rc;
    if (b->n_pairs == 0) return MSW_OK;
    if ((rc = check_bounds(sch, max_read_len, max_win_len))) return rc;
    if (max_read_len > b->read_stride || max_win_len > b->win_stride)
        return fail(MSW_E_INVALID, "max length exceeds stride");
    if ((rc = set_device(ctx))) return rc;
    msw::SwParams p = base_params(sch);
    p.reads = b->reads;
    p.wins = b->wins;
    p.read_len = b->read_len;
    p.win_len = b->win_len;
    p.order = nullptr;
    p.score = out->score;
    p.end_i = sch.coords ? out->end_i : nullptr;
    p.end_j = sch.coords ? out->end_j : nullptr;
    p.read_stride = b->read_stride;
    p.win_stride = b->win_stride;
    p.n_slots = (uint32_t)b->n_pairs;
    hipStream_t st = stream ? (hipStream_t)stream : ctx->compute;
    // bounds past the packed kernels: the whole batch on the long-pair kernel
    if (ctx->opt.force_long || is_long(max_read_len, max_win_len))
        return launch_long(sch, p, b->n_pairs, max_read_len, max_win_len, false, ctx->cu_count, st);
    p.win_vec = msw::vec_ok(p.wins, p.win_stride);
    return launch_packed(ctx, sch, p, max_read_len, max_win_len, st);
}

}  // extern "C"

struct msw_plan {
    const msw_ctx* ctx = nullptr;  // identity only: destroy must not touch the context
    int device = 0;
    Scheme sch{};
    uint64_t n = 0;
    uint32_t max_m = 0, max_n = 0;
    uint32_t* d_order = nullptr;
    // Non-identity order: the kernel writes results in slot order into d_tmp
    // (score i32 | end_i i16 | end_j i16, n each) and a gather pass puts them
    // in pair order through d_inv (pair -> slot): coalesced stores instead of
    // one scattered 4-byte store per pair.
    bool identity = true;
    uint32_t* d_inv = nullptr;
    uint8_t* d_tmp = nullptr;
    uint32_t* d_slot_lens = nullptr;  // read_len | win_len << 16 in slot order
    bool multi = false;
    msw::MultiTable table{};
    bool wide = false;  // the KR 17..24 buckets as one launch (wide_table)
    msw::MultiTable wide_table{};
    // packed-kernel buckets launched on their own (all of them without a
    // multi table, else the KR 17..24 ones), each with its layout
    std::vector<std::pair<Bucket, LaunchPlan>> singles;
    bool has_long = false;
    Bucket longs{};                   // pairs beyond the packed kernels (sw_long_kernel)
};

extern "C" {

int msw_plan_create(msw_ctx* ctx, const msw_scoring_t* sc, const uint16_t* read_len, const uint16_t* win_len,
                    uint64_t n_pairs, msw_plan** out) {
    if (!ctx || !out) return fail(MSW_E_INVALID, "ctx/out is NULL");
    *out = nullptr;
    Scheme sch;
    int rc;
    if ((rc = make_scheme(sc, ctx->opt, &sch))) return rc;
    if (n_pairs && (!read_len || !win_len)) return fail(MSW_E_INVALID, "NULL length array");
    if (n_pairs > 0xFFFFFFFFull) return fail(MSW_E_RANGE, "n_pairs > 2^32-1");
    uint32_t gm = 0, gn = 0;
    for (uint64_t i = 0; i < n_pairs; ++i) {
        gm = std::max<uint32_t>(gm, read_len[i]);
        gn = std::max<uint32_t>(gn, win_len[i]);
    }
    if ((rc = check_bounds(sch, gm, gn))) return rc;
    if ((rc = set_device(ctx))) return rc;
    msw_plan* pl = new msw_plan();
    pl->ctx = ctx;
    pl->device = ctx->device;
    pl->sch = sch;
    pl->n = n_pairs;
    pl->max_m = gm;
    pl->max_n = gn;
    if (n_pairs) {
        std::vector<uint32_t> order(n_pairs);
        std::vector<Bucket> buckets;
        uint32_t lens[4];
        bucket_chunk(read_len, win_len, n_pairs, order.data(), buckets, lens, ctx->opt.force_long);
        const size_t n_short = short_buckets(buckets);
        if (n_short < buckets.size()) {
            pl->has_long = true;
            pl->longs = buckets.back();
        }
        const size_t n_multi = multi_buckets(buckets);
        pl->multi = use_multi(n_multi, ctx->opt);
        if (pl->multi) fill_multi(buckets, 0, n_multi, sch, pl->table);
        pl->wide = use_wide_multi(n_short - n_multi, ctx->opt);
        if (pl->wide) fill_multi(buckets, n_multi, n_short, sch, pl->wide_table);
        for (size_t bi = pl->multi ? n_multi : 0; bi < (pl->wide ? n_multi : n_short); ++bi)
            pl->singles.push_back({buckets[bi], choose_layout(buckets[bi].count, buckets[bi].max_m, buckets[bi].max_n,
                                                              sch, ctx->cu_count)});
        rc = grow_dev(&pl->d_order, n_pairs);
        hipError_t e = rc ? hipSuccess : hipMemcpy(pl->d_order, order.data(), n_pairs * sizeof(uint32_t),
                                                   hipMemcpyHostToDevice);
        if (!rc && e != hipSuccess) rc = fail(MSW_E_DEVICE, "plan upload: %s", hipGetErrorString(e));
        for (uint64_t k = 0; k < n_pairs && pl->identity; ++k) pl->identity = order[k] == (uint32_t)k;
        if (!rc && !pl->identity) {
            std::vector<uint32_t> inv(n_pairs), lens(n_pairs);
            for (uint64_t k = 0; k < n_pairs; ++k) {
                inv[order[k]] = (uint32_t)k;
                lens[k] = (uint32_t)read_len[order[k]] | ((uint32_t)win_len[order[k]] << 16);
            }
            if (!(rc = grow_dev(&pl->d_inv, n_pairs)) && !(rc = grow_dev(&pl->d_tmp, n_pairs * kResBytesPerPair)) &&
                !(rc = grow_dev(&pl->d_slot_lens, n_pairs))) {
                e = hipMemcpy(pl->d_inv, inv.data(), n_pairs * sizeof(uint32_t), hipMemcpyHostToDevice);
                if (e == hipSuccess)
                    e = hipMemcpy(pl->d_slot_lens, lens.data(), n_pairs * sizeof(uint32_t), hipMemcpyHostToDevice);
                if (e != hipSuccess) rc = fail(MSW_E_DEVICE, "plan upload: %s", hipGetErrorString(e));
            }
        }
        if (rc) {
            msw_plan_destroy(pl);
            return rc;
        }
    }
    *out = pl;
    return MSW_OK;
}

int msw_align_batch_planned(msw_ctx* ctx, const msw_plan* plan, const msw_batch_t* b, msw_out_t* out,
                            void* stream) {
    if (!ctx || !plan) return fail(MSW_E_INVALID, "ctx/plan is NULL");
    if (plan->ctx != ctx) return fail(MSW_E_INVALID, "plan belongs to another context");
    int rc;
    if ((rc = validate_batch(b, out, plan->sch))) return rc;
    if (b->n_pairs != plan->n)
        return fail(MSW_E_INVALID, "batch has %llu pairs, plan %llu", (unsigned long long)b->n_pairs,
                    (unsigned long long)plan->n);
    if (plan->n == 0) return MSW_OK;
    if (plan->max_m > b->read_stride || plan->max_n > b->win_stride)
        return fail(MSW_E_INVALID, "max length exceeds stride");
    if ((rc = set_device(ctx))) return rc;
    const Scheme& sch = plan->sch;
    msw::SwParams p = base_params(sch);
    p.reads = b->reads;
    p.wins = b->wins;
    p.read_len = b->read_len;
    p.win_len = b->win_len;
    p.order = plan->d_order;
    p.score = out->score;
    p.end_i = sch.coords ? out->end_i : nullptr;
    p.end_j = sch.coords ? out->end_j : nullptr;
    p.read_stride = b->read_stride;
    p.win_stride = b->win_stride;
    p.win_vec = msw::vec_ok(p.wins, p.win_stride);
    hipStream_t st = stream ? (hipStream_t)stream : ctx->compute;
    const uint64_t n = plan->n;
    int32_t* t_score = reinterpret_cast<int32_t*>(plan->d_tmp);
    int16_t* t_i = reinterpret_cast<int16_t*>(plan->d_tmp + 4 * n);
    int16_t* t_j = reinterpret_cast<int16_t*>(plan->d_tmp + 6 * n);
    if (!plan->identity) {  // slot-ordered lengths and results, gathered below
        p.out_by_slot = 1;
        p.out_slot_base = 0;
        p.slot_lens = plan->d_slot_lens;
        p.score = t_score;
        p.end_i = sch.coords ? t_i : nullptr;
        p.end_j = sch.coords ? t_j : nullptr;
    }
    SideFork side;
    if (plan->has_long) {  // the long pairs' slots come last: [longs.begin, n)
        msw::SwParams q = p;
        q.order = plan->d_order + plan->longs.begin;
        q.out_slot_base = plan->longs.begin;
        q.slot_lens = nullptr;
        const bool beside = plan->multi || plan->wide || !plan->singles.empty();
        if (beside && (rc = fork_side(ctx, st, side))) return rc;
        if ((rc = launch_long(sch, q, plan->longs.count, plan->longs.max_m, plan->longs.max_n, plan->longs.spread,
                              ctx->cu_count, beside ? ctx->side : st)))
            return rc;
    }
    if (plan->multi) {
        msw::SwParams q = p;
        q.group_lanes = 16;
        q.groups = 4;
        HIP_TRY(msw::launch_sw_multi(q, plan->table, sch.affine, sch.coords, st));
    }
    if (plan->wide) {
        msw::SwParams q = p;
        q.group_lanes = 16;
        q.groups = 4;
        HIP_TRY(msw::launch_sw_multi(q, plan->wide_table, sch.affine, sch.coords, st));
    }
    for (const auto& sb : plan->singles) {  // slots [b.begin, b.begin + count)
        const Bucket& b = sb.first;
        msw::SwParams q = p;
        q.order = plan->d_order + b.begin;
        q.out_slot_base = b.begin;
        q.n_slots = b.count;
        q.lds_stride = msw::stream_stride(b.max_n);
        q.f16_ok = f16_fits(sch, b.max_m, b.max_n) ? 1u : 0u;
        q.pairs_blocks = sb.second.pairs_blocks;
        q.group_lanes = sb.second.group_lanes;
        q.groups = sb.second.groups;
        HIP_TRY(msw::launch_sw(q, sch.affine, sch.coords, b.max_m, sb.second.layout, st));
    }
    if (side.ev && (rc = join_side(ctx, st, side))) return rc;
    if (!plan->identity)
        HIP_TRY(msw::launch_gather_results(plan->d_inv, t_score, t_i, t_j, out->score, sch.coords ? out->end_i : nullptr,
                                           sch.coords ? out->end_j : nullptr, n, st));
    return MSW_OK;
}

void msw_plan_destroy(msw_plan* plan) {
    if (!plan) return;
    if (plan->d_order || plan->d_inv || plan->d_tmp || plan->d_slot_lens) {
        (void)hipSetDevice(plan->device);
        for (void* q : {(void*)plan->d_order, (void*)plan->d_inv, (void*)plan->d_tmp, (void*)plan->d_slot_lens})
            if (q) (void)hipFree(q);
    }
    delete plan;
}

int msw_align_compat(msw_ctx* ctx, const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2, uint32_t wg,
                     uint32_t max_groups, int32_t* score) {
    if (!ctx || !score) return fail(MSW_E_INVALID, "ctx/score is NULL");
    *score = 0;
    const size_t L = std::min(n1, n2);
    if (L == 0) return MSW_OK;                                 // aligner.rs:414-416
    if (!s1 || !s2) return fail(MSW_E_INVALID, "NULL sequence");
    int rc = set_device(ctx);
    if (rc) return rc;
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, ctx->device));
    const uint32_t W = wg ? wg : std::min<uint32_t>((uint32_t)prop.maxThreadsPerBlock, 1024u);  // aligner.rs:422
    const uint64_t G = std::min<uint64_t>((L + W - 1) / W, max_groups ? max_groups : 1000000u);  // :423-424
    // aligner.rs:436-456: min(1,000,000 * 1024 work items, 80 % of memory / 3).
    size_t fr = 0, tot = 0;
    HIP_TRY(hipMemGetInfo(&fr, &tot));
    const uint64_t cap = std::min<uint64_t>(1024000000ull, (uint64_t)(tot * 0.8) / 3);
    if (L > cap)
        return fail(MSW_E_RANGE, "Sequence too large (%zu bytes), max allowed: %llu bytes (%llu MB)", L,
                    (unsigned long long)cap, (unsigned long long)(cap / (1024 * 1024)));
    if (L > ctx->c_cap) {
        if ((rc = grow_dev(&ctx->c_s1, L)) || (rc = grow_dev(&ctx->c_s2, L))) return rc;
        ctx->c_cap = L;
    }
    if (!ctx->c_res && (rc = grow_dev(&ctx->c_res, 1))) return rc;
    HIP_TRY(hipMemcpyAsync(ctx->c_s1, s1, L, hipMemcpyHostToDevice, ctx->compute));
    HIP_TRY(hipMemcpyAsync(ctx->c_s2, s2, L, hipMemcpyHostToDevice, ctx->compute));
    HIP_TRY(hipMemsetAsync(ctx->c_res, 0, sizeof(int32_t), ctx->compute));
    if (!ctx->c_k0) {
        HIP_TRY(hipEventCreate(&ctx->c_k0));
        HIP_TRY(hipEventCreate(&ctx->c_k1));
    }
    HIP_TRY(hipEventRecord(ctx->c_k0, ctx->compute));
    HIP_TRY(msw::launch_compat(ctx->c_s1, ctx->c_s2, ctx->c_res, L, W, G, ctx->compute));
    HIP_TRY(hipEventRecord(ctx->c_k1, ctx->compute));
    HIP_TRY(hipMemcpyAsync(score, ctx->c_res, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->compute));
    HIP_TRY(hipStreamSynchronize(ctx->compute));
    add_kernel_interval(ctx, ctx->c_k0, ctx->c_k1);
    ctx->stats.launches += 1;
    ctx->stats.alg_bytes += 2ull * L + 4;
    return MSW_OK;
}

int msw_genome_create(msw_ctx* ctx, const uint8_t* seq, uint64_t len, msw_genome** out) {
    if (!ctx || !out) return fail(MSW_E_INVALID, "ctx/out is NULL");
    *out = nullptr;
    if (len && !seq) return fail(MSW_E_INVALID, "seq is NULL");
    int rc = set_device(ctx);
    if (rc) return rc;
    msw_genome* g = new msw_genome();
    g->ctx = ctx;
    g->device = ctx->device;
    g->len = len;
    hipError_t e = hipMalloc((void**)&g->d_seq, len + msw::kGenomePad);
    if (e != hipSuccess) {
        delete g;
        return fail(MSW_E_NOMEM, "hipMalloc(%llu B) for the genome: %s", (unsigned long long)len, hipGetErrorString(e));
    }
    // on the compute stream (the call is synchronous; a --full-wgs worker
    // then never creates its copy stream)
    e = hipMemsetAsync(g->d_seq + len, 0, msw::kGenomePad, ctx->compute);
    if (e == hipSuccess && len) e = hipMemcpyAsync(g->d_seq, seq, len, hipMemcpyHostToDevice, ctx->compute);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->compute);
    if (e != hipSuccess) {
        msw_genome_destroy(g);
        return fail(MSW_E_DEVICE, "genome upload: %s", hipGetErrorString(e));
    }
    *out = g;
    return MSW_OK;
}

void msw_genome_destroy(msw_genome* g) {
    if (!g) return;
    if (g->d_seq) {
        (void)hipSetDevice(g->device);
        (void)hipFree(g->d_seq);
    }
    delete g;
}

uint64_t msw_genome_length(const msw_genome* g) { return g ? g->len : 0; }

int msw_genome_cut_device(msw_ctx* ctx, const msw_genome* g, const int64_t* win_pos, const uint16_t* win_len,
                          uint64_t n, uint8_t* wins, uint32_t win_stride, uint16_t* win_len_out, void* stream) {
    if (!ctx || !g) return fail(MSW_E_INVALID, "ctx/genome is NULL");
    if (g->ctx != ctx) return fail(MSW_E_INVALID, "genome belongs to another context");
    if (n == 0) return MSW_OK;
    if (!win_pos || !win_len || !wins) return fail(MSW_E_INVALID, "NULL array");
    if (win_stride == 0 || win_stride % 16 != 0 || ((uintptr_t)wins & 15) != 0)
        return fail(MSW_E_INVALID, "win_stride must be a non-zero multiple of 16 and wins 16-byte aligned");
    int rc = set_device(ctx);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : ctx->compute;
    HIP_TRY(msw::launch_cut_windows(g->d_seq, g->len, win_pos, win_len, wins, win_len_out, win_stride, n, st));
    return MSW_OK;
}

int msw_align_reads(msw_ctx* ctx, const msw_scoring_t* sc, const msw_genome* g, const msw_read_batch_t* batch,
                    msw_out_t* out, uint64_t chunk_pairs) {
    if (!batch || !g) return fail(MSW_E_INVALID, "batch/genome is NULL");
    return run_batch(ctx, sc, reads_batch(*batch, g), out, chunk_pairs, true);
}

int msw_align_reads_async(msw_ctx* ctx, const msw_scoring_t* sc, const msw_genome* g,
                          const msw_read_batch_t* batch, msw_out_t* out, uint64_t chunk_pairs, uint64_t* ticket) {
    if (!ticket) return fail(MSW_E_INVALID, "ticket is NULL");
    if (!batch || !g) return fail(MSW_E_INVALID, "batch/genome is NULL");
    int rc = run_batch(ctx, sc, reads_batch(*batch, g), out, chunk_pairs, false);
    if (rc) return rc;
    *ticket = ctx->next_ticket++;
    return MSW_OK;
}

int msw_align_reads_device(msw_ctx* ctx, const msw_scoring_t* sc, const msw_genome* g, const uint8_t* reads,
                           const uint16_t* read_len, uint32_t read_stride, const int64_t* win_pos, uint64_t n,
                           uint32_t window, uint32_t max_read_len, msw_out_t* out, uint16_t* win_len_out,
                           void* stream) {
    if (!ctx || !g) return fail(MSW_E_INVALID, "ctx/genome is NULL");
    if (g->ctx != ctx) return fail(MSW_E_INVALID, "genome belongs to another context");
    if (n == 0) return MSW_OK;
    if (!reads || !read_len || !win_pos || !out || !out->score) return fail(MSW_E_INVALID, "NULL array");
    if (window > (uint32_t)msw::kMaxLongLen) return fail(MSW_E_RANGE, "window %u > %d", window, msw::kMaxLongLen);
    int rc = set_device(ctx);
    if (rc) return rc;
    const uint32_t max_win = window ? window : std::min<uint32_t>(2u * max_read_len, (uint32_t)msw::kMaxWinLen);
    hipStream_t st = stream ? (hipStream_t)stream : ctx->compute;
    harvest_dev_timings(ctx, false);
    const uint32_t ws = std::max<uint32_t>(16u, (max_win + 15u) & ~15u);
    const size_t wbytes = (size_t)n * ws;
    msw_ctx::ReadsScratch* rs = nullptr;
    for (auto& r : ctx->rscratch)
        if (r.st == st) rs = &r;
    if (!rs) {
        ctx->rscratch.emplace_back();
        rs = &ctx->rscratch.back();
        rs->st = st;
    }
    if (wbytes > rs->wins_cap) {
        if ((rc = grow_dev(&rs->wins, wbytes + wbytes / 4))) return rc;
        rs->wins_cap = wbytes + wbytes / 4;
    }
    uint16_t* wlen = win_len_out;
    if (!wlen) {
        if (n > rs->wlen_cap) {
            if ((rc = grow_dev(&rs->wlen, (size_t)n + n / 4))) return rc;
            rs->wlen_cap = (size_t)n + n / 4;
        }
        wlen = rs->wlen;
    }
    HIP_TRY(msw::launch_cut_windows_for_reads(g->d_seq, g->len, win_pos, read_len, window, rs->wins, wlen, ws, n,
                                              st));
    msw_batch_t b{reads, rs->wins, read_len, wlen, read_stride, ws, n};
    msw_ctx::DevTiming t{take_event(ctx), take_event(ctx), n};
    if (!t.k0 || !t.k1) return fail(MSW_E_DEVICE, "hipEventCreate failed");
    HIP_TRY(hipEventRecord(t.k0, st));
    if ((rc = msw_align_batch_device(ctx, sc, &b, out, max_read_len, max_win, stream))) return rc;
    HIP_TRY(hipEventRecord(t.k1, st));
    ctx->dev_timings.push_back(t);
    return MSW_OK;
}

int msw_memcpy_d2h_async(msw_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream) {
    if (!ctx) return fail(MSW_E_INVALID, "ctx is NULL");
    int rc = set_device(ctx);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : ctx->compute;
    // Into pinned host memory the copy is a kernel on the caller's stream,
    // not a DMA: the copy engines serve every stream of the process from
    // shared in-order rings, so a DMA that waits on its stream's scoring
    // kernel holds up the copies other workers queued behind it (config 3
    // from FASTQ: one worker's result copies 2 ms late, behind the other's
    // next batch).  Source and destination that differ in
    // alignment mod 16 go by DMA: the kernel would copy them byte by byte
    // (ADVICE r05).
    if (bytes && (((uintptr_t)dst ^ (uintptr_t)src) & 15) == 0 && pinned_cached(ctx, dst, bytes)) {
        void* dp = nullptr;
        if (hipHostGetDevicePointer(&dp, dst, 0) == hipSuccess && dp) {
            HIP_TRY(msw::launch_d2h_copy(dp, src, bytes, st));
            return MSW_OK;
        }
        (void)hipGetLastError();
    }
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
    return MSW_OK;
}

void* msw_host_alloc(size_t bytes) {
    void* p = nullptr;
    // portable: the --full-wgs readers fill slabs that any GPU's context DMAs
    if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess) {
        fail(MSW_E_NOMEM, "hipHostMalloc(%zu) failed", bytes);
        return nullptr;
    }
    return p;
}

void msw_host_free(void* p) {
    if (!p) return;
    (void)hipHostFree(p);
    g_host_free_epoch.fetch_add(1, std::memory_order_release);  // every context's pinned cache is stale
}

void* msw_dev_alloc(msw_ctx* ctx, size_t bytes) {
    if (!ctx || set_device(ctx)) return nullptr;
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        fail(MSW_E_NOMEM, "hipMalloc(%zu) failed", bytes);
        return nullptr;
    }
    return p;
}

void msw_dev_free(msw_ctx* ctx, void* p) {
    if (ctx) (void)hipSetDevice(ctx->device);
    if (p) (void)hipFree(p);
}

int msw_memcpy_h2d(msw_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx) return fail(MSW_E_INVALID, "ctx is NULL");
    int rc = set_device(ctx);
    if (rc) return rc;
    HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return MSW_OK;
}

int msw_memcpy_d2h(msw_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx) return fail(MSW_E_INVALID, "ctx is NULL");
    int rc = set_device(ctx);
    if (rc) return rc;
    HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return MSW_OK;
}

int msw_ctx_prepare(msw_ctx* ctx, const msw_scoring_t* sc) {
    if (!ctx) return fail(MSW_E_INVALID, "ctx is NULL");
    Scheme sch;
    int rc;
    if ((rc = make_scheme(sc, ctx->opt, &sch))) return rc;
    if ((rc = set_device(ctx))) return rc;
    // one occupancy query per kernel module (translation unit): the query
    // loads the module; the shapes are any valid ones of that unit
    msw::SwParams p = base_params(sch);
    p.n_slots = 1;
    p.lds_stride = msw::stream_stride(300);
    p.group_lanes = 16;
    p.groups = 4;
    p.pairs_blocks = 1;
    int ok = 1;
    ok &= msw::sw_blocks_per_cu(p, sch.affine, sch.coords, 16, msw::Layout::kPairs) > 0;    // pairs, KR <= 16
    ok &= msw::sw_blocks_per_cu(p, sch.affine, sch.coords, 300, msw::Layout::kPairs) > 0;   // pairs, KR 17..24
    ok &= msw::sw_blocks_per_cu(p, sch.affine, sch.coords, 32, msw::Layout::kSplit) > 0;    // split
    ok &= msw::sw_blocks_per_cu(p, sch.affine, sch.coords, 32, msw::Layout::kMixed) > 0;    // mixed grid
    msw::MultiTable t;
    memset(&t, 0, sizeof(t));
    t.n_buckets = 1;
    t.block_end[0] = 1;
    t.count[0] = 1;
    t.lds_stride[0] = p.lds_stride;
    static const uint32_t dummy_order = 0;
    p.order = &dummy_order;  // never dereferenced: nothing launches
    for (uint32_t kr : {1u, 17u}) {  // the bucketed grid and its wide instance
        t.kr[0] = kr;
        ok &= msw::sw_multi_blocks_per_cu(p, t, sch.affine, sch.coords) > 0;
    }
    p.order = nullptr;
    static const uint8_t dummy_genome = 0;
    p.win_src = &dummy_genome;  // genome-window instances
    ok &= msw::sw_blocks_per_cu(p, sch.affine, sch.coords, 16, msw::Layout::kPairs) > 0;
    p.win_src = nullptr;
    ok &= msw::long_blocks_per_cu(sch.affine, sch.coords, 600, 600) > 0;
    ok &= msw::cut_blocks_per_cu() > 0;
    (void)hipGetLastError();
    return ok ? MSW_OK : fail(MSW_E_DEVICE, "kernel module load failed");
}

int msw_ctx_stats(msw_ctx* ctx, msw_stats_t* out, int reset) {
    if (!ctx || !out) return fail(MSW_E_INVALID, "ctx/out is NULL");
    if (set_device(ctx) == MSW_OK) harvest_dev_timings(ctx, true);
    *out = ctx->stats;
    if (reset) ctx->stats = msw_stats_t{};
    return MSW_OK;
}

int msw_fence_record(msw_ctx* ctx, void* stream, uint64_t* fence) {
    if (!ctx || !fence) return fail(MSW_E_INVALID, "ctx/fence is NULL");
    int rc = set_device(ctx);
    if (rc) return rc;
    hipEvent_t e = take_event(ctx);
    if (!e) return fail(MSW_E_DEVICE, "hipEventCreate failed");
    std::lock_guard<std::mutex> lk(ctx->ev_mu);
    if (hipEventRecord(e, stream ? (hipStream_t)stream : ctx->compute) != hipSuccess) {
        ctx->free_events.push_back(e);
        return fail(MSW_E_DEVICE, "hipEventRecord failed");
    }
    *fence = ctx->next_fence++;
    ctx->fences.emplace(*fence, e);
    return MSW_OK;
}

int msw_fence_wait(msw_ctx* ctx, uint64_t fence) {
    if (!ctx) return fail(MSW_E_INVALID, "ctx is NULL");
    hipEvent_t e = nullptr;
    {
        std::lock_guard<std::mutex> lk(ctx->ev_mu);
        auto it = ctx->fences.find(fence);
        if (it == ctx->fences.end()) return fail(MSW_E_INVALID, "unknown fence %llu", (unsigned long long)fence);
        e = it->second;
        ctx->fences.erase(it);
    }
    int rc = set_device(ctx);
    if (rc) return rc;
    const hipError_t err = hipEventSynchronize(e);
    {
        std::lock_guard<std::mutex> lk(ctx->ev_mu);
        ctx->free_events.push_back(e);
    }
    if (err != hipSuccess) return fail(MSW_E_DEVICE, "GPU error before the fence: %s", hipGetErrorString(err));
    return MSW_OK;
}

int msw_synchronize(msw_ctx* ctx) {
    if (!ctx) return fail(MSW_E_INVALID, "ctx is NULL");
    int rc = set_device(ctx);
    if (rc) return rc;
    for (hipStream_t st : {ctx->compute, ctx->compute2, ctx->copy, ctx->d2h, ctx->side})
        if (st) HIP_TRY(hipStreamSynchronize(st));
    for (hipStream_t st : ctx->user_streams) HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipGetLastError());
    return MSW_OK;
}

int msw_stream_create(msw_ctx* ctx, void** out) {
    if (!ctx || !out) return fail(MSW_E_INVALID, "ctx/out is NULL");
    *out = nullptr;
    int rc = set_device(ctx);
    if (rc) return rc;
    hipStream_t st = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    ctx->user_streams.push_back(st);
    *out = st;
    return MSW_OK;
}

int msw_stream_destroy(msw_ctx* ctx, void* stream) {
    if (!ctx || !stream) return fail(MSW_E_INVALID, "ctx/stream is NULL");
    auto it = std::find(ctx->user_streams.begin(), ctx->user_streams.end(), (hipStream_t)stream);
    if (it == ctx->user_streams.end()) return fail(MSW_E_INVALID, "stream was not made by msw_stream_create on this context");
    int rc = set_device(ctx);
    if (rc) return rc;
    ctx->user_streams.erase(it);
    // its per-stream scratch goes too (a later stream may reuse the handle)
    for (size_t i = 0; i < ctx->rscratch.size(); ++i)
        if (ctx->rscratch[i].st == (hipStream_t)stream) {
            HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
            (void)hipFree(ctx->rscratch[i].wins);
            (void)hipFree(ctx->rscratch[i].wlen);
            ctx->rscratch.erase(ctx->rscratch.begin() + (long)i);
            break;
        }
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    return MSW_OK;
}

}  // extern "C"
