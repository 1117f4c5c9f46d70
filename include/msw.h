/*
 * msw.h -- C ABI of the MI355X-native batched Smith-Waterman scorer.
 *
 * This is the drop-in boundary for the `smith_waterman` crate's scoring path
 * (bmwoolf/mini_parallel, package `rustseq_mini`).  The reference has no FFI
 * layer of its own (binary-only crate, Cargo.toml:7-17); each entry point
 * below names the Rust item it replaces (file:line under smith_waterman/src/).
 * A Rust crate binds it with a plain `extern "C"` block.
 *
 * Contract
 *  - C99 POD only; no C++ exceptions cross this boundary; every int-returning
 *    call returns MSW_OK (0) or a negative MSW_E* code, and msw_last_error()
 *    returns the thread-local message (mirrors Result<_, String>, e.g.
 *    aligner.rs:452-455).
 *  - One msw_ctx per GPU, used by one host thread at a time.  Contexts on
 *    different GPUs run concurrently.  The library owns all device memory and
 *    streams; the caller owns every host array it passes in.
 *  - Byte semantics follow the reference kernel: substitution is byte
 *    equality (smith_waterman.cl:43,114), case-sensitive, 'N' == 'N'.
 *  - Score = global max cell, >= 0.  Coordinates = 0-based (i in read, j in
 *    window) of the best cell, smallest i then smallest j on ties; (-1,-1)
 *    when the score is 0 or the pair is empty.
 *  - Supported by the GPU kernels: read and window lengths <= 32767 (pairs
 *    up to 384 x 4096 run on the packed 16-bit kernels, longer ones on the
 *    i32 long-pair kernel, in the same call), 1 <= match <= 64,
 *    match - 64 <= mismatch <= 0, 0 <= gap_extend <= 1024,
 *    0 <= gap_open <= 30000.  Anything else -> MSW_E_RANGE.
 *    There is no CPU fallback: without a usable GPU every call fails.
 */
#ifndef MSW_H
#define MSW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSW_OK 0
#define MSW_E_INVALID (-1)   /* bad argument / NULL pointer              */
#define MSW_E_RANGE (-2)     /* length or scoring outside kernel limits  */
#define MSW_E_DEVICE (-3)    /* HIP runtime / launch failure             */
#define MSW_E_NODEVICE (-4)  /* no GPU (is_gpu_available() == false)     */
#define MSW_E_NOMEM (-5)     /* device or pinned allocation failed       */

/* Replaces GpuDevice{name, memory_gb, max_work_group_size} (gpu.rs:17-22). */
typedef struct {
    char name[256];
    uint64_t mem_bytes;
    uint64_t mem_free_bytes;    /* hipMemGetInfo; replaces system_info.rs:236-243 */
    uint32_t max_wg;            /* max work-group size (gpu.rs:62)           */
    uint32_t cu_count;
    char arch[64];              /* e.g. "gfx950"                             */
} msw_device_info_t;

/* Scoring.  Reference constants: match +2, mismatch -1, gap 2
 * (smith_waterman.cl:5-7).  Linear gap: affine = 0, gap_extend = gap penalty,
 * gap_open ignored.  Affine (Gotoh): a gap of length k costs
 * gap_open + k * gap_extend.  want_coords = 1 fills end_i / end_j. */
typedef struct {
    int32_t match;
    int32_t mismatch;
    int32_t gap_open;
    int32_t gap_extend;
    int32_t affine;
    int32_t want_coords;
} msw_scoring_t;

/* A padded SoA batch: pair p uses reads[p*read_stride ..][0, read_len[p]) and
 * wins[p*win_stride ..][0, win_len[p]).  In msw_align_batch the pointers are
 * host memory (pageable or msw_host_alloc'ed); in msw_align_batch_device they
 * are device memory.  Replaces the Vec<String> chunk handed to the loader
 * callback (aligner.rs:107-108, :128-147). */
typedef struct {
    const uint8_t* reads;
    const uint8_t* wins;
    const uint16_t* read_len;
    const uint16_t* win_len;
    uint32_t read_stride;
    uint32_t win_stride;
    uint64_t n_pairs;
} msw_batch_t;

/* Caller-owned outputs (host in msw_align_batch, device in _device).
 * end_i / end_j may be NULL when want_coords == 0. */
typedef struct {
    int32_t* score;
    int16_t* end_i;
    int16_t* end_j;
} msw_out_t;

typedef struct msw_ctx msw_ctx;

/* gpu.rs:33-45 is_gpu_available / gpu.rs:48-94 get_gpu_devices. */
int msw_device_count(int* n);
int msw_device_info(int ordinal, msw_device_info_t* out);

/* gpu.rs:97-132 get_opencl_context/init_opencl: one context per device with
 * compute, copy and readback streams and three pinned staging slots (up to
 * three chunks in flight). */
int msw_ctx_create(int ordinal, msw_ctx** out);
/* msw_ctx_create with flags.  MSW_CTX_LEAN: only the compute stream up
 * front; the copy / second compute / readback / side streams are made by the
 * first call that needs them (host-batch calls, long pairs beside packed
 * ones).  A stream costs 3-30 ms to create -- the first few of a process each
 * make a hardware queue -- and the --full-wgs GPU-reader workers, which
 * score device-resident batches only, never use them.  Without the flag all
 * five streams are made here, before any the caller creates, so they land
 * on their own hardware queues.  The library reads its environment switches
 *  once, here. */
#define MSW_CTX_LEAN 1u
int msw_ctx_create_ex(int ordinal, unsigned flags, msw_ctx** out);
void msw_ctx_destroy(msw_ctx* ctx);

/* Batched scoring from host memory, synchronous.  Streams the batch through
 * pinned staging in chunks of `chunk_pairs` (0 = GPU_CHUNK_SIZE_READS env, or
 * 65536) with H2D copies on the copy stream overlapped with the kernels (a
 * one-chunk call keeps its copies and kernels on one compute stream; async
 * one-chunk calls alternate two, so consecutive calls overlap).
 * Pageable arrays are staged (rows repacked to 16-byte-rounded strides, so
 * padding does not cross PCIe); arrays in pinned memory (msw_host_alloc or
 * hipHostRegister) are copied to the GPU directly.
 * Replaces the per-chunk gpu_align loop of aligner.rs:269-289 / :390-398. */
int msw_align_batch(msw_ctx* ctx, const msw_scoring_t* sc, const msw_batch_t* batch,
                    msw_out_t* out, uint64_t chunk_pairs);

/* Same, asynchronous: returns a ticket; host arrays must stay alive and
 * unmodified until msw_wait(ticket) returns. */
int msw_align_batch_async(msw_ctx* ctx, const msw_scoring_t* sc, const msw_batch_t* batch,
                          msw_out_t* out, uint64_t chunk_pairs, uint64_t* ticket);
int msw_wait(msw_ctx* ctx, uint64_t ticket);

/* Device-resident batch: pointers in `batch` and `out` are device memory.
 * Enqueued on `stream` (a hipStream_t; NULL = the context's compute stream),
 * no host synchronisation.  max_read_len / max_win_len bound the batch (the
 * caller knows them; they select the kernel instance and the LDS size). */
int msw_align_batch_device(msw_ctx* ctx, const msw_scoring_t* sc, const msw_batch_t* batch,
                           msw_out_t* out, uint32_t max_read_len, uint32_t max_win_len,
                           void* stream);

/* Length-bucketed plan for a device-resident batch of mixed lengths (BASELINE
 * config 5).  Built on the host from host copies of the length arrays (the
 * FASTQ loader has them): pairs are grouped by rows per lane (read length /
 * 16) and by window length, and the slot -> pair order is uploaded once;
 * msw_align_batch_planned then scores the whole batch in ONE kernel launch,
 * heaviest bucket first, enqueued on `stream` like msw_align_batch_device.
 * A plan belongs to its context and fixes the scoring scheme and the lengths:
 * reuse it for every pass over the same batch.  This is the device-resident
 * form of msw_align_batch's per-chunk bucketing (which replaces the
 * one-string-per-call gpu_align loop, aligner.rs:269-289). */
typedef struct msw_plan msw_plan;
int msw_plan_create(msw_ctx* ctx, const msw_scoring_t* sc, const uint16_t* read_len,
                    const uint16_t* win_len, uint64_t n_pairs, msw_plan** out);
int msw_align_batch_planned(msw_ctx* ctx, const msw_plan* plan, const msw_batch_t* batch,
                            msw_out_t* out, void* stream);
void msw_plan_destroy(msw_plan* plan);

/* == gpu_align(seq1, seq2, device) (aligner.rs:410-532): the kernel the
 * reference actually launches (smith_waterman.cl:11-71) with its host geometry
 * W = min(max_wg, 1024) (aligner.rs:422), G = min(ceil(L/W), max_groups)
 * (:423-424; reference max_groups = 1,000,000, gpu.rs:10), L = min(n1, n2),
 * L == 0 -> 0 (:414-416), L > 1,024,000,000 or > 0.8*mem/3 -> MSW_E_RANGE
 * (:436-456).  wg == 0 -> device max work-group size capped at 1024. */
int msw_align_compat(msw_ctx* ctx, const uint8_t* s1, size_t n1, const uint8_t* s2, size_t n2,
                     uint32_t wg, uint32_t max_groups, int32_t* score);

/* Pinned host memory (hipHostMalloc); replaces USE_PINNED_MEMORY /
 * alloc_host_ptr (aligner.rs:466-475). */
void* msw_host_alloc(size_t bytes);
void msw_host_free(void* p);

/* Reference genome resident in HBM.  The --full-wgs sw driver scores each
 * read against a window of the reference genome; the reference crate builds
 * every input on the host per chunk (aligner.rs:269-289).  Here the genome is
 * uploaded once per GPU and windows are cut on the GPU from (position,
 * length), so a chunk ships reads + 8-byte positions over PCIe instead of
 * reads + windows (~2.7x fewer bytes at 150 bp x 300 bp).  A genome belongs to
 * the context it was created on; destroy it before that context. */
typedef struct msw_genome msw_genome;
int msw_genome_create(msw_ctx* ctx, const uint8_t* seq, uint64_t len, msw_genome** out);
void msw_genome_destroy(msw_genome* g);
uint64_t msw_genome_length(const msw_genome* g);

/* Device-resident form: cut the windows of n (position, requested length)
 * pairs (device arrays) into a device slab wins[n][win_stride] (win_stride a
 * multiple of 16, wins 16-byte aligned; zero-padded), writing the clipped
 * lengths to win_len_out (may be NULL) -- the input msw_align_batch_device /
 * msw_align_batch_planned take.  Enqueued on `stream` (NULL = the context's
 * compute stream).  Windows are also clipped at win_stride. */
int msw_genome_cut_device(msw_ctx* ctx, const msw_genome* g, const int64_t* win_pos, const uint16_t* win_len,
                          uint64_t n, uint8_t* wins, uint32_t win_stride, uint16_t* win_len_out, void* stream);

/* Reads against genome windows: pair p scores reads[p*read_stride ..][0,
 * read_len[p]) against genome[win_pos[p], win_pos[p] + win_len[p]), the
 * window clipped at the genome end; win_pos < 0 or >= the genome length is an
 * empty window (score 0, coordinates (-1,-1)).  The requested win_len is
 * bounded like a window length (<= 4096).  Host arrays as in
 * msw_align_batch (pageable or msw_host_alloc'ed: pinned arrays are copied to
 * the GPU directly, without staging). */
typedef struct {
    const uint8_t* reads;
    const uint16_t* read_len;
    uint32_t read_stride;
    const int64_t* win_pos;
    const uint16_t* win_len;
    uint64_t n_pairs;
} msw_read_batch_t;

int msw_align_reads(msw_ctx* ctx, const msw_scoring_t* sc, const msw_genome* g, const msw_read_batch_t* batch,
                    msw_out_t* out, uint64_t chunk_pairs);
/* Same, asynchronous (completes with msw_wait; host arrays must stay alive). */
int msw_align_reads_async(msw_ctx* ctx, const msw_scoring_t* sc, const msw_genome* g,
                          const msw_read_batch_t* batch, msw_out_t* out, uint64_t chunk_pairs, uint64_t* ticket);

/* Device-resident reads against genome windows (the GPU lane reader's
 * batches, msw_gfastq_next): read p = reads[p * read_stride ..][0,
 * read_len[p]) scores against genome[win_pos[p], win_pos[p] + W), W = window,
 * or 2 x read_len[p] when window is 0 (the CLI's --window rule), capped at
 * 4096 and clipped at the genome end.  Windows are cut into a context scratch
 * slab on the GPU; everything is enqueued on `stream` (NULL = the context's
 * compute stream), no host synchronisation.  All arrays are device memory;
 * win_len_out (may be NULL) receives the clipped window lengths.
 * max_read_len bounds read_len (it selects the kernel instance). */
int msw_align_reads_device(msw_ctx* ctx, const msw_scoring_t* sc, const msw_genome* g, const uint8_t* reads,
                           const uint16_t* read_len, uint32_t read_stride, const int64_t* win_pos, uint64_t n,
                           uint32_t window, uint32_t max_read_len, msw_out_t* out, uint16_t* win_len_out,
                           void* stream);

/* Device memory helpers for callers that keep batches resident in HBM. */
void* msw_dev_alloc(msw_ctx* ctx, size_t bytes);
void msw_dev_free(msw_ctx* ctx, void* p);
int msw_memcpy_h2d(msw_ctx* ctx, void* dst, const void* src, size_t bytes);
int msw_memcpy_d2h(msw_ctx* ctx, void* dst, const void* src, size_t bytes);
/* enqueued on `stream` (NULL = the context's compute stream); dst should be
 * pinned: into pinned memory the copy runs as a kernel on that stream (not a
 * DMA on the process-wide copy-engine rings, where a copy waiting on one
 * stream holds up the copies of others); pageable dst: hipMemcpyAsync. */
int msw_memcpy_d2h_async(msw_ctx* ctx, void* dst, const void* src, size_t bytes, void* stream);
int msw_synchronize(msw_ctx* ctx);
/* A host-waitable point in `stream`'s work (NULL = the context's compute
 * stream): msw_fence_wait blocks until everything enqueued on that stream
 * before msw_fence_record has finished, without waiting for what came after
 * (msw_synchronize drains all of the context's streams).  A fence is waited
 * on once; the context keeps unwaited fences until it is destroyed.  Several
 * threads may wait on (different) fences of one context at once. */
int msw_fence_record(msw_ctx* ctx, void* stream, uint64_t* fence);
int msw_fence_wait(msw_ctx* ctx, uint64_t fence);
/* A stream of the context's device for callers that keep two batches in
 * flight (e.g. --full-wgs alternates its batches over the compute stream and
 * one of these, so one batch's read emit and window cut run beside the other
 * batch's scoring).  Any call taking `void* stream` accepts it; calls on two
 * streams may run concurrently.  msw_synchronize drains it; msw_ctx_destroy
 * destroys any the caller has not.  (The reference scores one batch at a
 * time on one queue: gpu.rs:117-125.) */
int msw_stream_create(msw_ctx* ctx, void** out);
int msw_stream_destroy(msw_ctx* ctx, void* stream);

/* Counters of the host-batch calls (msw_align_batch*, msw_align_reads*) on a
 * context, for run records (the reference's BenchmarkResult,
 * tools/benchmark.rs:17-34, reports only wall-clock rates):
 * kernel_ms = GPU time covered by the scoring launches: the union of their
 * [start, end] intervals (HIP events around each chunk's launch on its
 * compute stream -- a multi-chunk call alternates two compute streams, whose
 * launches overlap -- added when the chunk is drained; and around
 * msw_align_reads_device launches, added when they have finished),
 * alg_bytes = read + window bytes + 4 B score (+ 4 B coordinates) per pair,
 * the kernel's algorithmic HBM traffic.  reset != 0 zeroes them after the copy. */
typedef struct {
    double kernel_ms;
    uint64_t launches;
    uint64_t pairs;
    uint64_t cells;
    uint64_t alg_bytes;
} msw_stats_t;
int msw_ctx_stats(msw_ctx* ctx, msw_stats_t* out, int reset);

/* Optional, before a timed region: load the code objects of every scoring
 * kernel module a call under this scheme may use (the packed layouts, the
 * length-bucketed grid, genome windows, long pairs, the window cut).  HIP
 * loads a module on its first launch, ~1-2 ms each, which a short run --
 * one lane file per worker -- would otherwise pay inside its first batch
 * (the reference has no analogue: it JIT-builds its OpenCL program on every
 * gpu_align call, aligner.rs:504-508).  Launches nothing. */
int msw_ctx_prepare(msw_ctx* ctx, const msw_scoring_t* scoring);

/* Thread-local message of the last failing call on this thread. */
const char* msw_last_error(void);

/* Library version string (also names the compiled GPU target). */
const char* msw_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MSW_H */
