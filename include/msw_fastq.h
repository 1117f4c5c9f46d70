/*
 * msw_fastq.h -- FASTQ(.gz) chunk reader of the MI355X scorer (C ABI).
 *
 * Replaces process_fastq_file_in_chunks (smith_waterman/src/aligner.rs:107-178)
 * and count_bases_in_fastq (:535-544).  Same record semantics:
 *   - a line is the bytes up to '\n' with a trailing "\r" stripped (Rust
 *     BufRead::lines, :133);
 *   - a line that is not valid UTF-8 is a read error: it is skipped and not
 *     counted (:155-158); more than 10 errors abort the file (:160-162);
 *   - the sequence line is the 1-based line number with line % 4 == 2 (:138);
 *     headers and '+' lines are not validated;
 *   - full chunks of N reads, then one final partial chunk (:143-147, :168-170).
 * Instead of a Vec<String> per chunk, sequences are written straight into a
 * caller-provided padded SoA slab (e.g. msw_host_alloc'ed pinned memory), the
 * layout msw_align_batch takes.  .gz files (multi-member included) are read
 * with zlib in-process (the reference spawns `zcat`, :111-115).
 */
#ifndef MSW_FASTQ_H
#define MSW_FASTQ_H

#include <stdint.h>

#include "msw.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct msw_fastq msw_fastq;

int msw_fastq_open(const char* path, msw_fastq** out);
void msw_fastq_close(msw_fastq* fq);

/* Read up to max_reads sequence lines into seqs[i*stride ..], lens[i].
 * *n_read = reads delivered (0 at end of file).  A sequence longer than
 * stride is MSW_E_RANGE.  pos (optional, may be NULL): the integer after
 * "pos=" in the record's header line, -1 when absent (synthetic datasets tag
 * each read with its reference window offset). */
int msw_fastq_next(msw_fastq* fq, uint8_t* seqs, uint16_t* lens, uint32_t stride,
                   uint64_t max_reads, uint64_t* n_read, int64_t* pos);

/* Packed form, for callers that concatenate a chunk's sequences (the compat
 * driver: chunk.concat() at aligner.rs:270, any read length): up to max_reads
 * sequences appended back to back into buf[0, cap), lengths in lens[].  Stops
 * early when the next sequence does not fit the space left; *need (optional)
 * is then its length and the next call delivers it first (grow the buffer by
 * at least that).  *n_bytes = bytes written; *n_read = 0 and *need = 0 at end
 * of file. */
int msw_fastq_next_packed(msw_fastq* fq, uint8_t* buf, uint64_t cap, uint32_t* lens, uint64_t max_reads,
                          uint64_t* n_read, uint64_t* n_bytes, uint64_t* need);

/* Counters so far: lines (valid lines, aligner.rs:136), reads, read errors. */
void msw_fastq_stats(const msw_fastq* fq, uint64_t* lines, uint64_t* reads, uint64_t* errors);

/* count_bases_in_fastq (aligner.rs:535-544): total bases and reads. */
int msw_fastq_count_bases(const char* path, uint64_t* bases, uint64_t* reads);

/* ------------------------------------------------------------------------
 * GPU-side lane reader for BGZF files (the --full-wgs hot path's caller).
 * The host reads compressed bytes only; inflate (RFC 1951), the CRC-32 check,
 * the line split / UTF-8 / record numbering above and the sequence copy run
 * on the GPU, and the reads land in HBM in the slab layout the scoring
 * entry points take (msw_align_batch_device, msw_genome_cut_device).  Same
 * semantics and error messages as msw_fastq_next; same reads in the same
 * order.  Replaces process_fastq_file_in_chunks (aligner.rs:107-178) for
 * BGZF lane files (a plain gzip member is MSW_E_INVALID: use msw_fastq_*).
 * ------------------------------------------------------------------------ */
typedef struct msw_gfastq msw_gfastq;

typedef struct {
    const uint8_t* reads;      /* device: reads[n][read_stride], zero-padded */
    const uint16_t* read_len;  /* device */
    const int64_t* pos;        /* device, or NULL unless opened with want_pos: pos= of the header, -1 */
    uint32_t read_stride;
    uint64_t n;                /* reads in this batch; 0 = end of file */
    uint64_t first_read;       /* file index of the batch's first read */
    uint32_t min_len, max_len; /* bounds over the span the batch comes from */
} msw_dev_reads_t;

/* is path a BGZF file (first member has the 'BC' extra field)? 1 / 0 */
int msw_is_bgzf(const char* path);

/* read_stride: multiple of 16, <= 32768 (longer sequences are MSW_E_RANGE);
 * max_reads: batch size (device slabs for two batches are allocated);
 * span_bytes: decompressed bytes inflated and parsed per step (0 = default
 * 1 GiB, env MSW_GFASTQ_SPAN_MB).  path may be NULL: the buffers are
 * allocated now and msw_gfastq_reset names the first file.
 * A lane file must not be modified or truncated while a reader has it open:
 * its page-cache pages are mapped (MAP_SHARED) and DMA'd in place.  A file
 * found shorter than when it was opened is reported (MSW_E_INVALID) at the
 * next span; one truncated while a span's member headers are being indexed
 * can raise SIGBUS.  MSW_GZ_NO_MAP=1 reads through pread copies instead.
 * The reader inflates and parses on a stream of its own, made with a CU mask
 * (all CUs) so that it has a hardware queue of its own; such a stream is
 * ordered with work on the null stream. */
int msw_gfastq_open(msw_ctx* ctx, const char* path, uint32_t read_stride, uint64_t max_reads, int want_pos,
                    uint64_t span_bytes, msw_gfastq** out);
/* The next batch, enqueued on `stream` (a hipStream_t; NULL = the context's
 * compute stream) -- scoring launched after it on that stream sees it.  The
 * device arrays stay valid until the call after next (two slabs alternate). */
int msw_gfastq_next(msw_gfastq* g, void* stream, msw_dev_reads_t* out);
/* Point an open reader at another lane file (same context, stride, batch
 * size and span): the device and pinned buffers are kept, so a worker that
 * walks many files allocates once, and the new file's compressed bytes start
 * loading in the background.  Batches keep the rule above across files (the
 * two slabs alternate), so scoring enqueued on the previous file's last
 * batches may still be running while the new file is inflated and parsed. */
int msw_gfastq_reset(msw_gfastq* g, const char* path);
/* Name the lane file the next msw_gfastq_reset will open: it is opened,
 * mapped, its first window of compressed bytes pinned and that window's
 * first span of BGZF members indexed by a host thread now, beside the
 * current file's spans, so the reset adopts it instead of
 * waiting for it (a new file's first window cost ~18-25 ms against 2-4 ms
 * for later ones: tools/gfastq_trace_c4.sh).  Optional; a reset to another
 * path opens that path as usual, and failures here only leave the reset to
 * do the work.  The --full-wgs driver's per-file loop (aligner.rs:246-339)
 * prefetches the file it will take next. */
int msw_gfastq_prefetch(msw_gfastq* g, const char* path);
/* lines (valid), reads, errors (invalid lines), bases, compressed and inflated bytes so far (this file) */
void msw_gfastq_stats(const msw_gfastq* g, uint64_t* lines, uint64_t* reads, uint64_t* errors, uint64_t* bases,
                      uint64_t* bytes_in, uint64_t* bytes_out);
void msw_gfastq_close(msw_gfastq* g);

/* Host-to-host BGZF inflate on the GPU (test / tool form of the same
 * kernels): data[0, len) is a whole BGZF file; out receives the
 * decompressed bytes (*out_len).  MSW_E_INVALID on bad data (message names
 * the member and the error), MSW_E_RANGE if cap is too small. */
int msw_bgzf_inflate(msw_ctx* ctx, const uint8_t* data, uint64_t len, uint8_t* out, uint64_t cap,
                     uint64_t* out_len);

#ifdef __cplusplus
}
#endif
#endif /* MSW_FASTQ_H */
