// msw_gz.h -- GPU-side BGZF inflate and FASTQ parse (internal; host code in
// msw_gfastq.cpp, kernels in msw_inflate.hip and msw_parse.hip).
//
// The --full-wgs lane files are read on the host as compressed bytes only;
// inflate, CRC check, line split and record parse run on the GPU, and the
// reads land in HBM in the slab layout the SW kernels take.  This replaces
// process_fastq_file_in_chunks (smith_waterman/src/aligner.rs:107-178) --
// `zcat` + one String per line, one core per file -- for BGZF lane files.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace msw {

// One BGZF member of a span, as indexed on the host from the member headers
// (the 'BC' extra field gives the member size, the trailer the CRC and size).
struct GzMember {
    uint64_t coff;   // raw deflate data: byte offset in the span's compressed buffer
    uint64_t ooff;   // its output: byte offset in the span's output buffer
    uint32_t clen;   // raw deflate bytes (member size - 18 header - 8 trailer)
    uint32_t isize;  // uncompressed bytes (trailer ISIZE, <= 65536)
    uint32_t crc;    // trailer CRC-32 of the uncompressed bytes
    uint32_t pad;
};

// Per-member status words written by the kernels (0 = ok).
enum GzStatus : uint32_t {
    GZ_OK = 0,
    GZ_E_BTYPE = 1,     // reserved block type 3
    GZ_E_STORED = 2,    // stored block LEN != ~NLEN
    GZ_E_HEADER = 3,    // dynamic header: too many length or distance symbols / bad repeat
    GZ_E_CODES = 4,     // over-subscribed or incomplete code set, or no end-of-block code
    GZ_E_SYMBOL = 5,    // invalid literal/length or distance code
    GZ_E_DIST = 6,      // distance too far back
    GZ_E_OVERRUN = 7,   // more output than the trailer's ISIZE
    GZ_E_TRUNC = 8,     // deflate data runs past the member
    GZ_E_SIZE = 9,      // less output than ISIZE
    GZ_E_CRC = 10,      // CRC-32 mismatch
};

// CRC-32 constants (zlib's x^(2^k) mod p table and the 256-byte advance), host-built.
struct GzCrcConsts {
    uint32_t x2n[32];       // x^(2^k) mod p(x), reflected
    uint32_t adv[4][256];   // adv[i][v] = (v << 8i) * x^(8 * 256) mod p: a raw CRC state
                            // advanced over 256 bytes, one byte of the state at a time
};

// Inflate every member of a span (one wave per member); status[m] set for each.
// cdata: the span's compressed bytes, 4-byte aligned, cbytes of them readable
// (device memory, or pinned host memory read in place); the kernel clamps
// every load to them, so no padding after the span is needed.
// prof (MSW_GZ_PROFILE builds only, else ignored): 16 u32 counters per member
hipError_t launch_gz_inflate(const uint8_t* cdata, size_t cbytes, const GzMember* members, uint32_t n, uint8_t* out,
                             uint32_t* status, uint32_t* any_error, hipStream_t stream, uint32_t* prof = nullptr);
// CRC-32 of every member's output against its trailer (one wave per member).
hipError_t launch_gz_crc(const uint8_t* out, const GzMember* members, uint32_t n, const GzCrcConsts* consts,
                         uint32_t* status, uint32_t* any_error, hipStream_t stream);
// Load the inflate / CRC and the parse / emit code objects now (a reader's
// setup) instead of at their first launch, which sat inside the first span.
hipError_t gz_preload();
hipError_t parse_preload();

// ---------------------------------------------------------------------------
// FASTQ parse of an inflated span (msw_parse.hip).  The span buffer holds the
// previous span's unfinished line, then this span's bytes.  Semantics of
// aligner.rs:128-170: lines end at '\n', one trailing '\r' stripped; a line
// that is not valid UTF-8 is skipped and not counted (an error); valid line
// number (1-based, over the whole file) % 4 == 2 is a sequence.
// ---------------------------------------------------------------------------
constexpr uint32_t kParseTile = 4096;  // bytes per line-count tile
constexpr uint32_t kLenBuckets = 256;  // per-span read-length maxima (ParseOut::bmax)

struct ParseState {   // device-resident, carried from span to span
    uint64_t valid_lines;   // valid lines of the file before this span
    uint64_t errors;        // invalid (non-UTF-8) lines so far
    int64_t pending_pos;    // pos= of a header line that ended the previous span
    uint64_t reads;         // reads of the file before this span
};

struct ParseOut {     // per span, read back by the host
    uint64_t lines;         // complete lines in the span (incl. invalid ones; + a final line at EOF)
    uint64_t newlines;      // '\n' bytes in the span
    uint64_t tail_start;    // first byte after the last newline (the carry), len at EOF
    uint64_t valid;         // valid lines in the span
    uint64_t reads;         // reads (sequence lines) in the span
    uint64_t bases;         // sum of their lengths
    uint64_t v0;            // valid lines of the file before the span
    int64_t pending_in;     // pos= carried into the span (its first line may be a sequence)
    uint32_t any_high;      // some byte >= 0x80 (UTF-8 validation ran)
    uint32_t overflow;      // more lines than the line arrays hold
    uint32_t min_len, max_len;
    uint32_t too_long;      // a sequence line longer than the slab stride
    uint32_t err_over;      // the file passed 10 invalid lines in this span
    uint64_t too_long_line; // smallest valid line number (1-based, file) of such a line
    uint64_t err_line;      // valid lines read before the file's 11th invalid line
    // longest read of each run of ParseBufs::bucket_reads reads of the span
    // (a batch of the reader lies inside one run): the batch's bound, so one
    // long read sends only its own batch to a wider kernel, not the span
    uint32_t bmax[kLenBuckets];
};

struct ParseBufs {
    const uint8_t* buf;     // 16-byte aligned base, >= 64 bytes of padding past len
    uint64_t len;           // the span is bytes [begin, len) of buf
    uint32_t begin;         // < 16: the span starts that far into the aligned base
    uint32_t eof;           // last span of the file: a final line without '\n' counts
    uint32_t want_pos;
    uint32_t* tile_nl;      // per tile: newlines, then their exclusive scan
    uint32_t* tile_hi;      // per tile: any byte >= 0x80
    uint32_t ntiles;
    uint32_t* line_end;     // per line: byte offset of its '\n' (len for a final line)
    uint64_t line_cap;
    uint32_t* vidx;         // (non-ASCII spans) per line: valid flag, then valid index or ~0u
    uint32_t* vline;        // (non-ASCII spans) valid index -> line index
    uint32_t* blk;          // scan scratch, line_cap / 1024 + 2 entries
    uint32_t stride;        // slab row bytes (multiple of 16, <= 32768 checked by the host)
    uint64_t bucket_reads;  // reads per ParseOut::bmax entry (a multiple of the batch size; phase B)
    ParseState* state;
    ParseOut* out;
};

// Phase A: per-tile newline counts, their scan, *out initialised (lines,
// any_high).  The host reads *out, sizes line_end (>= lines) and, for a span
// with a byte >= 0x80, vidx / vline / blk, then runs phase B: line ends, the
// UTF-8 pass, lengths and the carried state (*state for the next span).
hipError_t launch_parse_a(const ParseBufs& b, hipStream_t stream);
hipError_t launch_parse_b(const ParseBufs& b, uint64_t lines, bool any_high, hipStream_t stream);

struct EmitSpan {     // facts of the parsed span the emit kernel needs (host copies)
    uint64_t v0;
    int64_t pending_in;
    uint32_t any_high;
    uint32_t pad;
};
// Reads [r_begin, r_begin + count) of the parsed span into a slab
// (reads[count][stride], read_len[count], pos[count] when pos != NULL).
hipError_t launch_emit_reads(const ParseBufs& b, const EmitSpan& sp, uint64_t r_begin, uint64_t count,
                             uint8_t* reads, uint16_t* read_len, int64_t* pos, hipStream_t stream);

}  // namespace msw
