// msw_parse.hip -- FASTQ record parse of an inflated span on gfx950.
//
// Semantics of process_fastq_file_in_chunks (smith_waterman/src/aligner.rs:
// 107-178, as restated by msw_fastq.cpp): a line is the bytes up to '\n' with
// one trailing '\r' stripped; a line that is not valid UTF-8 is skipped and
// not counted (:155-163, an error; more than 10 abort the file); the valid
// line whose 1-based number % 4 == 2 is a sequence; the "pos=" tag of the
// header before it gives the read's window position (synthetic datasets).
//
// Data-parallel form over a span of S bytes (HBM-bound byte work):
//   count   per 4 KiB tile: newlines and any byte >= 0x80 (16 B per lane)
//   scan    one workgroup: exclusive scan of the tile counts (+ init of *out)
//   ends    per tile: byte offset of every newline -> line_end[]
//   utf8    only if some byte >= 0x80: per-line validation, a scan of the
//           valid flags -> valid index per line and line per valid index
//   lens    per read: length, min / max / sum, the too-long check
//   fin     one lane: reads in the span, the carry, the state for the next span
//   emit    per read, 16 lanes: the sequence into a zero-padded slab row with
//           16-byte stores, and the header's pos= (after all of the above)
// The valid-line numbering continues across spans through ParseState, so a
// record may straddle two spans (the host carries the unfinished line).
#include <algorithm>

#include "msw_gz.h"

namespace msw {
namespace {

// high bit of each zero byte of x (exact, no borrow false positives)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}

// bytes [0, r) of a word are inside the span
__device__ __forceinline__ uint32_t byte_mask(uint64_t r) {
    return r >= 4 ? 0xFFFFFFFFu : (uint32_t)((1ull << (8 * r)) - 1);
}

// bytes of the word at offset p that lie in [begin, len)
__device__ __forceinline__ uint32_t span_mask(uint64_t p, uint64_t begin, uint64_t len) {
    const uint32_t hi = byte_mask(len > p ? len - p : 0);
    const uint32_t lo = begin > p ? byte_mask(begin - p) : 0u;
    return hi & ~lo;
}

template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total) {
    __shared__ uint32_t wsum[NT / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) {
        const uint32_t s = wsum[k];
        if ((uint32_t)k < w) pre += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return pre + x - v;
}

__device__ __forceinline__ uint32_t line_start(const ParseBufs& b, uint64_t k) {
    return k ? b.line_end[k - 1] + 1u : b.begin;
}

// [start, end) of line k without its trailing '\r'
__device__ __forceinline__ void line_bounds(const ParseBufs& b, uint64_t k, uint32_t& st, uint32_t& en) {
    st = line_start(b, k);
    en = b.line_end[k];
    if (en > st && b.buf[en - 1] == '\r') --en;
}

// Strict UTF-8 (what Rust's String conversion in BufRead::lines checks).
__device__ bool utf8_ok(const uint8_t* s, uint32_t n) {
    uint32_t i = 0;
    while (i < n) {
        const uint32_t c = s[i];
        if (c < 0x80) { ++i; continue; }
        uint32_t len, cp;
        if ((c & 0xE0) == 0xC0) { len = 2; cp = c & 0x1F; }
        else if ((c & 0xF0) == 0xE0) { len = 3; cp = c & 0x0F; }
        else if ((c & 0xF8) == 0xF0) { len = 4; cp = c & 0x07; }
        else return false;
        if (i + len > n) return false;
        for (uint32_t k = 1; k < len; ++k) {
            const uint32_t d = s[i + k];
            if ((d & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (d & 0x3F);
        }
        if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && cp < 0x10000) || cp > 0x10FFFF ||
            (cp >= 0xD800 && cp <= 0xDFFF))
            return false;
        i += len;
    }
    return true;
}

// The integer after the first "pos=" that is followed by digits (msw_fastq.cpp
// parse_pos), -1 if none.
__device__ int64_t parse_pos(const uint8_t* s, uint32_t n) {
    for (uint32_t i = 0; i + 4 <= n; ++i) {
        if (s[i] == 'p' && s[i + 1] == 'o' && s[i + 2] == 's' && s[i + 3] == '=') {
            uint32_t j = i + 4;
            const bool neg = j < n && s[j] == '-';
            if (neg) ++j;
            int64_t v = 0;
            bool any = false;
            while (j < n && s[j] >= '0' && s[j] <= '9') {
                v = v * 10 + (s[j] - '0');
                ++j;
                any = true;
            }
            if (any) return neg ? -v : v;
        }
    }
    return -1;
}

__constant__ int64_t kPow10[16] = {1ll, 10ll, 100ll, 1000ll, 10000ll, 100000ll, 1000000ll, 10000000ll,
                                   100000000ll, 1000000000ll, 10000000000ll, 100000000000ll, 1000000000000ll,
                                   10000000000000ll, 100000000000000ll, 1000000000000000ll};

__device__ __forceinline__ bool is_digit(uint32_t c) { return c - '0' < 10u; }

// parse_pos of the header [hs, hs + n) by the 16 lanes of a read group (l16 =
// lane in the group, all 16 active): lane l holds header dwords l..l+2 and
// tests the four alignments of "pos=" it starts; the first occurrence that
// a number follows wins (group min); its digits are one byte per lane and
// the value a group sum of digit x 10^k.  Headers over 60 bytes or numbers
// of 16+ digits take the serial parse_pos (same result).  buf has >= 72
// readable bytes past any header start (the span buffer's slack).
__device__ int64_t group_parse_pos(const uint8_t* buf, uint32_t hs, uint32_t n, uint32_t l16) {
    if (n > 60) return parse_pos(buf + hs, n);
    const uint32_t sh = hs & 3u;
    const uint32_t* p = (const uint32_t*)(buf + (hs - sh)) + l16;
    const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];
    uint32_t best = 0xFFFFu;
#pragma unroll
    for (uint32_t s = 0; s < 4; ++s) {
        const int32_t at = (int32_t)(4u * l16 + s) - (int32_t)sh;  // header offset of this candidate
        const uint32_t w = __builtin_amdgcn_alignbyte(d1, d0, s);
        const uint32_t nx = __builtin_amdgcn_alignbyte(d2, d1, s);  // the 4 bytes after it
        const uint32_t c1 = nx & 0xFFu, c2 = (nx >> 8) & 0xFFu;
        const bool num = (is_digit(c1) && at + 5 <= (int32_t)n) ||
                         (c1 == '-' && is_digit(c2) && at + 6 <= (int32_t)n);
        if (at >= 0 && w == 0x3D736F70u && num) best = min(best, (uint32_t)at);  // "pos="
    }
#pragma unroll
    for (int d = 8; d >= 1; d >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, d, 16));
    if (best == 0xFFFFu) return -1;
    const bool neg = buf[hs + best + 4] == '-';
    const uint32_t q = best + 4u + (neg ? 1u : 0u) + l16;
    const bool dig = q < n && is_digit(buf[hs + q]);
    const uint64_t bal = __ballot(dig);
    const uint32_t mine = (uint32_t)(bal >> (threadIdx.x & 48u)) & 0xFFFFu;  // this group's 16 lanes
    const uint32_t cnt = (uint32_t)__builtin_ctz(~mine);                    // leading digits (<= 16)
    if (cnt >= 16) return parse_pos(buf + hs, n);
    int64_t v = l16 < cnt ? (int64_t)(buf[hs + q] - '0') * kPow10[cnt - 1 - l16] : 0;
#pragma unroll
    for (int d = 8; d >= 1; d >>= 1) v += __shfl_xor(v, d, 16);
    return neg ? -v : v;
}

// first valid index of a sequence line, given the valid lines before the span
__device__ __forceinline__ uint32_t seq_phase(uint64_t v0) { return (uint32_t)((5u - (v0 & 3u)) & 3u); }

__device__ __forceinline__ uint64_t reads_in(uint64_t valid, uint64_t v0) {
    const uint32_t o = seq_phase(v0);
    return valid > o ? (valid - o + 3) / 4 : 0;
}

__global__ __launch_bounds__(256) void k_count(ParseBufs b) {
    const uint64_t base = (uint64_t)blockIdx.x * kParseTile + 16ull * threadIdx.x;
    uint32_t nl = 0, hi = 0;
    if (base < b.len) {
        const uint4 v = *(const uint4*)(b.buf + base);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t m = span_mask(base + 4u * k, b.begin, b.len);
            nl += __popc(zero_bytes(w[k] ^ 0x0A0A0A0Au) & m);
            hi |= w[k] & m;
        }
        hi &= 0x80808080u;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        nl += __shfl_xor(nl, d);
        hi |= __shfl_xor(hi, d);
    }
    __shared__ uint32_t s_nl[4], s_hi[4];
    if ((threadIdx.x & 63) == 0) {
        s_nl[threadIdx.x >> 6] = nl;
        s_hi[threadIdx.x >> 6] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        b.tile_nl[blockIdx.x] = s_nl[0] + s_nl[1] + s_nl[2] + s_nl[3];
        b.tile_hi[blockIdx.x] = (s_hi[0] | s_hi[1] | s_hi[2] | s_hi[3]) != 0;
    }
}

// 256 threads: a single workgroup that fits on a CU beside inflate waves.
// Thread t owns a contiguous run of tiles (a multiple of 4: 16-byte loads
// and stores, four in flight per iteration), then adds its block-scan prefix.
__global__ __launch_bounds__(256) void k_scan_tiles(ParseBufs b) {
    const uint32_t n = b.ntiles, t = threadIdx.x;
    const uint32_t per = (((n + 255) / 256) + 3u) & ~3u;
    const uint32_t a = min(n, t * per), e = min(n, a + per);
    const uint32_t e4 = a + ((e - a) & ~3u);
    uint32_t s = 0, h = 0;
    uint32_t i = a;
    for (; i + 16 <= e4; i += 16) {
        uint4 v[4], q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[k] = *(const uint4*)(b.tile_nl + i + 4 * k);
            q[k] = *(const uint4*)(b.tile_hi + i + 4 * k);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            s += v[k].x + v[k].y + v[k].z + v[k].w;
            h |= q[k].x | q[k].y | q[k].z | q[k].w;
        }
    }
    for (; i < e4; i += 4) {
        const uint4 v = *(const uint4*)(b.tile_nl + i), q = *(const uint4*)(b.tile_hi + i);
        s += v.x + v.y + v.z + v.w;
        h |= q.x | q.y | q.z | q.w;
    }
    for (; i < e; ++i) {
        s += b.tile_nl[i];
        h |= b.tile_hi[i];
    }
    uint32_t tot;
    uint32_t pre = block_excl_scan<256>(s, &tot);
    for (i = a; i < e4; i += 4) {
        const uint4 v = *(const uint4*)(b.tile_nl + i);
        uint4 o;
        o.x = pre;
        o.y = o.x + v.x;
        o.z = o.y + v.y;
        o.w = o.z + v.z;
        pre = o.w + v.w;
        *(uint4*)(b.tile_nl + i) = o;
    }
    for (; i < e; ++i) {
        const uint32_t c = b.tile_nl[i];
        b.tile_nl[i] = pre;
        pre += c;
    }
    const int anyh = __syncthreads_or(h != 0);
    if (t < kLenBuckets) b.out->bmax[t] = 0;
    if (t == 0) {
        ParseOut* o = b.out;
        const bool final_line = b.eof && b.len > b.begin && b.buf[b.len - 1] != '\n';
        const uint64_t lines = (uint64_t)tot + (final_line ? 1u : 0u);
        o->lines = lines;
        o->newlines = tot;
        o->tail_start = 0;
        o->valid = lines;  // unless the UTF-8 pass says otherwise
        o->reads = 0;
        o->bases = 0;
        o->v0 = b.state->valid_lines;
        o->pending_in = b.state->pending_pos;
        o->any_high = anyh ? 1u : 0u;
        o->overflow = lines > b.line_cap ? 1u : 0u;
        o->min_len = 0xFFFFFFFFu;
        o->max_len = 0;
        o->too_long = 0;
        o->err_over = 0;
        o->too_long_line = ~0ull;
        o->err_line = 0;
    }
}

__global__ __launch_bounds__(256) void k_line_ends(ParseBufs b) {
    if (b.out->overflow) return;
    const uint64_t base = (uint64_t)blockIdx.x * kParseTile + 16ull * threadIdx.x;
    uint32_t flags = 0;  // bit i: byte base + i is '\n'
    if (base < b.len) {
        const uint4 v = *(const uint4*)(b.buf + base);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t z = zero_bytes(w[k] ^ 0x0A0A0A0Au) & span_mask(base + 4u * k, b.begin, b.len);
            const uint32_t f = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
            flags |= f << (4 * k);
        }
    }
    uint32_t tot;
    const uint32_t off = block_excl_scan<256>((uint32_t)__popc(flags), &tot);
    if (blockIdx.x == 0 && threadIdx.x == 0 && b.out->lines > b.out->newlines)
        b.line_end[b.out->newlines] = (uint32_t)b.len;  // the final line of the file, without '\n'
    uint32_t* dst = b.line_end + b.tile_nl[blockIdx.x] + off;
    while (flags) {
        const int i = __ffs(flags) - 1;
        *dst++ = (uint32_t)(base + (uint32_t)i);
        flags &= flags - 1;
    }
}

// --- UTF-8 pass (spans with a byte >= 0x80 only) ---------------------------
__global__ __launch_bounds__(256) void k_utf8(ParseBufs b) {
    const ParseOut* o = b.out;
    if (!o->any_high || o->overflow) return;
    const uint64_t nl = o->lines;
    for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < nl; k += (uint64_t)gridDim.x * 256) {
        uint32_t st, en;
        line_bounds(b, k, st, en);
        b.vidx[k] = utf8_ok(b.buf + st, en - st) ? 1u : 0u;
    }
}

constexpr uint32_t kScanChunk = 1024;  // lines per scan chunk (256 threads x 4)

__global__ __launch_bounds__(256) void k_vsum(ParseBufs b) {
    const ParseOut* o = b.out;
    if (!o->any_high || o->overflow) return;
    const uint64_t nl = o->lines, nch = (nl + kScanChunk - 1) / kScanChunk;
    for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
        uint32_t s = 0;
        for (uint32_t i = 0; i < 4; ++i) {
            const uint64_t k = c * kScanChunk + 4u * threadIdx.x + i;
            if (k < nl) s += b.vidx[k];
        }
        uint32_t tot;
        block_excl_scan<256>(s, &tot);
        if (threadIdx.x == 0) b.blk[c] = tot;
    }
}

__global__ __launch_bounds__(1024) void k_vscan(ParseBufs b) {
    ParseOut* o = b.out;
    if (!o->any_high || o->overflow) return;
    const uint64_t nl = o->lines;
    const uint32_t n = (uint32_t)((nl + kScanChunk - 1) / kScanChunk), t = threadIdx.x;
    const uint32_t per = (n + 1023) / 1024;
    const uint32_t a = min(n, t * per), e = min(n, a + per);
    uint32_t s = 0;
    for (uint32_t i = a; i < e; ++i) s += b.blk[i];
    uint32_t tot;
    uint32_t pre = block_excl_scan<1024>(s, &tot);
    for (uint32_t i = a; i < e; ++i) {
        const uint32_t c = b.blk[i];
        b.blk[i] = pre;
        pre += c;
    }
    if (t == 0) o->valid = tot;
}

__global__ __launch_bounds__(256) void k_vapply(ParseBufs b) {
    ParseOut* o = b.out;
    if (!o->any_high || o->overflow) return;
    const uint64_t nl = o->lines, nch = (nl + kScanChunk - 1) / kScanChunk;
    const uint64_t err0 = b.state->errors;
    for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
        uint32_t f[4], s = 0;
        for (uint32_t i = 0; i < 4; ++i) {
            const uint64_t k = c * kScanChunk + 4u * threadIdx.x + i;
            f[i] = k < nl ? b.vidx[k] : 0u;
            s += f[i];
        }
        uint32_t tot;
        uint32_t idx = b.blk[c] + block_excl_scan<256>(s, &tot);
        for (uint32_t i = 0; i < 4; ++i) {
            const uint64_t k = c * kScanChunk + 4u * threadIdx.x + i;
            if (k >= nl) break;
            if (f[i]) {
                b.vidx[k] = idx;
                b.vline[idx] = (uint32_t)k;
                ++idx;
            } else {
                b.vidx[k] = ~0u;
                // this line is invalid line number err0 + (k - idx) + 1 of the file
                if (err0 + (k - idx) == 10) {
                    o->err_over = 1;
                    o->err_line = o->v0 + idx;
                }
            }
        }
    }
}

// --- per read: lengths and the span totals ---------------------------------
__device__ inline uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d));
    return v;
}

__global__ __launch_bounds__(256) void k_lens(ParseBufs b) {
    ParseOut* o = b.out;
    if (o->overflow) return;
    const bool ascii = !o->any_high;
    const uint64_t v0 = o->v0, n = reads_in(o->valid, v0);
    const uint32_t ph = seq_phase(v0);
    uint32_t mn = 0xFFFFFFFFu, mx = 0;
    uint64_t bases = 0, tl = ~0ull;
    // per-run maxima (bmax): a wave whose 64 reads share a run keeps the run's
    // max in a register and flushes it (one wave-reduced atomic) when the run
    // changes; a wave straddling two runs flushes per lane
    const uint64_t bq = b.bucket_reads ? b.bucket_reads : ~0ull;
    uint32_t cur = ~0u, bm = 0;
    for (uint64_t r0 = (uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u); r0 < n; r0 += (uint64_t)gridDim.x * 256) {
        const uint64_t r = r0 + (threadIdx.x & 63u);
        uint32_t len = 0;
        if (r < n) {
            const uint64_t j = ph + 4 * r;
            const uint64_t k = ascii ? j : b.vline[j];
            uint32_t st, en;
            line_bounds(b, k, st, en);
            len = en - st;
            if (len > b.stride) tl = min(tl, v0 + j + 1);
            mn = min(mn, len);
            mx = max(mx, len);
            bases += len;
        }
        const uint64_t rl = min(r0 + 63, n - 1);
        const uint32_t k0 = (uint32_t)min<uint64_t>(r0 / bq, kLenBuckets - 1);
        const uint32_t k1 = (uint32_t)min<uint64_t>(rl / bq, kLenBuckets - 1);
        if (k0 != k1) {  // wave-uniform: this wave's reads cross a run boundary
            if (r < n) atomicMax(&o->bmax[(uint32_t)min<uint64_t>(r / bq, kLenBuckets - 1)], len);
            continue;
        }
        if (k0 != cur) {
            if (cur != ~0u) {
                const uint32_t w = wave_max_u32(bm);
                if ((threadIdx.x & 63) == 0) atomicMax(&o->bmax[cur], w);
            }
            cur = k0;
            bm = 0;
        }
        bm = max(bm, len);
    }
    if (cur != ~0u) {
        const uint32_t w = wave_max_u32(bm);
        if ((threadIdx.x & 63) == 0) atomicMax(&o->bmax[cur], w);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        mn = min(mn, (uint32_t)__shfl_xor(mn, d));
        mx = max(mx, (uint32_t)__shfl_xor(mx, d));
        bases += __shfl_xor(bases, d);
        tl = min(tl, (uint64_t)__shfl_xor(tl, d));
    }
    if ((threadIdx.x & 63) == 0 && mn != 0xFFFFFFFFu) {
        atomicMin(&o->min_len, mn);
        atomicMax(&o->max_len, mx);
        atomicAdd((unsigned long long*)&o->bases, (unsigned long long)bases);
        if (tl != ~0ull) {
            atomicMin((unsigned long long*)&o->too_long_line, (unsigned long long)tl);
            atomicOr(&o->too_long, 1u);
        }
    }
}

__global__ void k_fin(ParseBufs b) {
    if (threadIdx.x != 0) return;
    ParseOut* o = b.out;
    ParseState* st = b.state;
    if (o->overflow) return;
    const uint64_t V = o->valid, v0 = o->v0;
    o->reads = reads_in(V, v0);
    o->tail_start = b.eof ? b.len : (o->newlines ? (uint64_t)b.line_end[o->newlines - 1] + 1 : b.begin);
    if (o->min_len == 0xFFFFFFFFu) o->min_len = 0;
    int64_t pend = st->pending_pos;
    if (V > 0) {
        pend = -1;
        if (((v0 + V) & 3u) == 1u && b.want_pos) {  // the span ends with a header line
            const uint64_t k = o->any_high ? b.vline[V - 1] : V - 1;
            uint32_t s, e;
            line_bounds(b, k, s, e);
            pend = parse_pos(b.buf + s, e - s);
        }
    }
    st->valid_lines = v0 + V;
    st->errors += o->lines - V;
    st->reads += o->reads;
    st->pending_pos = pend;
}

__global__ __launch_bounds__(256) void k_emit(ParseBufs b, EmitSpan sp, uint64_t r_begin, uint64_t count,
                                              uint8_t* reads, uint16_t* rlen, int64_t* pos) {
    const bool ascii = !sp.any_high;
    const uint64_t v0 = sp.v0;
    const uint32_t ph = seq_phase(v0);
    const uint32_t l16 = threadIdx.x & 15;
    const uint64_t ng = (uint64_t)gridDim.x * 16;
    for (uint64_t g = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 4; g < count; g += ng) {
        const uint64_t j = ph + 4 * (r_begin + g);
        const uint64_t k = ascii ? j : b.vline[j];
        uint32_t st, en;
        line_bounds(b, k, st, en);
        uint32_t len = en - st;
        if (len > b.stride) len = 0;  // the span is flagged too_long; the host fails the file
        // 256 bytes of the row per pass of the group's 16 lanes (strides > 256: long reads)
        for (uint32_t c0 = 16u * l16; c0 < b.stride; c0 += 256u) {
            uint32_t w[4] = {0, 0, 0, 0};
            if (c0 < len) {
                const uint64_t a = (uint64_t)st + c0;
                const uint32_t* p = (const uint32_t*)(b.buf + (a & ~3ull));
                const uint32_t sh = (uint32_t)(a & 3u);
                const uint32_t d0 = p[0], d1 = p[1], d2 = p[2], d3 = p[3], d4 = p[4];
                const uint32_t nb = min(16u, len - c0);
                w[0] = __builtin_amdgcn_alignbyte(d1, d0, sh) & byte_mask(nb);
                w[1] = __builtin_amdgcn_alignbyte(d2, d1, sh) & byte_mask(nb > 4 ? nb - 4 : 0);
                w[2] = __builtin_amdgcn_alignbyte(d3, d2, sh) & byte_mask(nb > 8 ? nb - 8 : 0);
                w[3] = __builtin_amdgcn_alignbyte(d4, d3, sh) & byte_mask(nb > 12 ? nb - 12 : 0);
            }
            *(uint4*)(reads + g * b.stride + c0) = make_uint4(w[0], w[1], w[2], w[3]);
        }
        if (l16 == 0) rlen[g] = (uint16_t)len;
        if (pos) {  // the header before the sequence line, parsed by the group's 16 lanes
            int64_t p = sp.pending_in;
            if (j != 0) {
                const uint64_t kh = ascii ? j - 1 : b.vline[j - 1];
                uint32_t hs, he;
                line_bounds(b, kh, hs, he);
                p = group_parse_pos(b.buf, hs, he - hs, l16);
            }
            if (l16 == 0) pos[g] = p;
        }
    }
}

}  // namespace

hipError_t parse_preload() {
    int nb = 0;  // an occupancy query loads the kernel's code object (msw_ctx_prepare does the same)
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_count, 256, 0);
}

hipError_t launch_parse_a(const ParseBufs& b, hipStream_t stream) {
    const uint32_t nt = b.ntiles ? b.ntiles : 1;
    hipLaunchKernelGGL(k_count, dim3(nt), dim3(256), 0, stream, b);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(256), 0, stream, b);
    return hipGetLastError();
}

hipError_t launch_parse_b(const ParseBufs& b, uint64_t lines, bool any_high, hipStream_t stream) {
    const uint32_t nt = b.ntiles ? b.ntiles : 1;
    hipLaunchKernelGGL(k_line_ends, dim3(nt), dim3(256), 0, stream, b);
    if (any_high) {
        const uint32_t g = (uint32_t)std::min<uint64_t>(1024, (lines + 255) / 256 + 1);
        const uint32_t gc = (uint32_t)std::min<uint64_t>(1024, (lines + kScanChunk - 1) / kScanChunk + 1);
        hipLaunchKernelGGL(k_utf8, dim3(g), dim3(256), 0, stream, b);
        hipLaunchKernelGGL(k_vsum, dim3(gc), dim3(256), 0, stream, b);
        hipLaunchKernelGGL(k_vscan, dim3(1), dim3(1024), 0, stream, b);
        hipLaunchKernelGGL(k_vapply, dim3(gc), dim3(256), 0, stream, b);
    }
    const uint32_t gl = (uint32_t)std::min<uint64_t>(1024, (lines / 4 + 255) / 256 + 1);
    hipLaunchKernelGGL(k_lens, dim3(gl), dim3(256), 0, stream, b);
    hipLaunchKernelGGL(k_fin, dim3(1), dim3(64), 0, stream, b);
    return hipGetLastError();
}

hipError_t launch_emit_reads(const ParseBufs& b, const EmitSpan& sp, uint64_t r_begin, uint64_t count,
                             uint8_t* reads, uint16_t* read_len, int64_t* pos, hipStream_t stream) {
    if (count == 0) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>((count + 15) / 16, 8192);
    hipLaunchKernelGGL(k_emit, dim3((uint32_t)blocks), dim3(256), 0, stream, b, sp, r_begin, count, reads,
                       read_len, pos);
    return hipGetLastError();
}

}  // namespace msw
