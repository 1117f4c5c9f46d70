// msw_inflate.hip -- BGZF member inflate (RFC 1951 DEFLATE) and CRC-32 check
// on gfx950, one wave per member.
//
// Why on the GPU: the --full-wgs lane files are gzip'ed FASTQ.  The reference
// pipes each through `zcat` and splits lines into Strings on one core per file
// (smith_waterman/src/aligner.rs:107-178); even libdeflate on the host tops
// out near 1.6 M reads/s per CPU, two orders of magnitude below
// what one MI355X scores.  BGZF members are independent deflate streams of
// <= 64 KiB output whose sizes are in their headers, so a span of thousands of
// members inflates with thousands of waves at once and only compressed bytes
// cross PCIe.
//
// Mapping.  A wave owns a member.  Block headers and table builds run on
// wave-uniform values with the 64 lanes where the format is parallel
// (canonical code tables by ballots; 9-bit literal/length and 7-bit distance
// lookup tables in LDS).  The Huffman data is decoded by speculative windows:
//  * the only serial fact is where the next token starts, so lane L decodes
//    the token that would start at bit P + L (both table lookups, length and
//    distance with their extra bits) into a record; the scalar unit walks the
//    chain of records (token at lane k, next at k + its bits), and at each
//    chain token the output lanes from its first byte on take its record;
//  * lane b then makes output byte b of the window -- a literal byte, a byte
//    of the 2 KiB output ring in LDS (j mod dist back for overlapping
//    copies), a byte of the flushed output in L2, or an earlier lane's value
//    by pointer jumping when a match reads this window's own output -- and
//    one masked write stores the window's bytes in the ring; every completed
//    256-byte chunk is flushed to HBM with one coalesced store per lane;
//  * windows producing more than 64 bytes take a serial walk of the same
//    records, and tokens no window resolves (long codes, end of block,
//    invalid codes, the member's last bits) a one-token scalar step;
//  * the CRC-32 check is a second kernel: a wave reads the member's output
//    in coalesced 256-byte chunks, lane l folds dword l of every chunk into
//    its own state with a table-driven 256-byte advance, and the 64 lane
//    states are combined in a 6-level tree with GF(2) shift constants
//    (zlib's crc32_combine).
// Errors follow zlib's inflate (inftrees.c rules for code sets): any error
// marks the member and stops its wave; no byte is ever written outside the
// member's ISIZE bytes of output.
#include <algorithm>
#include <cstdlib>

#include "msw_gz.h"

namespace msw {
namespace {

#ifndef MSW_GZ_RING_KB
#define MSW_GZ_RING_KB 2
#endif
constexpr int kDefaultRingKb = MSW_GZ_RING_KB;  // 2: best measured throughput (tools/inflate_bench.py, profiles/r02/gz)

// MSW_GZ_PROFILE builds (tools/build_variant.sh gzprof -DMSW_GZ_PROFILE=1):
// per-member event counts and cycle stamps into prof[m * 16 ..].
#ifndef MSW_GZ_PROFILE
#define MSW_GZ_PROFILE 0
#endif
#if MSW_GZ_PROFILE
#define GZP(i, v) (pc[i] += (v))
#else
#define GZP(i, v) ((void)0)
#endif

constexpr uint32_t kChunk = 256;  // flush unit: 64 lanes x 4 bytes

// order of the code-length code lengths in a dynamic block header
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

constexpr uint32_t kFastBits = 9;   // lit/len lookup: next 9 stream bits -> up to 3 literals or one symbol
constexpr uint32_t kFastDBits = 7;  // distance lookup
// lit/len entry: [3:0] bits consumed, [5:4] n literals (their bytes in
// [31:8]); with n = 0: bit 6 = code longer than kFastBits or invalid
// (canonical decode), bit 7 = a length code; neither = end of block.
// A length code's entry is laid out for s_bfe_u32, whose control operand is
// offset [4:0] | width [22:16]: [3:0] code bits L (the extra bits' offset),
// [13:8] L + extra bits, [22:16] extra bits, [31:23] base length -- the
// entry itself extracts the extra bits, one SALU op.
constexpr uint32_t kFastLong = 0x40u;
constexpr uint32_t kFastMatch = 0x80u;
// distance entry, the same s_bfe_u32 layout: [3:0] code bits, [12:8] code +
// extra bits, [22:16] extra bits; the base distance sits in fast_dbase;
// bit 31 = code longer than kFastDBits or invalid
constexpr uint32_t kFastDLong = 0x80000000u;
// a lit/len "entry" for no code of the set (canonical decode failed)
constexpr uint32_t kFastBadE = 0x100u;

// s_bfe_u32 d, v, ctl: (v >> ctl[4:0]) & ((1 << ctl[22:16]) - 1), wave-uniform
// (it also writes SCC, which the compiler must not keep live across it)
__device__ __forceinline__ uint32_t sbfe(uint32_t v, uint32_t ctl) {
    uint32_t d;
    asm("s_bfe_u32 %0, %1, %2" : "=s"(d) : "s"(v), "s"(ctl) : "scc");
    return d;
}

// v_bfe_u32 d, v, off, wid: (v >> off[4:0]) & ((1 << wid[4:0]) - 1) per lane;
// the hardware reads only those bits, so a fast-table entry is passed whole
// as off and shifted once as wid (no masks)
__device__ __forceinline__ uint32_t vbfe(uint32_t v, uint32_t off, uint32_t wid) {
    uint32_t d;
    asm("v_bfe_u32 %0, %1, %2, %3" : "=v"(d) : "v"(v), "v"(off), "v"(wid));
    return d;
}

// v_readlane_b32 with the lane select held in the SGPR given (the builtin
// lets the compiler substitute any value with the same low 6 bits, which in
// the walk kept an extra copy of the record live: one s_mov per token)
__device__ __forceinline__ uint32_t readlane_s(uint32_t v, uint32_t lane_sel) {
    uint32_t d;
    asm("v_readlane_b32 %0, %1, %2" : "=s"(d) : "v"(v), "s"(lane_sel));
    return d;
}

__device__ __forceinline__ uint32_t len_base(uint32_t sym, uint32_t& extra) {
    if (sym < 265) { extra = 0; return sym - 254; }
    if (sym < 285) { extra = (sym - 261) >> 2; return ((4u + ((sym - 265) & 3u)) << extra) + 3u; }
    extra = 0;
    return 258;
}
__device__ __forceinline__ uint32_t dist_base(uint32_t d, uint32_t& extra) {
    if (d < 4) { extra = 0; return d + 1; }
    extra = (d >> 1) - 1;
    return ((2u + (d & 1u)) << extra) + 1u;
}

// Tables: ~3 KB per wave.  The code-length decode's scratch (lens, sym_c)
// lives in fast_ll, which is only built after it.  The output ring (the
// kernel's RING template parameter) comes on top: deflate distances reach
// 32 KiB, and FASTQ members use the whole range (a 64 KiB member of
// synthetic reads: 38 % of matches within 2 KiB, 72 % within 8 KiB, 93 %
// within 16 KiB); a match further back than the ring reads the flushed
// output from L2, so the ring size trades waves per SIMD against L2 trips.
struct __align__(16) InflateLds {
    union {
        uint32_t fast_ll[1u << kFastBits];
        struct {
            uint16_t sym_c[20];  // code-length alphabet
            uint8_t lens[320];   // code lengths of the block being built (<= 286 + 30)
        } hdr;
    } u;
    uint32_t fast_d[1u << kFastDBits];
    uint32_t fast_dbase[1u << kFastDBits];  // base distance of each fast_d entry (u32: one address for both)
    uint16_t sym_ll[288];  // lit/len symbols sorted by (code length, symbol)
    uint16_t sym_d[32];    // distance symbols
};
static_assert(sizeof(InflateLds) <= 3712, "inflate tables: <= 3.625 KB of LDS per wave (7 waves per SIMD with the 2 KiB ring)");

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x; }
// A call's result is divergent to the compiler; every control value of the
// decode loop must stay wave-uniform (SGPRs, scalar branches), so results of
// the out-of-line table builders go through readfirstlane.
__device__ __forceinline__ bool uni_bool(bool b) { return __builtin_amdgcn_readfirstlane(b ? 1 : 0) != 0; }

// zlib inftrees.c rules: kind 0 = code-length code (must be complete),
// 1 = lit/len, 2 = distance (incomplete only as a single 1-bit code).
// Builds the sorted symbol array and each lane's (lj_end, base) pair:
// lane L in 1..15 gets lim = (first[L] + count[L]) << (15 - L) and
// bas = offs[L] - first[L]; other lanes lim = 0.  Returns false on an
// over-subscribed or (disallowed) incomplete set.
__device__ __noinline__ bool build_code(const uint8_t* lens, uint32_t n, uint16_t* syms, uint32_t& lim,
                                        int32_t& bas, int kind) {
    const uint32_t lane = lane_id();
    uint32_t cnt = 0;
    for (uint32_t s0 = 0; s0 < n; s0 += 64) {
        const uint32_t s = s0 + lane;
        const uint32_t L = s < n ? lens[s] : 0u;
#pragma unroll
        for (uint32_t l = 1; l <= 15; ++l) {
            const uint32_t c = (uint32_t)__popcll(__ballot(L == l));
            if (lane == l) cnt += c;
        }
    }
    uint32_t code = 0, off = 0, maxlen = 0, slot = 0;
    int32_t left = 1;
    lim = 0;
    bas = 0;
#pragma unroll
    for (uint32_t L = 1; L <= 15; ++L) {
        const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cnt, (int)L);
        if (lane == L) {
            lim = (code + c) << (15 - L);
            bas = (int32_t)off - (int32_t)code;
            slot = off;
        }
        left = (left << 1) - (int32_t)c;
        if (left < 0) return false;  // over-subscribed
        if (c) maxlen = L;
        off += c;
        code = (code + c) << 1;
    }
    if (maxlen == 0) {  // no codes: every decode fails (a distance code may be unused)
        lim = 0;
        return kind != 1;
    }
    if (left > 0 && (kind == 0 || maxlen != 1)) return false;  // incomplete set
    // symbols sorted by (length, symbol): rank within a length by ballot
    for (uint32_t s0 = 0; s0 < n; s0 += 64) {
        const uint32_t s = s0 + lane;
        const uint32_t L = s < n ? lens[s] : 0u;
#pragma unroll
        for (uint32_t l = 1; l <= 15; ++l) {
            const uint64_t m = __ballot(L == l);
            if (m) {
                const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)slot, (int)l);
                if (L == l) {
                    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    syms[base + below] = (uint16_t)s;
                }
                if (lane == l) slot += (uint32_t)__popcll(m);
            }
        }
    }
    __syncthreads();
    return true;
}

// Lookup tables over the next kFastBits (lit/len) / kFastDBits (distance)
// stream bits, built from the canonical (lim, bas) pairs: an entry holds up to
// three literals whose codes all fit (sequence and quality letters of FASTQ
// have 1-4 bit codes, so one LDS read usually yields two or three output
// bytes), or one symbol, or the "long" flag for the ballot decode.  A code's
// length is exact from its known bits: r < lim[L] depends only on r's top L bits.
__device__ __noinline__ void build_fast(uint32_t lim_ll, int32_t bas_ll, uint32_t lim_d, int32_t bas_d,
                                        InflateLds& S) {
    const uint32_t lane = lane_id();
    uint32_t ll[16], ld[16];
    int32_t bl[16], bd[16];
#pragma unroll
    for (int L = 1; L <= 15; ++L) {
        ll[L] = (uint32_t)__builtin_amdgcn_readlane((int)lim_ll, L);
        bl[L] = __builtin_amdgcn_readlane(bas_ll, L);
        ld[L] = (uint32_t)__builtin_amdgcn_readlane((int)lim_d, L);
        bd[L] = __builtin_amdgcn_readlane(bas_d, L);
    }
    // one lit/len symbol from the low `known` bits of v: returns its length (0 = not determined)
    auto dec = [&](uint32_t v, uint32_t known, uint32_t& sym) __attribute__((always_inline)) -> uint32_t {
        const uint32_t r = __builtin_bitreverse32(v) >> 17;
        uint32_t L = 0;
        int32_t B = 0;
#pragma unroll
        for (int k = kFastBits; k >= 1; --k)
            if ((uint32_t)k <= known && r < ll[k]) {
                L = (uint32_t)k;
                B = bl[k];
            }
        if (L) sym = S.sym_ll[(uint32_t)(B + (int32_t)(r >> (15 - L)))];
        return L;
    };
    for (uint32_t i = lane; i < (1u << kFastBits); i += 64) {
        uint32_t s1 = 0, e = kFastLong;
        const uint32_t L1 = dec(i, kFastBits, s1);
        if (L1) {
            if (s1 == 256) {
                e = L1;  // end of block
            } else if (s1 >= 257 && s1 <= 285) {
                uint32_t x;
                const uint32_t base = len_base(s1, x);
                e = L1 | kFastMatch | ((L1 + x) << 8) | (x << 16) | (base << 23);
            } else if (s1 >= 256) {
                e = kFastLong;  // 286 / 287: the canonical decode reports it
            } else {
                uint32_t n = 1, used = L1, bytes = s1, s2 = 0;
                const uint32_t L2 = dec(i >> used, kFastBits - used, s2);
                if (L2 && s2 < 256) {
                    bytes |= s2 << 8;
                    ++n;
                    used += L2;
                    uint32_t s3 = 0;
                    const uint32_t L3 = dec(i >> used, kFastBits - used, s3);
                    if (L3 && s3 < 256) {
                        bytes |= s3 << 16;
                        ++n;
                        used += L3;
                    }
                }
                e = used | (n << 4) | (bytes << 8);
            }
        }
        S.u.fast_ll[i] = e;
    }
    for (uint32_t i = lane; i < (1u << kFastDBits); i += 64) {
        const uint32_t r = __builtin_bitreverse32(i) >> 17;
        uint32_t L = 0;
        int32_t B = 0;
#pragma unroll
        for (int k = kFastDBits; k >= 1; --k)
            if (r < ld[k]) {
                L = (uint32_t)k;
                B = bd[k];
            }
        uint32_t e = kFastDLong, base = 0;
        if (L) {
            const uint32_t d = S.sym_d[(uint32_t)(B + (int32_t)(r >> (15 - L)))];
            if (d <= 29) {
                uint32_t x;
                base = dist_base(d, x);
                e = L | ((L + x) << 8) | (x << 16);
            }
        }
        S.fast_d[i] = e;
        S.fast_dbase[i] = base;
    }
    __syncthreads();
}

// The bit reader: stream bits LSB-first from a 64-bit buffer (wave-uniform)
// refilled with dwords from a 64-dword window of the input held one per lane
// in a VGPR (v_readlane).  The next window is loaded when this one runs out,
// every 256 input bytes (~600 symbols): one memory latency there is ~1 % of
// the decode, and nothing in the symbol loop waits on memory.
struct Bits {
    const uint32_t* src;  // the span's compressed buffer as dwords
    uint32_t last;        // its last readable dword: every load is clamped to it
                          // (a buffer read in place from pinned host memory
                          // has no zero padding after the span)
    uint64_t bb;
    uint32_t bcnt;        // valid bits in bb
    uint32_t wi;          // dword index of the next dword to merge
    uint32_t wbase;       // dword index held by lane 0 of `cur`
    uint32_t cur;         // per lane: src[wbase + lane]
    uint32_t wmax;        // refills past this dword index mean truncated data

    __device__ __forceinline__ uint32_t ld(uint32_t i) const { return src[min(i, last)]; }
    __device__ __forceinline__ void prime(uint64_t byte_pos) {
        const uint32_t w = (uint32_t)(byte_pos >> 2), sh = 8u * (uint32_t)(byte_pos & 3);
        wbase = w;
        cur = ld(w + lane_id());
        bb = (uint64_t)((uint32_t)__builtin_amdgcn_readlane((int)cur, 0) >> sh);
        bcnt = 32u - sh;
        wi = w + 1;
    }
    // true if the refill stayed within the member (+ slack)
    __device__ __forceinline__ bool refill() {
        if (bcnt < 32) {
            if (wi > wmax) return false;
            if (wi - wbase >= 64) {
                wbase = wi;
                cur = ld(wbase + lane_id());
            }
            const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)cur, (int)(wi - wbase));
            bb |= (uint64_t)d << bcnt;
            bcnt += 32;
            ++wi;
        }
        return true;
    }
    // The token loop's refill (the caller checked bcnt < 32): no truncation
    // test -- past the member's end it merges whatever follows (window loads
    // clamped to wmax, so they stay in the buffer); the block loop tests
    // wi > wmax at every block header, which bounds a runaway decode, and a
    // member whose decode read past its end reports GZ_E_TRUNC (kernel end).
    __device__ __forceinline__ void refill_fast() {
        if (wi - wbase >= 64) {
            wbase = min(wi, wmax);
            cur = ld(wbase + lane_id());
        }
        const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)cur, (int)((wi - wbase) & 63u));
        bb |= (uint64_t)d << bcnt;
        bcnt += 32;
        ++wi;
    }
    __device__ __forceinline__ uint32_t peek(uint32_t n) const { return (uint32_t)bb & ((1u << n) - 1u); }
    __device__ __forceinline__ void drop(uint32_t n) {
        bb >>= n;
        bcnt -= n;
    }
    __device__ __forceinline__ uint32_t take(uint32_t n) {
        const uint32_t v = peek(n);
        drop(n);
        return v;
    }
    // stream bits consumed since byte 0 of the buffer
    __device__ __forceinline__ uint64_t bit_pos() const { return (uint64_t)wi * 32u - bcnt; }
};

// One Huffman symbol (canonical decode, see the file comment); -1 if the
// next bits are no code of this set.  Needs bcnt >= 15.
__device__ __forceinline__ int decode_sym(Bits& br, uint32_t lim, int32_t bas, const uint16_t* syms) {
    const uint32_t r = __builtin_bitreverse32((uint32_t)br.bb) >> 17;  // next 15 bits, first as MSB
    const uint64_t m = __ballot(r < lim);
    if (m == 0) return -1;
    const uint32_t L = (uint32_t)__builtin_ctzll(m);
    const int32_t base = __builtin_amdgcn_readlane(bas, (int)L);
    const uint32_t idx = (uint32_t)(base + (int32_t)(r >> (15 - L)));
    br.drop(L);
    return (int)__builtin_amdgcn_readfirstlane((uint32_t)syms[idx]);
}

__device__ __forceinline__ uint32_t coherent_load(const uint8_t* p) {
    return __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// waves per SIMD the LDS allows (160 KB per CU) for a ring of RING bytes
template <uint32_t RING>
constexpr int inflate_waves() {
    return (int)(160u * 1024u / (RING + 64u + (uint32_t)sizeof(InflateLds)) / 4u) > 8
               ? 8
               : (int)(160u * 1024u / (RING + 64u + (uint32_t)sizeof(InflateLds)) / 4u);
}

template <uint32_t RING>
__global__ __launch_bounds__(64, inflate_waves<RING>()) void gz_inflate_kernel(const uint8_t* __restrict__ cdata,
                                                        uint32_t cdata_last, const GzMember* __restrict__ members, uint32_t n,
                                                        uint8_t* __restrict__ out, uint32_t* __restrict__ status,
                                                        uint32_t* __restrict__ any_error, uint32_t* __restrict__ prof) {
    constexpr uint32_t kRing = RING, kRingMask = RING - 1;
#if MSW_GZ_PROFILE
    uint32_t pc[12] = {0};
    const uint64_t t_start = __builtin_amdgcn_s_memtime();
#endif
    static_assert((RING & (RING - 1)) == 0 && RING >= 1024, "ring: a power of two >= 1 KiB");
    __shared__ InflateLds S;
    // the ring, then 64 per-lane dummy bytes: lane-conditional ring writes
    // become unconditional writes whose inactive lanes hit their own dummy
    // byte (a VALU select instead of exec-mask SALU work in the hot loop)
    __shared__ uint32_t ring_words[RING / 4 + 16];
    // one member per block, or (a capped grid, launch_gz_inflate) members
    // blockIdx.x, + gridDim.x, ... in turn: the wave's LDS tables and ring are
    // rebuilt per member anyway
    for (uint32_t m = blockIdx.x; m < n; m += gridDim.x) {
        const uint32_t lane = lane_id();
        uint8_t* ring = (uint8_t*)ring_words;
        const uint32_t dummy = RING + lane;  // this lane's dummy byte
        const uint32_t lit_shift = 8u + 8u * min(lane, 2u);
        const GzMember mem = members[m];
        uint8_t* dst = out + mem.ooff;
        const uint32_t isize = mem.isize;
        const bool dst_al4 = (mem.ooff & 3) == 0;

        Bits br;
        br.src = (const uint32_t*)cdata;
        br.last = cdata_last;
        br.wmax = (uint32_t)((mem.coff + mem.clen) >> 2) + 2u;
        br.prime(mem.coff);

        uint32_t opos = 0, flushed = 0, err = GZ_OK;
        uint32_t lim_ll = 0, lim_d = 0, lim_c = 0;
        int32_t bas_ll = 0, bas_d = 0, bas_c = 0;
        int tables = -1;  // 1 = fixed tables loaded, 2 = dynamic

        // flush [from, from + 256) of the output (ring-resident) to HBM
        auto flush_chunk = [&](uint32_t from) __attribute__((always_inline)) {
            const uint32_t v = ring_words[((from + 4u * lane) & kRingMask) >> 2];
            uint8_t* d = dst + from + 4u * lane;
            if (dst_al4) {
                *(uint32_t*)d = v;
            } else {
                d[0] = (uint8_t)v;
                d[1] = (uint8_t)(v >> 8);
                d[2] = (uint8_t)(v >> 16);
                d[3] = (uint8_t)(v >> 24);
            }
        };

        bool last = false;
        while (!last && err == GZ_OK) {
            if (br.wi > br.wmax || !br.refill()) { err = GZ_E_TRUNC; break; }
#if MSW_GZ_PROFILE
            const uint64_t t_hdr = __builtin_amdgcn_s_memtime();
#endif
            GZP(9, 1);
            const uint32_t hdr = br.take(3);
            last = (hdr & 1u) != 0;
            const uint32_t btype = hdr >> 1;
            if (btype == 0) {
                // stored block: byte-align, LEN, NLEN, LEN raw bytes
                br.drop(br.bcnt & 7u);
                if (!br.refill()) { err = GZ_E_TRUNC; break; }
                const uint32_t len = br.take(16), nlen = br.take(16);
                if (len != (~nlen & 0xFFFFu)) { err = GZ_E_STORED; break; }
                if (opos + len > isize) { err = GZ_E_OVERRUN; break; }
                uint32_t k = 0;
                while (k < len && br.bcnt >= 8) {  // bytes already in the bit buffer
                    const uint32_t v = br.take(8);
                    if (lane == 0) ring[opos & kRingMask] = (uint8_t)v;
                    ++opos;
                    ++k;
                    if ((opos & (kChunk - 1)) == 0) { flush_chunk(opos - kChunk); flushed = opos; }
                }
                if (k < len) {
                    // the buffer is empty: the stream continues at byte 4 * wi
                    uint64_t p = (uint64_t)br.wi * 4u;
                    const uint32_t rest = len - k;
                    if (p + rest > mem.coff + mem.clen) { err = GZ_E_TRUNC; break; }
                    for (uint32_t j0 = 0; j0 < rest; j0 += kChunk) {
                        const uint32_t j = j0 + 4u * lane;
                        if (j < rest) {
                            const uint64_t q = p + j;
                            const uint32_t lo = br.ld((uint32_t)(q >> 2)), hi = br.ld((uint32_t)(q >> 2) + 1u);
                            const uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(q & 3));
                            const uint32_t nb = min(4u, rest - j);
                            // opos already counts the earlier rounds (j0 bytes)
                            for (uint32_t b = 0; b < nb; ++b)
                                ring[(opos + 4u * lane + b) & kRingMask] = (uint8_t)(v >> (8 * b));
                        }
                        const uint32_t adv = min(kChunk, rest - j0);
                        opos += adv;
                        while (opos - flushed >= kChunk) { flush_chunk(flushed); flushed += kChunk; }
                    }
                    br.prime(p + rest);
                }
                continue;
            }
            if (btype == 3) { err = GZ_E_BTYPE; break; }
            if (btype == 1) {
                if (tables != 1) {
                    for (uint32_t s = lane; s < 288; s += 64)
                        S.u.hdr.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
                    __syncthreads();
                    (void)uni_bool(build_code(S.u.hdr.lens, 288, S.sym_ll, lim_ll, bas_ll, 1));
                    for (uint32_t s = lane; s < 32; s += 64) S.u.hdr.lens[s] = 5;
                    __syncthreads();
                    (void)uni_bool(build_code(S.u.hdr.lens, 32, S.sym_d, lim_d, bas_d, 2));
                    build_fast(lim_ll, bas_ll, lim_d, bas_d, S);
                    tables = 1;
                }
            } else {
                // dynamic block header
                if (!br.refill()) { err = GZ_E_TRUNC; break; }
                const uint32_t nlen = br.take(5) + 257, ndist = br.take(5) + 1, ncode = br.take(4) + 4;
                if (nlen > 286 || ndist > 30) { err = GZ_E_HEADER; break; }
                if (lane < 19) S.u.hdr.lens[lane] = 0;
                __syncthreads();
                // code-length code lengths, 3 bits each, in kClOrder (RFC 1951 3.2.7)
                for (uint32_t i = 0; i < ncode; ++i) {
                    if (!br.refill()) { err = GZ_E_TRUNC; break; }
                    const uint32_t v = br.take(3);
                    if (lane == 0) S.u.hdr.lens[kClOrder[i]] = (uint8_t)v;
                }
                if (err) break;
                __syncthreads();
                if (!uni_bool(build_code(S.u.hdr.lens, 19, S.u.hdr.sym_c, lim_c, bas_c, 0))) { err = GZ_E_CODES; break; }
                // lit/len + distance code lengths (one sequence; repeats may cross)
                const uint32_t total = nlen + ndist;
                uint32_t idx = 0;
                while (idx < total) {
                    if (!br.refill()) { err = GZ_E_TRUNC; break; }
                    const int sym = decode_sym(br, lim_c, bas_c, S.u.hdr.sym_c);
                    if (sym < 0) { err = GZ_E_CODES; break; }
                    if (sym < 16) {
                        if (lane == 0) S.u.hdr.lens[idx] = (uint8_t)sym;
                        ++idx;
                        continue;
                    }
                    uint32_t rep, val = 0;
                    if (sym == 16) {
                        if (idx == 0) { err = GZ_E_HEADER; break; }
                        val = __builtin_amdgcn_readfirstlane((uint32_t)S.u.hdr.lens[idx - 1]);
                        rep = 3 + br.take(2);
                    } else if (sym == 17) {
                        rep = 3 + br.take(3);
                    } else {
                        rep = 11 + br.take(7);
                    }
                    if (idx + rep > total) { err = GZ_E_HEADER; break; }
                    for (uint32_t k = lane; k < rep; k += 64) S.u.hdr.lens[idx + k] = (uint8_t)val;
                    idx += rep;
                }
                if (err) break;
                __syncthreads();
                if (__builtin_amdgcn_readfirstlane((uint32_t)S.u.hdr.lens[256]) == 0) { err = GZ_E_CODES; break; }
                if (!uni_bool(build_code(S.u.hdr.lens, nlen, S.sym_ll, lim_ll, bas_ll, 1))) { err = GZ_E_CODES; break; }
                if (!uni_bool(build_code(S.u.hdr.lens + nlen, ndist, S.sym_d, lim_d, bas_d, 2))) { err = GZ_E_CODES; break; }
                build_fast(lim_ll, bas_ll, lim_d, bas_d, S);
                tables = 2;
            }
            // Huffman-coded data until end-of-block.  Token loop with the next
            // lookup issued before the current token's ring writes / copy, so its
            // LDS latency overlaps them.  ISIZE is enforced where output leaves
            // the ring (flush) and at the end; the ring absorbs an overrun.
            auto lookup = [&]() __attribute__((always_inline)) -> uint32_t {
                return S.u.fast_ll[(uint32_t)br.bb & ((1u << kFastBits) - 1u)];
            };
            auto flush_to = [&]() __attribute__((always_inline)) -> bool {
                if (opos > isize) return false;
                while (opos - flushed >= kChunk) { flush_chunk(flushed); flushed += kChunk; }
                return true;
            };
#if MSW_GZ_PROFILE
            GZP(1, (uint32_t)(__builtin_amdgcn_s_memtime() - t_hdr));
#endif
            // A code longer than the table (or invalid), decoded canonically and
            // returned as the table entry it would have had (no bits dropped): a
            // one-literal entry, a length entry, end of block, or kFastBadE --
            // the token loop then treats it like any table entry.
            auto slow_ll = [&]() __attribute__((always_inline)) -> uint32_t {
                const uint32_t r = __builtin_bitreverse32((uint32_t)br.bb) >> 17;  // next 15 bits, first as MSB
                const uint64_t m = __ballot(r < lim_ll);
                if (m == 0) return kFastBadE;
                const uint32_t L = (uint32_t)__builtin_ctzll(m);
                const int32_t base = __builtin_amdgcn_readlane(bas_ll, (int)L);
                const uint32_t sym =
                    __builtin_amdgcn_readfirstlane((uint32_t)S.sym_ll[(uint32_t)(base + (int32_t)(r >> (15 - L)))]);
                if (sym < 256) return L | (1u << 4) | (sym << 8);
                if (sym == 256) return L;
                if (sym > 285) return kFastBadE;
                uint32_t x;
                const uint32_t b = len_base(sym, x);
                return L | kFastMatch | ((L + x) << 8) | (x << 16) | (b << 23);
            };
            if (!br.refill()) { err = GZ_E_TRUNC; break; }
            // Speculative window decode.  The serial part of inflate is only
            // "where does the next token start"; everything else about a token
            // (table lookups, length and distance with their extra bits) is a
            // function of its start bit.  So lane L decodes the token that
            // WOULD start at bit P + L of the stream (64 candidate starts, all
            // on the VALU, both table lookups per lane), packs it into one
            // dword, and the wave then walks the chain -- token at offset k,
            // next at k + its bits -- with one v_readlane per token, doing the
            // ring writes / copies in order.  A window covers 64 bits (~4
            // tokens of FASTQ); the scalar unit, which bounds the one-token-at-
            // a-time loop (~50 SALU per match token), only runs the walk.
            // Tokens the window does not resolve -- codes longer than the fast
            // tables, end of block, invalid codes, a distance too far back, and
            // the last 112 bits of the member -- go to the scalar step below
            // (one token, the exact bit reader and error rules of the loop it
            // replaces), after which the window resumes at its end.
            //   info bits: [31] simple, [30] match, [5:0] 0 (the walk's slot);
            //   match:   [14:6] length, [29:15] distance - 1
            //   literal: [29:6] the bytes (1..3)
            //   nxo: the next token's lane | output length << 8 (255: not simple)
            // Lanes past the match's end repeat its last byte (the same value to
            // the same ring address), so no lane needs a select or a dummy byte.
            auto copy_near = [&](uint32_t len, uint32_t dist) __attribute__((always_inline)) {
                const uint32_t last = len - 1u;
                if (dist >= len) {
                    // ring -> ring, source and destination apart: byte j from
                    // byte j of the source (no modulo on the dependent path)
                    const uint32_t base = opos - dist;
                    uint32_t j0 = 0;
                    do {
                        const uint32_t j = min(j0 + lane, last);
                        const uint8_t v = ring[(base + j) & kRingMask];
                        ring[(opos + j) & kRingMask] = v;
                        j0 += 64;
                    } while (j0 < len);
                } else {
                    // overlapping (dist < len <= 258, so within the ring): byte j
                    // copies source byte j mod dist (the last `dist` bytes repeat)
                    const float rd = __builtin_amdgcn_rcpf((float)dist);
                    const uint32_t base = opos - dist;
                    uint32_t j0 = 0;
                    do {
                        const uint32_t j = min(j0 + lane, last);
                        int32_t r = (int32_t)j - (int32_t)((uint32_t)((float)j * rd)) * (int32_t)dist;
                        r += r < 0 ? (int32_t)dist : 0;
                        r -= r >= (int32_t)dist ? (int32_t)dist : 0;
                        const uint8_t v = ring[(base + (uint32_t)r) & kRingMask];
                        ring[(opos + j) & kRingMask] = v;
                        j0 += 64;
                    } while (j0 < len);
                }
            };
            auto copy_far = [&](uint32_t len, uint32_t dist) __attribute__((always_inline)) {
                const uint32_t last = len - 1u;
                {
                    // further back than the ring: the flushed output in L2 (the
                    // source ends well before `flushed`), once the flush stores
                    // have landed
                    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
                    const uint64_t base = mem.ooff + (uint64_t)(opos - dist);
                    uint32_t j0 = 0;
                    do {
                        const uint32_t j = min(j0 + lane, last);
                        const uint64_t q = base + j;
                        const uint32_t w = coherent_load(out + (q & ~(uint64_t)3));
                        ring[(opos + j) & kRingMask] = (uint8_t)(w >> (8u * (uint32_t)(q & 3)));
                        j0 += 64;
                    } while (j0 < len);
                }
            };
            auto copy_match = [&](uint32_t len, uint32_t dist) __attribute__((always_inline)) {
                if (dist + len <= kRing) copy_near(len, dist);
                else copy_far(len, dist);
            };
            const uint32_t lit_shift6 = 6u + 8u * min(lane, 2u);
            // lane l: ceil(4096 / l) (lane 0: 0).  A window lane's offset off
            // < 64 into a match of distance d has off mod d = off - d * ((off *
            // M) >> 12) with M = this value of lane min(d, 64) mod 64: exact for
            // d < 64 (the estimate's error is below off / 4096 < 1 / d), and
            // d >= 64 reads lane 0 (M = 0: off mod d = off).  Integer ops and
            // one ds_bpermute instead of a float reciprocal and a 32-bit multiply.
            const uint32_t rmag = lane ? (4096u + lane - 1u) / lane : 0u;
            const uint64_t cend = mem.coff + mem.clen;
            const uint32_t ew = (uint32_t)(cend >> 2), eb = 8u * (uint32_t)(cend & 3u);
            // stream position (dword, bit) of the bit reader: wi * 32 - bcnt
            uint32_t pw = br.wi - (br.bcnt >> 5) - ((br.bcnt & 31u) ? 1u : 0u);
            uint32_t pb = (32u - (br.bcnt & 31u)) & 31u;
            uint32_t bad = 0;
            // the window runs while the member has >= 112 bits left at its start
            // (remain = (ew - pw) * 32 + eb - pb >= 112 <=> pw <= pw_last): the
            // last token of a window starts below bit 64 and takes <= 48 bits
            const uint32_t pw_last = ew >= 4u ? ew - 4u : 0u;  // (4 * 32 + eb - pb >= 112 holds when eb >= pb - 16)
            for (;;) {
                uint32_t k = 64;
                const bool room = pw < pw_last || (pw == pw_last && ew >= 4u && eb + 16u >= pb);
                if (room) {  // every candidate token ends inside the member
#if MSW_GZ_PROFILE
                    const uint64_t t_w = __builtin_amdgcn_s_memtime();
#endif
                    if (pw - br.wbase > 59u) {
                        br.wbase = pw;
                        br.cur = br.ld(pw + lane);
                    }
                    // lane L's stream bits from bit P + L: dwords j .. j + 2 of the
                    // window, j = (pb + L) / 32, fetched from `cur` across lanes
                    const uint32_t o = pb + lane, bs = o & 31u;
                    const uint32_t base4 = (pw - br.wbase) << 2;  // uniform: scalar unit
                    uint32_t dw = o >> 5;
                    asm("" : "+v"(dw));  // keeps (o >> 5) << 2 from becoming a shift and a mask
                    const int a0 = (int)((dw << 2) + base4);  // one v_lshl_add_u32
                    const uint32_t A = (uint32_t)__builtin_amdgcn_ds_bpermute(a0, (int)br.cur);
                    const uint32_t B = (uint32_t)__builtin_amdgcn_ds_bpermute(a0 + 4, (int)br.cur);
                    const uint32_t C = (uint32_t)__builtin_amdgcn_ds_bpermute(a0 + 8, (int)br.cur);
                    const uint32_t x = __builtin_amdgcn_alignbit(B, A, bs);  // stream bits [P + lane, +32)
                    const uint32_t y = __builtin_amdgcn_alignbit(C, B, bs);  // [+32, +64)
                    const uint32_t e = S.u.fast_ll[x & ((1u << kFastBits) - 1u)];
                    const uint32_t c = (e >> 8) & 63u;                      // a length's code + extra bits
                    const uint32_t z = __builtin_amdgcn_alignbit(y, x, c);  // the distance's bits
                    const uint32_t di = z & ((1u << kFastDBits) - 1u);
                    const uint32_t ed = S.fast_d[di], dbase = S.fast_dbase[di];
                    // (entries laid out for bfe: offset in [4:0], width in [20:16]; see kFastMatch)
                    const uint32_t len = (e >> 23) + vbfe(x, e, e >> 16);
                    const uint32_t dist = dbase + vbfe(z, ed, ed >> 16);
                    const uint32_t tm = c + ((ed >> 8) & 31u);
                    // bits 5:0 of both records stay 0: the walk puts the token's
                    // first output byte in the window there
                    const uint32_t lit = 0x80000000u | ((e >> 8) << 6);
                    const uint32_t mat = 0xC0000000u | (len << 6) | ((dist - 1u) << 15);
                    const uint32_t m_lit = 0u - (uint32_t)((e & 0x30u) != 0);
                    // a match resolves here if both codes were in the fast tables
                    // and its distance reaches no further back than the output
                    // so far (opos only grows during the walk; a match that fails
                    // this but not the exact test goes to the scalar step, which
                    // copies it)
                    const uint32_t m_mat = 0u - (uint32_t)((e & kFastMatch) != 0 && (ed & kFastDLong) == 0 && dist <= opos);
                    const uint32_t info = (lit & m_lit) | (mat & m_mat & ~m_lit);
                    GZP(7, 1);
#if MSW_GZ_PROFILE
                    (void)__builtin_amdgcn_readfirstlane(info);  // the decode has landed
                    const uint64_t t_k = __builtin_amdgcn_s_memtime();
                    GZP(3, (uint32_t)(t_k - t_w));
#endif
                    // Lane-parallel emission.  The chain is walked on the scalar
                    // unit from a per-lane record "next token's lane (255: this
                    // lane's token is not simple) | output length << 8"; at each
                    // chain token every output lane b >= (bytes so far) takes the
                    // token's record and first byte (a later token overwrites), so
                    // after the walk lane b holds the token covering output byte
                    // b.  Then lane b makes that byte -- a literal byte, a ring
                    // byte, a byte of the flushed output in L2, or (a match
                    // reading this window's own output) the value of an earlier
                    // lane by pointer jumping -- and one ring write stores the
                    // window's W bytes.  Windows of more than 64 output bytes take
                    // the serial walk.
                    // (a lane L whose token is not simple: "next lane" 192 + L, length
                    // 0 -- past any simple token's next lane, <= 111, and it names L)
                    uint32_t nx_lit = (lane + (e & 15u)) | (((e >> 4) & 3u) << 8), nx_mat = (lane + tm) | (len << 8);
                    asm volatile("" : "+v"(nx_lit), "+v"(nx_mat));  // both on every lane, then selects
                    const uint32_t nxo = m_lit ? nx_lit : (m_mat ? nx_mat : 192u + lane);
                    // The chain's first token starts the window: every lane takes
                    // it.  A later token's record carries its first byte W in bits
                    // 5:0 (OR'd on the scalar unit; W < 64 for every token of a
                    // window that emits), so a lane's select is one v_cndmask.
                    uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)nxo, 0);
                    uint32_t ti = (uint32_t)__builtin_amdgcn_readlane((int)info, 0);
                    uint32_t W = t >> 8;
                    // one exit: k leaves the window (>= 64) or hits a token that
                    // is not simple (k = 192 + its lane; it added nothing)
                    k = t & 255u;
                    while (k < 64) {
                        t = readlane_s(nxo, k);
                        const uint32_t s0 = readlane_s(info, k) | W;
                        ti = lane >= W ? s0 : ti;
                        W += t >> 8;
                        k = t & 255u;
                    }
                    if (k >= 192u) k -= 192u;
                    if (W <= 64u) {
                        if (W) {
                            // offset in the token: lane - its first byte (ti's bits 5:0)
                            const uint32_t off = (lane - ti) & 63u;
                            const bool lit = (ti & 0x40000000u) == 0;
                            const uint32_t d = ((ti >> 15) & 0x7FFFu) + 1u;
                            // overlapping copies repeat the token's last d bytes:
                            // r = off mod d (see rmag; lane address wraps mod 64)
                            const uint32_t m = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(min(d, 64u) << 2), (int)rmag);
                            const uint32_t q = __umul24(off, m) >> 12;  // floor(off / d)
                            // window-relative source: start + (off mod d) - d = lane - d (q + 1)
                            const int32_t src = (int32_t)lane - __mul24((int32_t)(q + 1u), (int32_t)d);
                            const bool dep = !lit && src >= 0;
                            const bool far = !lit && src < -(int32_t)RING;
                            // Both candidate bytes, then a select: the ring read
                            // runs on every lane (a literal lane's address is any
                            // ring byte) instead of behind an exec-mask branch.
                            uint32_t rbyte = ring[(opos + (uint32_t)src) & kRingMask];
                            // keeps the load out of a select-to-branch rewrite
                            asm volatile("" : "+v"(rbyte));
                            uint32_t val = lit ? (((ti >> 6) >> (8u * (off & 3u))) & 0xFFu) : rbyte;
                            // Lane masks straight from v_cmp into SGPRs (a ballot of
                            // a bool went through a VGPR and back: 2 VALU each)
                            const uint64_t in_w = __builtin_amdgcn_uicmp(lane, W, 36 /* ult */);
                            const uint64_t not_lit = __builtin_amdgcn_uicmp(ti & 0x40000000u, 0u, 33 /* ne */);
                            if (__builtin_amdgcn_sicmp(src, -(int32_t)RING, 40 /* slt */) & not_lit & in_w) {
#if MSW_GZ_PROFILE
                                const uint64_t t_far = __builtin_amdgcn_s_memtime();
#endif
                                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the flush stores have landed
                                const uint64_t q = mem.ooff + (uint64_t)(far ? opos + (uint32_t)src : 0u);
                                const uint32_t w = coherent_load(out + (q & ~(uint64_t)3));
                                if (far) val = (w >> (8u * (uint32_t)(q & 3))) & 0xFFu;
#if MSW_GZ_PROFILE
                                (void)__builtin_amdgcn_readfirstlane(val);  // the load has landed
                                GZP(6, 1);
                                GZP(10, (uint32_t)(__builtin_amdgcn_s_memtime() - t_far));
#endif
                            }
                            // bytes made by an earlier lane of this window: follow
                            // the pointers (a resolved lane points to itself)
                            uint32_t ptr = dep ? (uint32_t)src : lane;
                            while (__builtin_amdgcn_uicmp(ptr, lane, 33 /* ne */) & in_w) {
                                const int pa = (int)(ptr << 2);
                                const uint32_t tv = (uint32_t)__builtin_amdgcn_ds_bpermute(pa, (int)val);
                                const uint32_t tp = (uint32_t)__builtin_amdgcn_ds_bpermute(pa, (int)ptr);
                                const bool settle = ptr != lane && tp == ptr;
                                val = settle ? tv : val;
                                ptr = settle ? lane : tp;
                            }
                            // lanes past the window's W bytes store to their dummy byte
                            ring[lane < W ? ((opos + lane) & kRingMask) : dummy] = (uint8_t)val;
                            GZP(5, 1);
                            opos += W;
                            if (__builtin_expect(opos - flushed >= kChunk, 0)) {
                                if (opos > isize) bad = GZ_E_OVERRUN;
                                else do { flush_chunk(flushed); flushed += kChunk; } while (opos - flushed >= kChunk);
                            }
                        }
                    } else {
                        GZP(2, 1);
                        // the walk: one exit (k past the window); a token the window
                        // cannot take, or an overrun, ends it by pushing k out of range
                        k = 0;
                        uint32_t kstop = 0;
                        do {
                            const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)info, (int)k);
                            const uint32_t tn = (uint32_t)__builtin_amdgcn_readlane((int)nxo, (int)k);
                            if (s & 0x40000000u) {
                                const uint32_t ln = tn >> 8, ds = ((s >> 15) & 0x7FFFu) + 1u;
                                GZP(5, 1);
                                copy_match(ln, ds);
                                opos += ln;
                                k = tn & 255u;
                            } else if ((int32_t)s < 0) {
                                GZP(2, 1);
                                const uint32_t nlit = tn >> 8;
                                ring[lane < nlit ? ((opos + lane) & kRingMask) : dummy] = (uint8_t)(s >> lit_shift6);
                                opos += nlit;
                                k = tn & 255u;
                            } else {
                                kstop = k;  // not a simple token: the scalar step takes it
                                k = 0x10000u;
                            }
                            if (__builtin_expect(opos - flushed >= kChunk, 0)) {
                                if (opos > isize) {
                                    bad = GZ_E_OVERRUN;
                                    kstop = k;
                                    k = 0x10000u;
                                } else {
                                    do { flush_chunk(flushed); flushed += kChunk; } while (opos - flushed >= kChunk);
                                }
                            }
                        } while (k < 64);
                        if (k == 0x10000u) k = kstop;
                    }
#if MSW_GZ_PROFILE
                    GZP(11, (uint32_t)(__builtin_amdgcn_s_memtime() - t_k));
#endif
                    pb += k;
                    pw += pb >> 5;
                    pb &= 31u;
                    if (bad) {
                        br.wi = pw + 1;  // the position for the truncation test at the end
                        br.bcnt = 32u - pb;
                        break;
                    }
                    if (k >= 64) continue;
                }
                // Scalar step: one token from (pw, pb) with the bit reader.
                GZP(4, 1);
                if (pw - br.wbase > 62u) {
                    br.wbase = min(pw, br.wmax);
                    br.cur = br.ld(br.wbase + lane);
                }
                {
                    const uint32_t q = pw - br.wbase;
                    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)br.cur, (int)(q & 63u));
                    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)br.cur, (int)((q + 1u) & 63u));
                    br.bb = ((((uint64_t)hi) << 32) | lo) >> pb;
                    br.bcnt = 64u - pb;
                    br.wi = pw + 2u;
                }
                uint32_t e = __builtin_amdgcn_readfirstlane(lookup());
                if (e & kFastLong) e = slow_ll();
                bool eob = false;
                if (e & 0x30u) {
                    const uint32_t nlit = (e >> 4) & 3u;
                    br.drop(e & 15u);
                    if (br.bcnt < 32) br.refill_fast();
                    ring[lane < nlit ? ((opos + lane) & kRingMask) : dummy] = (uint8_t)(e >> lit_shift);
                    opos += nlit;
                    if (opos - flushed >= kChunk && !flush_to()) bad = GZ_E_OVERRUN;
                } else if (!(e & kFastMatch)) {  // end of block, or no code of this set
                    if (e & kFastBadE) bad = GZ_E_SYMBOL;
                    else { br.drop(e & 15u); eob = true; }
                } else {
                    const uint32_t len = (e >> 23) + sbfe((uint32_t)br.bb, e);
                    br.drop((e >> 8) & 63u);
                    if (br.bcnt < 32) br.refill_fast();
                    const uint32_t di = (uint32_t)br.bb & ((1u << kFastDBits) - 1u);
                    uint32_t ed = __builtin_amdgcn_readfirstlane(S.fast_d[di]);
                    uint32_t dbase = __builtin_amdgcn_readfirstlane(S.fast_dbase[di]);
                    if (ed & kFastDLong) {
                        const uint32_t r = __builtin_bitreverse32((uint32_t)br.bb) >> 17;
                        const uint64_t m = __ballot(r < lim_d);
                        uint32_t L = 0, d = 31;
                        if (m) {
                            L = (uint32_t)__builtin_ctzll(m);
                            const int32_t base = __builtin_amdgcn_readlane(bas_d, (int)L);
                            d = __builtin_amdgcn_readfirstlane((uint32_t)S.sym_d[(uint32_t)(base + (int32_t)(r >> (15 - L)))]);
                        }
                        ed = 0;
                        dbase = 0xFFFFFFFFu;
                        if (d > 29) {
                            bad = GZ_E_SYMBOL;
                        } else {
                            uint32_t xb;
                            dbase = dist_base(d, xb);
                            ed = L | ((L + xb) << 8) | (xb << 16);
                        }
                    }
                    const uint32_t dist = dbase + sbfe((uint32_t)br.bb, ed);
                    br.drop((ed >> 8) & 31u);
                    if (br.bcnt < 32) br.refill_fast();
                    if (dist > opos) {
                        bad = bad ? bad : (uint32_t)GZ_E_DIST;
                    } else {
                        copy_match(len, dist);
                        opos += len;
                        if (opos - flushed >= kChunk && !flush_to()) bad = GZ_E_OVERRUN;
                    }
                }
                if (bad || eob) break;
                pw = br.wi - (br.bcnt >> 5) - ((br.bcnt & 31u) ? 1u : 0u);
                pb = (32u - (br.bcnt & 31u)) & 31u;
            }
            if (bad) {
                err = bad;
                break;
            }
        }
        // a decode that ran into the bytes after the member (its last refills
        // merge them unchecked) failed because the member is truncated
        if (err != GZ_OK && br.bit_pos() > (mem.coff + mem.clen) * 8u) err = GZ_E_TRUNC;
        if (err == GZ_OK) {
            if (opos > isize) err = GZ_E_OVERRUN;
            else if (opos != isize) err = GZ_E_SIZE;
            else if ((br.bit_pos() - mem.coff * 8u + 7u) / 8u > mem.clen) err = GZ_E_TRUNC;
        }
        if (err == GZ_OK) {
            // the last partial chunk
            for (uint32_t k = lane; k < opos - flushed; k += 64) dst[flushed + k] = ring[(flushed + k) & kRingMask];
        }
        if (lane == 0) {
            status[m] = err;
            if (err) atomicOr(any_error, 1u);
        }
#if MSW_GZ_PROFILE
        pc[0] = (uint32_t)(__builtin_amdgcn_s_memtime() - t_start);
        if (prof && lane == 0)
            for (int i = 0; i < 12; ++i) prof[m * 16 + i] = pc[i];
        for (int i = 0; i < 12; ++i) pc[i] = 0;
#else
        (void)prof;
#endif
    }  // members
}

// ---------------------------------------------------------------------------
// CRC-32 (zlib's polynomial, reflected) of each member's output.
// ---------------------------------------------------------------------------
constexpr uint32_t kPoly = 0xEDB88320u;

__device__ uint32_t multmodp(uint32_t a, uint32_t b) {  // a * b mod p(x), reflected (x^0 = bit 31)
    uint32_t p = 0;
    for (uint32_t m = 1u << 31; m; m >>= 1) {
        if (a & m) p ^= b;
        b = b & 1 ? (b >> 1) ^ kPoly : b >> 1;
    }
    return p;
}

__device__ uint32_t x2nmodp(const GzCrcConsts& c, uint64_t n, uint32_t k) {  // x^(n * 2^k) mod p
    uint32_t p = 1u << 31;
    while (n) {
        if (n & 1) p = multmodp(c.x2n[k & 31], p);
        n >>= 1;
        ++k;
    }
    return p;
}

// One wave per member, four members per block (the advance tables are shared
// in LDS).  The member is cut into 256-byte chunks aligned to its END (the
// front of the first chunk is virtual zeros, which leave a raw CRC -- no
// pre/post conditioning -- unchanged), and lane l owns bytes [4l, 4l + 4) of
// every chunk, so each chunk is one coalesced load per wave.  Lane l's share
// of the message (its dwords, zeros elsewhere) runs through the recurrence
// t <- A(t ^ d) with A = advance over 256 bytes (a linear map: four table
// lookups, no serial byte chain), which keeps every lane's state aligned to
// the start of its dword; the last dword is not advanced, and the 64 lane
// states are combined as consecutive dwords in a 6-level tree:
// raw(X || Y) = raw(X) * x^(8|Y|) ^ raw(Y)   (zlib crc32_combine).
constexpr uint32_t kCrcMembersPerBlock = 4;

__global__ __launch_bounds__(256) void gz_crc_kernel(const uint8_t* __restrict__ out,
                                                     const GzMember* __restrict__ members, uint32_t n,
                                                     const GzCrcConsts* __restrict__ consts,
                                                     uint32_t* __restrict__ status, uint32_t* __restrict__ any_error) {
    __shared__ uint32_t A[4][256];
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) (&A[0][0])[i] = (&consts->adv[0][0])[i];
    __syncthreads();
    const uint32_t m = blockIdx.x * kCrcMembersPerBlock + (threadIdx.x >> 6);
    if (m >= n || status[m] != GZ_OK) return;  // no barrier below; failed members stay failed
    const uint32_t lane = threadIdx.x & 63;
    const GzMember mem = members[m];
    if (mem.isize == 0) {
        if (lane == 0 && mem.crc != 0) {
            status[m] = GZ_E_CRC;
            atomicOr(any_error, 1u);
        }
        return;
    }
    const uint32_t chunks = (mem.isize + 255) >> 8;
    const uint64_t end = mem.ooff + mem.isize;
    // dword q of chunk k starts at byte end - 256 (chunks - k) + 4 lane
    const int64_t q0 = (int64_t)end - 256 * (int64_t)chunks + 4 * (int64_t)lane;
    const uint32_t sh = (uint32_t)(end & 3);  // every q has the same misalignment
    auto dword = [&](uint32_t k) -> uint32_t {
        const int64_t q = q0 + 256 * (int64_t)k;
        if (q + 4 <= (int64_t)mem.ooff) return 0u;  // wholly in the virtual front
        const uint64_t w = (uint64_t)max(q, (int64_t)mem.ooff) & ~(uint64_t)3;  // never before the member's word
        const uint64_t wq = (uint64_t)(q & ~(int64_t)3);
        uint32_t lo = *(const uint32_t*)(out + w);
        if (w != wq) lo = 0u;  // bytes before the member: masked below anyway
        uint32_t d = lo;
        if (sh) {
            const uint32_t hi = *(const uint32_t*)(out + wq + 4);  // same aligned word as a valid byte
            d = __builtin_amdgcn_alignbyte(hi, lo, sh);
        }
        if (q < (int64_t)mem.ooff) d &= 0xFFFFFFFFu << (8u * (uint32_t)(mem.ooff - q));
        return d;
    };
    uint32_t t = 0;
    uint32_t k = 0;
    // four chunks in flight per step
    for (; k + 4 < chunks; k += 4) {
        const uint32_t d0 = dword(k), d1 = dword(k + 1), d2 = dword(k + 2), d3 = dword(k + 3);
#define ADV(d)                                                                                       \
        {                                                                                            \
            const uint32_t x = t ^ (d);                                                              \
            t = A[0][x & 0xFF] ^ A[1][(x >> 8) & 0xFF] ^ A[2][(x >> 16) & 0xFF] ^ A[3][x >> 24];    \
        }
        ADV(d0) ADV(d1) ADV(d2) ADV(d3)
    }
    for (; k + 1 < chunks; ++k) ADV(dword(k))
#undef ADV
    uint32_t c = t ^ dword(chunks - 1);
    // tree over consecutive dwords: node of 2^k lanes = 4 * 2^k bytes
#pragma unroll
    for (uint32_t lv = 0; lv < 6; ++lv) {
        const uint32_t step = 1u << lv;
        const uint32_t right = __shfl_down(c, step);
        if ((lane & (2 * step - 1)) == 0) c = multmodp(consts->x2n[5 + lv], c) ^ right;
    }
    if (lane == 0) {
        c = multmodp(consts->x2n[5], c);  // lane 0's state is aligned to its dword's start: 4 more bytes
        // standard CRC: pre-condition 0xFFFFFFFF shifted over the data, post-xor
        const uint32_t crc = c ^ multmodp(x2nmodp(*consts, mem.isize, 3), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
        if (crc != mem.crc) {
            status[m] = GZ_E_CRC;
            atomicOr(any_error, 1u);
        }
    }
}

}  // namespace

hipError_t launch_gz_inflate(const uint8_t* cdata, size_t cbytes, const GzMember* members, uint32_t n, uint8_t* out,
                             uint32_t* status, uint32_t* any_error, hipStream_t stream, uint32_t* prof) {
    if (n == 0) return hipSuccess;
    if (cbytes == 0 || ((uintptr_t)cdata & 3) || (cbytes + 3) / 4 > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const uint32_t last = (uint32_t)((cbytes + 3) / 4 - 1);
    // One wave per member; the 2 KiB output ring in LDS (kDefaultRingKb:
    // 1 KiB measured the same, 4 / 8 KiB slower -- DESIGN.md 4.7).
    hipLaunchKernelGGL(gz_inflate_kernel<kDefaultRingKb * 1024>, dim3(n), dim3(64), 0, stream, cdata, last, members, n,
                       out, status, any_error, prof);
    return hipGetLastError();
}

hipError_t gz_preload() {
    int nb = 0;  // an occupancy query loads the kernel's code object (msw_ctx_prepare does the same)
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, gz_crc_kernel, 256, 0);
}

hipError_t launch_gz_crc(const uint8_t* out, const GzMember* members, uint32_t n, const GzCrcConsts* consts,
                         uint32_t* status, uint32_t* any_error, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gz_crc_kernel, dim3((n + kCrcMembersPerBlock - 1) / kCrcMembersPerBlock), dim3(256), 0, stream, out, members, n, consts, status, any_error);
    return hipGetLastError();
}

}  // namespace msw
