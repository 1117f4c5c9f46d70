// msw_kernels.h -- device-side parameter block and launchers (internal).
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msw {

// Substitution codes: a real byte b becomes b << code_shift (< 0x4000), so two
// different bytes XOR to >= 2^code_shift >= delta and min(x, delta) is exactly
// the mismatch penalty.  Sentinels XOR to >= 0x4000 with every real code and
// with each other, i.e. they always mismatch (padding never scores).
constexpr uint32_t kReadSentinel = 0x8000u;
constexpr uint32_t kWinSentinel = 0x4000u;
constexpr uint32_t kWinSentinel2 = 0x40004000u;

constexpr int kGroupLanes = 16;        // one DPP row
constexpr int kPairsPerWave = 8;       // 4 groups x 2 packed pairs
constexpr int kMaxRowsPerLane = 24;    // pairs layout, any G (17..24 in narrow groups: large batches only)
constexpr int kMaxMultiKR = 16;        // sw_multi_kernel's rows-per-lane range
constexpr int kMaxReadLen = 384;       // 16 x 24
constexpr int kMaxWinLen = 4096;
constexpr int kLead = 32;
// Pairs with a read > kMaxReadLen or a window > kMaxWinLen go to the long-pair
// kernel (msw_long.hip): i32 cells, any length up to kMaxLongLen (the i16
// best-cell coordinates of msw_out_t).
constexpr int kMaxLongLen = 32767;
constexpr int kLongMaxR = 8;           // rows per lane; strips of 64 * R rows              // sentinel words in front of each window stream

// u32 words per lane-group stream: kLead + (max_win + 31) steps rounded to even
// + 4 lookahead,
// rounded so that the four groups of a wave start 16 banks apart (== 16 mod 32).
inline uint32_t stream_stride(uint32_t max_win_len) {
    uint32_t words = kLead + max_win_len + 2 * kGroupLanes + 5;
    words = (words + 31u) & ~31u;
    return words + 16u;
}

struct SwParams {
    const uint8_t* reads;
    const uint8_t* wins;
    const uint16_t* read_len;
    const uint16_t* win_len;
    const uint32_t* order;    // kernel slot -> pair index; nullptr = identity
    int32_t* score;
    int16_t* end_i;           // nullptr unless coordinates are wanted
    int16_t* end_j;
    uint64_t read_stride;
    uint64_t win_stride;
    uint32_t n_slots;
    uint32_t lds_stride;      // u32 words per lane-group window stream
    uint32_t code_shift;
    uint32_t win_vec;         // 1: win_stride % 16 == 0 and wins 16-byte aligned
    uint32_t pairs_blocks;    // mixed grid: leading blocks that use the pairs layout
    uint32_t slot_base;       // first slot index of this (sub)grid when order == nullptr
    uint32_t match2;          // match, duplicated into both u16 halves
    uint32_t delta2;          // match - mismatch
    uint32_t gap2;            // linear: gap penalty; affine: gap_extend
    uint32_t open_ext2;       // affine: gap_open + gap_extend + K
    uint32_t bias2;           // affine: K = 256 + gap_extend (see msw_kernels.hip)
    uint64_t* trace;          // diagnostics (MSW_WAVE_TRACE): 4 words per block, or nullptr
    uint32_t group_lanes;     // G: lanes per lane group (8..16)
    uint32_t groups;          // lane groups per wave = 64 / G (lanes past groups * G idle)
    // f16 fast path (ACGT windows): cell values H * 2^-11 as packed f16.
    uint32_t f16_ok;          // 1: the scheme and this launch's bound fit (msw_runtime.cpp)
    uint32_t f16_hi;          // high byte of f16(+match) | high byte of f16(mismatch) << 8
    uint32_t f16_ngap2;       // f16(-gap) (linear) / f16(-gap_extend) (affine), both halves
    uint32_t f16_noe2;        // affine: f16(-(gap_open + gap_extend)), both halves
    // Results by slot (needs order): score[out_slot_base + slot] instead of
    // score[pair], so each wave's stores are contiguous; the caller restores
    // pair order (msw_runtime.cpp: the host drain, or launch_gather_results).
    uint32_t out_by_slot;
    uint32_t out_slot_base;
    // Optional lengths in slot order, read_len | win_len << 16 per slot (index
    // out_slot_base + slot): planned batches read them contiguously instead of
    // gathering two 2-byte lengths per pair through the order array.
    const uint32_t* slot_lens;
    // Long pairs (sw_long_kernel, msw_long.hip): per-block boundary rows,
    // long_cols i32 columns each (x2 for affine: H then F).
    int32_t* long_scratch;
    uint32_t long_cols;
    // sw_long_kernel work queue (zeroed u32, or null): with fewer blocks than
    // slots, a block that finishes a slot takes the next unclaimed one
    // (gridDim.x + counter) instead of striding by gridDim.x
    uint32_t* long_next;
    // Genome-resident windows (instances with GEN = true: pairs layout, KR <=
    // 16): the window of pair p is win_src[win_pos[p] ..], win_len[p] bytes
    // (clipped by the host), read straight from the resident genome at any
    // alignment instead of from a cut slab (wins / win_stride unused); the
    // genome allocation extends >= 20 bytes past every window (kGenomePad).
    const uint8_t* win_src;
    const int64_t* win_pos;
};

// f16 bits of the cell value v * 2^-11 (|v| < 2048: exact, normal or zero).
inline uint32_t f16_cell_bits(int32_t v) {
    if (v == 0) return 0u;
    const uint32_t sign = v < 0 ? 0x8000u : 0u;
    uint32_t a = (uint32_t)(v < 0 ? -v : v);
    int e = 31 - __builtin_clz(a);  // a = 1.f * 2^e
    const uint32_t mant = (a << (10 - e)) & 0x3FFu;
    return sign | ((uint32_t)(e + 4) << 10) | mant;  // exponent bias 15, scale 2^-11
}

// Packed rows per lane for a read-length bound: ceil(m / 16) in the pairs
// layout, ceil(m / 32) in the split layout (each packed row holds two rows).
inline int rows_per_lane(uint32_t max_read_len, bool split, uint32_t group_lanes = kGroupLanes) {
    const uint32_t per = split ? 2 * group_lanes : group_lanes;
    int kr = (int)((max_read_len + per - 1) / per);
    return kr < 1 ? 1 : kr;
}

// Pairs one wave scores: two per group (pairs layout) or one (split).
__host__ __device__ inline uint32_t pairs_per_wave(bool split, uint32_t groups) { return split ? groups : 2 * groups; }

// 16-byte vector loads of the window rows are legal.
inline uint32_t vec_ok(const void* base, uint64_t stride) {
    return (stride >= 16 && stride % 16 == 0 && ((uintptr_t)base & 15) == 0) ? 1u : 0u;
}

// Dynamic LDS bytes for one 64-lane block (one window stream per group).
inline size_t lds_bytes(uint32_t lds_stride, uint32_t groups) { return (size_t)groups * lds_stride * sizeof(uint32_t); }

enum class Layout { kPairs, kSplit, kMixed };

// Length-bucketed grid (sw_multi_kernel): bucket b holds the slots
// [slot_begin[b], slot_begin[b] + count[b]) of the order array, all with
// rows_per_lane(read length) <= kr[b], and owns blocks
// [b ? block_end[b - 1] : 0, block_end[b]) of ONE launch (pairs layout, G = 16,
// 8 pairs per block).  Buckets are listed heaviest first, so the long waves
// are dispatched first and the short ones fill the tail.
constexpr int kMaxBuckets = 16;
struct MultiTable {
    uint32_t n_buckets;
    uint32_t block_end[kMaxBuckets];
    uint32_t slot_begin[kMaxBuckets];
    uint32_t count[kMaxBuckets];
    uint32_t kr[kMaxBuckets];
    uint32_t lds_stride[kMaxBuckets];
    uint32_t f16_ok[kMaxBuckets];
};

hipError_t launch_sw(const SwParams& p, bool affine, bool coords, uint32_t max_read_len, Layout layout,
                     hipStream_t stream);

// Blocks (waves) per CU of the instance launch_sw / launch_sw_multi would run
// for these arguments (its VGPRs and p's LDS), without launching; the query
// loads the instance's code object (HIP loads a module on its first use).
// 0 on error.  cut_blocks_per_cu: the same for the window cut kernel.
int sw_blocks_per_cu(const SwParams& p, bool affine, bool coords, uint32_t max_read_len, Layout layout);
int sw_multi_blocks_per_cu(const SwParams& p, const MultiTable& t, bool affine, bool coords);
int cut_blocks_per_cu();

// All buckets of `t` in one launch; p.order is required (slot -> pair), the
// per-bucket fields of p (n_slots, lds_stride, f16_ok) come from the table.
hipError_t launch_sw_multi(const SwParams& p, const MultiTable& t, bool affine, bool coords,
                           hipStream_t stream);

// Genome-resident windows: out[p * ws ..] = genome[pos[p], pos[p] + len),
// len = want[p] clipped to the genome (0 outside it), zero-padded to ws;
// out_len[p] = len when out_len != nullptr.  ws % 16 == 0, genome allocation
// padded by >= 20 bytes past its end.
constexpr uint32_t kGenomePad = 64;
hipError_t launch_cut_windows(const uint8_t* genome, uint64_t glen, const int64_t* pos, const uint16_t* want,
                              uint8_t* out, uint16_t* out_len, uint32_t ws, uint64_t n, hipStream_t stream);
// Same, for device-resident reads: want = window, or 2 x rlen[p] capped at
// kMaxWinLen when window is 0 (msw_align_reads_device).
hipError_t launch_cut_windows_for_reads(const uint8_t* genome, uint64_t glen, const int64_t* pos,
                                        const uint16_t* rlen, uint32_t window, uint8_t* out, uint16_t* out_len,
                                        uint32_t ws, uint64_t n, hipStream_t stream);

// dst[i] = src[inv[i]] for score (and end_i / end_j when non-null): pair
// order restored from slot-ordered results (one thread per pair, coalesced
// stores; the slot-ordered source is small enough to stay in L2).
// bytes from device memory to pinned host memory (dst: its device address),
// as a kernel on `stream` (msw_memcpy_d2h_async)
hipError_t launch_d2h_copy(void* dst, const void* src, uint64_t bytes, hipStream_t stream);
// Up to kPullRanges ranges copied by ONE kernel on `stream`: a one-chunk
// host call pulls its pinned rows and metadata into the slot's device
// buffers on its compute stream (no DMA engine, no cross-queue event between
// the upload and the scoring launch).  Sources are device addresses of
// pinned host memory; each range's source and destination share their
// alignment mod 16 (16-byte loads between a byte head and tail).
constexpr int kPullRanges = 3;
struct PullRanges {
    uint8_t* dst[kPullRanges];
    const uint8_t* src[kPullRanges];
    uint64_t bytes[kPullRanges];  // 0: unused
};
hipError_t launch_pull_copy(const PullRanges& r, hipStream_t stream);
hipError_t launch_gather_results(const uint32_t* inv, const int32_t* src_score, const int16_t* src_i,
                                 const int16_t* src_j, int32_t* score, int16_t* end_i, int16_t* end_j, uint64_t n,
                                 hipStream_t stream);

// Long pairs: R = rows per lane for a read-length bound (the fewest strips of
// <= 512 rows, rows spread evenly over them); scratch columns per block; LDS bytes.
int long_rows_per_lane(uint32_t max_read_len);
uint32_t long_scratch_cols(uint32_t max_win_len);
// Blocks (waves) of the long-pair launch one CU holds at once (registers and
// LDS of the kernel instance these bounds select).
int long_blocks_per_cu(bool affine, bool coords, uint32_t max_read_len, uint32_t max_win_len);
size_t long_lds_bytes(uint32_t max_win_len);
// One wave per pair, `blocks` blocks striding over p.n_slots (order / slot
// results as in launch_sw).  p.long_scratch must hold blocks x long_cols
// (x2 affine) i32 when the read bound exceeds 64 * R rows.
hipError_t launch_sw_long(const SwParams& p, bool affine, bool coords, uint32_t max_read_len, uint32_t max_win_len,
                          uint32_t blocks, hipStream_t stream);

// smith_waterman_align restated: result must be zeroed before the launch.
hipError_t launch_compat(const uint8_t* s1, const uint8_t* s2, int32_t* result, uint64_t L,
                         uint32_t W, uint64_t G, hipStream_t stream);

}  // namespace msw
