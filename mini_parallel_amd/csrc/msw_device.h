// msw_device.h -- device code of the Smith-Waterman kernels (internal):
// the DP body sw_body<KR, AFFINE, COORDS, SPLIT> and the kernel templates
// sw_kernel / sw_mixed_kernel / sw_multi_kernel.  Included by the launcher
// translation units (msw_launch_*.hip), which instantiate disjoint subsets so
// the instance set compiles in parallel; msw_kernels.hip holds the dispatch.
#pragma once
// Design notes (hand-written gfx950 kernels for batched Smith-Waterman).
//
// Replaces the reference's OpenCL kernels (smith_waterman/src/smith_waterman.cl):
//   * sw_linear_kernel<KR,COORDS> : linear-gap score (+ best cell), the
//                                   recurrence smith_waterman_detailed
//                                   (:74-152) intended, with a global max.
//   * sw_affine_kernel<KR,COORDS> : Gotoh affine-gap score (+ best cell).
//   * sw_compat_kernel            : smith_waterman_align (:11-71), the kernel
//                                   gpu_align (aligner.rs:410-532) launches.
//
// Design (DESIGN.md has the derivation and the roofline):
//  - Integer max-plus DP, VALU-bound: no MFMA, no LDS tiling of the matrix.
//  - One wave64 = 64 / G lane groups of G lanes (G = 8..16, chosen per launch
//    so the batch fills the SIMDs evenly).  A group scores TWO pairs at once:
//    pair "a" in the low 16 bits and pair "b" in the high 16 bits of every
//    register, so each packed-u16 VALU op updates two cells.
//  - Lane l of a group owns read rows [l*KR, l*KR+KR) in VGPRs and sweeps the
//    window with a one-column skew per lane (anti-diagonal wavefront): at step
//    t lane l scores column t-l, reading that column's packed window code from
//    an LDS stream.  Lane l-1's bottom-row H enters through one
//    v_and_b32_dpp wave_shr:1 whose mask zeroes each group's first lane: the
//    zero top boundary.
//  - Cell values are small non-negative integers kept as u16; the three-way max
//    runs as v_pk_maximum3_f16 on their (denormal, ordered) f16 bit patterns,
//    and the zero floor comes from u16 saturating subtracts.
//  - Padding (rows past a read, columns past a window, the wavefront's
//    fill/drain columns) uses sentinel codes that mismatch everything, so no
//    per-cell masking is needed: such cells never reach the pair's score.
#include "msw_kernels.h"

#include <type_traits>

namespace msw {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_satsub(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(
        __builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}
__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(
        __builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(
        __builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}
// Three-way max of packed u16 values < 0x7C00: as f16 bit patterns they are
// non-negative and finite and order like the integers -> one v_pk_maximum3_f16.
__device__ __forceinline__ uint32_t pk_max3(uint32_t a, uint32_t b, uint32_t c) {
    f16x2 x = __builtin_bit_cast(f16x2, a), y = __builtin_bit_cast(f16x2, b),
          z = __builtin_bit_cast(f16x2, c);
    return __builtin_bit_cast(uint32_t,
                              __builtin_elementwise_maximum(x, __builtin_elementwise_maximum(y, z)));
}
// Packed f16 arithmetic of the fast path (cell values are H * 2^-11, exact).
__device__ __forceinline__ uint32_t hadd(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2, a) + __builtin_bit_cast(f16x2, b));
}
// a + b clamped to [0, 1]: one v_pk_add_f16 ... clamp (hipcc folds the min/max).
__device__ __forceinline__ uint32_t hadd_clamp(uint32_t a, uint32_t b) {
    const f16x2 z = {(_Float16)0.0f, (_Float16)0.0f}, one = {(_Float16)1.0f, (_Float16)1.0f};
    const f16x2 v = __builtin_bit_cast(f16x2, a) + __builtin_bit_cast(f16x2, b);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_elementwise_max(v, z), one));
}
__device__ __forceinline__ uint32_t hmax(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_maximum(__builtin_bit_cast(f16x2, a),
                                                                      __builtin_bit_cast(f16x2, b)));
}
// f16 cell value (H * 2^-11, H < 2048) -> integer score H.
__device__ __forceinline__ uint32_t f16_to_score(uint32_t bits) {
    return (uint32_t)((float)__builtin_bit_cast(_Float16, (unsigned short)bits) * 2048.0f);
}

// Score tracking max (opaque so the compiler keeps one op per two rows
// instead of re-associating into a tree).
__device__ __forceinline__ uint32_t track_max3(uint32_t best, uint32_t a, uint32_t b) {
    uint32_t d;
    asm("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(d) : "v"(best), "v"(a), "v"(b));
    return d;
}

// Hand-off from lane l-1: DPP wave_shr:1 over the whole wave (lane 0 reads 0
// through bound_ctrl), then top_mask zeroes the first lane of every group --
// the matrix's zero top boundary for H and F.  hipcc folds the pair into one
// v_and_b32_dpp.
__device__ __forceinline__ uint32_t shr1_group(uint32_t src, uint32_t top_mask) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)src, 0x138, 0xF, 0xF, true) & top_mask;
}

// Packed (H + match): a full-rate v_add_u32 suffices -- each u16 half stays
// below 0x7C00 + 64, so no carry crosses into the high half.
__device__ __forceinline__ uint32_t add_nc(uint32_t a, uint32_t b) { return a + b; }

// Split layout: {lo = dpp.hi, hi = own.lo} in one v_alignbit_b32.
__device__ __forceinline__ uint32_t hi_to_lo_own_lo_to_hi(uint32_t own, uint32_t dpp) {
    return __builtin_amdgcn_alignbit(own, dpp, 16);
}

// Lane-group layouts (template flag SPLIT), G lanes per group:
//  pairs (SPLIT = false): a group scores two pairs, pair a in the low and pair
//      b in the high u16 half; lane l owns rows [l*KR, l*KR+KR) of both and
//      scores column t - l at step t.  2 * (64 / G) pairs per wave.
//  split (SPLIT = true): a group scores one pair; lane l owns rows
//      [2l*KR, 2l*KR+KR) in the low half and the next KR rows in the high
//      half, which runs one column behind: low half column t - 2l, high half
//      t - 2l - 1.  64 / G pairs per wave: half the work per wave, for batches
//      too small to give every SIMD two pairs-waves.
struct PairMeta {
    uint32_t pa, pb;  // pair indices (the same pair twice in the split layout)
    uint32_t oa, ob;  // output indices: the pair's, or its slot's (p.out_by_slot)
    bool va, vb;
    int ma, mb, na, nb;
    int64_t sa, sb;   // genome windows (GEN): first window byte in the genome (0 if empty)
};

// Traffic probes (tools/traffic_split.sh, built by tools/build_variant.sh with
// -DMSW_PROBE_NO_WIN=1 or -DMSW_PROBE_NO_READ=1): the window / read loads are
// replaced by constants so rocprofv3 FETCH_SIZE of the variant splits a
// launch's HBM reads by buffer.  Scores are wrong in a probe build.
#ifndef MSW_PROBE_NO_WIN
#define MSW_PROBE_NO_WIN 0
#endif
#ifndef MSW_PROBE_NO_READ
#define MSW_PROBE_NO_READ 0
#endif
// -DMSW_PROBE_CONST_LEN=1: the pair lengths are the config-2 constants (150 /
// 300) instead of loads, so with the two probes above FETCH_SIZE is what the
// launch fetches besides the sequence bytes and the lengths (code, arguments).
#ifndef MSW_PROBE_CONST_LEN
#define MSW_PROBE_CONST_LEN 0
#endif

template <bool SPLIT, bool GEN>
__device__ __forceinline__ PairMeta load_meta(const SwParams& p, int g, uint32_t block, bool active) {
    // Branch-free: clamped indices keep every load legal (n_slots >= 1), the
    // lengths of padding slots (and of idle lanes) are masked to 0 afterwards.
    PairMeta q;
    const uint32_t slot_a = block * pairs_per_wave(SPLIT, p.groups) + (SPLIT ? g : 2u * g);
    const uint32_t slot_b = SPLIT ? slot_a : slot_a + 1;
    const uint32_t last = p.n_slots - 1;
    const uint32_t sa = min(slot_a, last), sb = min(slot_b, last);
    q.va = active && slot_a < p.n_slots;
    q.vb = active && slot_b < p.n_slots;
    q.pa = p.order ? p.order[sa] : p.slot_base + sa;
    q.pb = SPLIT ? q.pa : (p.order ? p.order[sb] : p.slot_base + sb);
    // Slot-ordered results (length-bucketed batches): a wave's pairs are
    // scattered over the batch, its slots are consecutive -- the stores stay
    // contiguous and the host / a gather pass restores pair order.
    q.oa = p.out_by_slot ? p.out_slot_base + sa : q.pa;
    q.ob = p.out_by_slot ? p.out_slot_base + sb : q.pb;
    int ma, na, mb, nb;
    if (p.slot_lens) {  // lengths in slot order (planned batches): contiguous, not gathered
        const uint32_t la = p.slot_lens[p.out_slot_base + sa];
        const uint32_t lb = SPLIT ? la : p.slot_lens[p.out_slot_base + sb];
        ma = (int)(la & 0xFFFFu);
        na = (int)(la >> 16);
        mb = (int)(lb & 0xFFFFu);
        nb = (int)(lb >> 16);
    } else if (MSW_PROBE_CONST_LEN) {
        ma = mb = 150;
        na = nb = 300;
    } else {
        ma = p.read_len[q.pa];
        na = p.win_len[q.pa];
        mb = SPLIT ? ma : (int)p.read_len[q.pb];
        nb = SPLIT ? na : (int)p.win_len[q.pb];
    }
    q.ma = q.va ? ma : 0;
    q.mb = q.vb ? mb : 0;
    q.na = q.va ? na : 0;
    q.nb = q.vb ? nb : 0;
    if constexpr (GEN) {  // loaded beside the lengths (same round trip); an empty window reads the genome's start
        const int64_t sa = p.win_pos[q.pa];
        const int64_t sb = SPLIT ? sa : p.win_pos[q.pb];
        q.sa = q.na > 0 ? sa : 0;
        q.sb = q.nb > 0 ? sb : 0;
    }
    return q;
}

// Window rows: a slab row (16-byte aligned, win_stride apart) or, for GEN
// instances, a genome position (any alignment).
template <bool GEN>
__device__ __forceinline__ const uint8_t* win_row(const SwParams& p, uint32_t pair, int64_t pos) {
    if constexpr (GEN) return p.win_src + pos;
    else return p.wins + (uint64_t)pair * p.win_stride;
}

// 16 window bytes at row + 16 k: one 16-byte load from a slab row; from the
// genome, the five dwords around the chunk (dword loads need only 4-byte
// alignment) and one v_alignbyte per output dword.
template <bool GEN>
__device__ __forceinline__ uint4 win_chunk(const uint8_t* row, int k) {
    const uint8_t* a = row + 16 * k;
    if constexpr (!GEN) {
        return *reinterpret_cast<const uint4*>(a);
    } else {
        // the dword base by pointer arithmetic (not an integer mask), so the
        // compiler keeps the global address space: global, not flat, loads
        const uint32_t b = (uint32_t)(reinterpret_cast<uintptr_t>(a) & 3u);
        const uint32_t* al = reinterpret_cast<const uint32_t*>(a - b);
        const uint32_t x0 = al[0], x1 = al[1], x2 = al[2], x3 = al[3], x4 = al[4];
        return make_uint4(__builtin_amdgcn_alignbyte(x1, x0, b), __builtin_amdgcn_alignbyte(x2, x1, b),
                          __builtin_amdgcn_alignbyte(x3, x2, b), __builtin_amdgcn_alignbyte(x4, x3, b));
    }
}

// Last byte index a byte load of a window may use: the slab row's, or the
// genome window's own (never past the genome).
template <bool GEN>
__device__ __forceinline__ int win_last(const SwParams& p, int n) {
    if constexpr (GEN) return max(n, 1) - 1;
    else return (int)p.win_stride - 1;
}

__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
    return v;
}

// Wave-wide max of non-negative values, uniform result: DPP row_shr 1/2/4/8
// (row maxima in lane 15 of each row), row_bcast 15/31, readlane 63 -- six
// VALU ops instead of six dependent ds_bpermute round trips (__shfl_xor).
__device__ __forceinline__ int wave_max_nonneg(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true));   // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true));   // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true));   // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true));   // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ uint32_t wcode(uint32_t byte, bool valid, uint32_t shift) {
    return valid ? (byte << shift) : kWinSentinel;
}

// Packed window stream of this lane group in LDS, kLead sentinel words first:
//   pairs: stream[kLead + c] = code(win_a[c]) | code(win_b[c])   << 16
//   split: stream[kLead + c] = code(win[c])   | code(win[c - 1]) << 16
// Sentinels past each window.  Vector path: 16-byte loads, a round of up to
// two chunks of 16 columns per lane in flight together.  Scalar path
// (unaligned batches): byte loads with clamped addresses, no branches.
template <bool SPLIT, bool GEN>
__device__ __forceinline__ void stage_window(const SwParams& p, const PairMeta& q, uint32_t* stream,
                                             int steps, int lg, int G, bool active) {
    if (!active) return;
    const uint8_t* wa = win_row<GEN>(p, q.pa, q.sa);
    const uint8_t* wb = win_row<GEN>(p, q.pb, q.sb);
    const uint32_t sh = p.code_shift;
    const int last = win_last<GEN>(p, q.na), last_b = win_last<GEN>(p, q.nb);
    for (int k = lg; k < kLead; k += G) stream[k] = kWinSentinel2;
    const int nch = (steps + 15) >> 4;  // chunks of 16 columns to stage
    if (p.win_vec) {
        const int loadable = (int)(p.win_stride >> 4);
        // genome windows: chunk indices clamped to each window's last chunk
        // (columns past the window are masked), every load unconditional
        const int top_a = GEN ? max((q.na + 15) / 16 - 1, 0) : 0, top_b = GEN ? max((q.nb + 15) / 16 - 1, 0) : 0;
        for (int k0 = 0; k0 < nch; k0 += 2 * G) {
            uint4 va[2], vb[2];
            uint32_t prev[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int k = k0 + u * G + lg;
                if constexpr (GEN) {
                    va[u] = win_chunk<true>(wa, min(k, top_a));
                    if constexpr (SPLIT) prev[u] = wa[min(max(16 * k - 1, 0), last)];
                    else vb[u] = win_chunk<true>(wb, min(k, top_b));
                } else {
                    const bool ld = k < nch && k < loadable && !MSW_PROBE_NO_WIN;
                    va[u] = ld ? *reinterpret_cast<const uint4*>(wa + 16 * k) : make_uint4(0, 0, 0, 0);
                    if constexpr (SPLIT) {
                        prev[u] = wa[min(max(16 * k - 1, 0), last)];
                    } else {
                        vb[u] = ld ? *reinterpret_cast<const uint4*>(wb + 16 * k) : make_uint4(0, 0, 0, 0);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int k = k0 + u * G + lg;
                if (k < nch) {
                    const uint32_t xa[4] = {va[u].x, va[u].y, va[u].z, va[u].w};
                    uint32_t xb[4] = {0u, 0u, 0u, 0u};
                    if constexpr (!SPLIT) { xb[0] = vb[u].x; xb[1] = vb[u].y; xb[2] = vb[u].z; xb[3] = vb[u].w; }
                    uint4* dst = reinterpret_cast<uint4*>(stream + kLead + 16 * k);
                    uint32_t carry = 0u;
                    if constexpr (SPLIT) carry = prev[u] & 0xFFu;  // byte of column 16k - 1
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        uint32_t w4[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int c = 16 * k + 4 * d + e;
                            const uint32_t ba = (xa[d] >> (8 * e)) & 0xFFu;
                            if constexpr (SPLIT) {
                                w4[e] = wcode(ba, c < q.na, sh) | (wcode(carry, c >= 1 && c - 1 < q.na, sh) << 16);
                                carry = ba;
                            } else {
                                const uint32_t bb = (xb[d] >> (8 * e)) & 0xFFu;
                                w4[e] = wcode(ba, c < q.na, sh) | (wcode(bb, c < q.nb, sh) << 16);
                            }
                        }
                        dst[d] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
                    }
                }
            }
        }
    } else {
        for (int c0 = 0; c0 < steps; c0 += 4 * G) {
            uint32_t ba[4], bb[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int c = c0 + u * G + lg;
                ba[u] = wa[min(c, last)];
                bb[u] = SPLIT ? wa[min(max(c - 1, 0), last)] : wb[min(c, GEN ? last_b : last)];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int c = c0 + u * G + lg;
                const bool vb = SPLIT ? (c >= 1 && c - 1 < q.na) : (c < q.nb);
                if (c < steps) stream[kLead + c] = wcode(ba[u], c < q.na, sh) | (wcode(bb[u], vb, sh) << 16);
            }
        }
    }
}

// Read bytes of this lane's packed rows: unconditional loads with clamped
// addresses (all in flight at once, issued before the pair lengths arrive).
template <int KR, bool SPLIT>
__device__ __forceinline__ void load_read_bytes(const SwParams& p, uint32_t pa, uint32_t pb, int lg,
                                                uint32_t (&ba)[KR], uint32_t (&bb)[KR]) {
    const uint8_t* ra = p.reads + (uint64_t)pa * p.read_stride;
    const uint8_t* rb = p.reads + (uint64_t)pb * p.read_stride;
    const int last = (int)p.read_stride - 1;
#pragma unroll
    for (int r = 0; r < KR; ++r) {
        const int ia = SPLIT ? lg * 2 * KR + r : lg * KR + r;
        const int ib = SPLIT ? ia + KR : ia;
#if MSW_PROBE_NO_READ
        ba[r] = (uint32_t)(ia + pa) & 3u;
        bb[r] = (uint32_t)(ib + pb) & 3u;
        (void)ra; (void)rb; (void)last;
#else
        ba[r] = ra[min(ia, last)];
        bb[r] = rb[min(ib, last)];
#endif
    }
}

// Read codes (byte << code_shift, or the sentinel past the read) of this
// lane's packed rows, pair a in the low and pair b in the high half.
template <int KR, bool SPLIT>
__device__ __forceinline__ void read_codes(const SwParams& p, const PairMeta& q, int lg, const uint32_t (&ba)[KR],
                                           const uint32_t (&bb)[KR], uint32_t (&rc)[KR]) {
#pragma unroll
    for (int r = 0; r < KR; ++r) {
        const int ia = SPLIT ? lg * 2 * KR + r : lg * KR + r;
        const int ib = SPLIT ? ia + KR : ia;
        const uint32_t ca = ia < q.ma ? (ba[r] << p.code_shift) : kReadSentinel;
        const uint32_t cb = ib < q.mb ? (bb[r] << p.code_shift) : kReadSentinel;
        rc[r] = ca | (cb << 16);
    }
}

// Reductions over a group's G lanes into its first lane: a tree clipped at the
// group's end (lane lg gathers [lg, min(lg + 2^k, G)) after step k).
__device__ __forceinline__ uint32_t group_pk_max(uint32_t v, int lg, int G) {
    const int lane = threadIdx.x;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
        const uint32_t o = (uint32_t)__shfl((int)v, lane + off, 64);
        v = lg + off < G ? pk_max(v, o) : v;
    }
    return v;
}

// Best-cell key: score in the high word, (0xFFFF - i, 0xFFFF - j) in the low
// word, so the max key is max score, then smallest i, then smallest j -- the
// oracle's row-major scan with strict '>'.
__device__ __forceinline__ uint64_t group_max_u64(uint64_t v, int lg, int G) {
    const int lane = threadIdx.x;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
        const uint64_t o = __shfl(v, lane + off, 64);
        v = (lg + off < G && o > v) ? o : v;
    }
    return v;
}

__device__ __forceinline__ void store_score(const SwParams& p, bool valid, uint32_t pair, uint32_t s) {
    if (valid) p.score[pair] = (int32_t)s;
}

__device__ __forceinline__ void store_hit(const SwParams& p, bool valid, uint32_t pair, uint64_t key,
                                          uint32_t bias, bool f16) {
    if (!valid) return;
    const uint32_t s = f16 ? f16_to_score((uint32_t)(key >> 32)) : (uint32_t)(key >> 32) - bias;
    p.score[pair] = (int32_t)s;
    if (p.end_i) {
        const uint32_t lo = (uint32_t)key;
        p.end_i[pair] = s ? (int16_t)(0xFFFFu - (lo >> 16)) : (int16_t)-1;
        p.end_j[pair] = s ? (int16_t)(0xFFFFu - (lo & 0xFFFFu)) : (int16_t)-1;
    }
}

// Per-row keys (h << 16 | 0xFFFF - j, one per u16 half) -> best hits.
template <int KR, bool SPLIT>
__device__ __forceinline__ void finish_coords(const SwParams& p, const PairMeta& q, int lg, int G,
                                              const uint32_t (&key_a)[KR], const uint32_t (&key_b)[KR],
                                              uint32_t bias, bool f16) {
    uint64_t ga = 0, gb = 0;
#pragma unroll
    for (int r = 0; r < KR; ++r) {
        const uint32_t ia = SPLIT ? (uint32_t)(lg * 2 * KR + r) : (uint32_t)(lg * KR + r);
        const uint32_t ib = SPLIT ? ia + KR : ia;
        const uint64_t ka = ((uint64_t)(key_a[r] >> 16) << 32) | ((uint64_t)(0xFFFFu - ia) << 16) |
                            (key_a[r] & 0xFFFFu);
        const uint64_t kb = ((uint64_t)(key_b[r] >> 16) << 32) | ((uint64_t)(0xFFFFu - ib) << 16) |
                            (key_b[r] & 0xFFFFu);
        ga = ka > ga ? ka : ga;
        gb = kb > gb ? kb : gb;
    }
    if constexpr (SPLIT) {
        ga = gb > ga ? gb : ga;
        ga = group_max_u64(ga, lg, G);
        if (lg == 0) store_hit(p, q.va, q.oa, ga, bias, f16);
    } else {
        ga = group_max_u64(ga, lg, G);
        gb = group_max_u64(gb, lg, G);
        if (lg == 0) {
            store_hit(p, q.va, q.oa, ga, bias, f16);
            store_hit(p, q.vb, q.ob, gb, bias, f16);
        }
    }
}

template <bool SPLIT>
__device__ __forceinline__ void finish_score(const SwParams& p, const PairMeta& q, int lg, int G,
                                             uint32_t best, uint32_t bias, bool f16) {
    // Non-negative f16 bit patterns order like the integers: one u16 max serves both.
    best = group_pk_max(best, lg, G);
    if (lg == 0) {
        auto val = [&](uint32_t h) { return f16 ? f16_to_score(h) : h - bias; };
        if constexpr (SPLIT) {
            store_score(p, q.va, q.oa, val(max(best & 0xFFFFu, best >> 16)));
        } else {
            store_score(p, q.va, q.oa, val(best & 0xFFFFu));
            store_score(p, q.vb, q.ob, val(best >> 16));
        }
    }
}

// Bottom-row hand-off from lane l-1 (DPP row_shr:1, lane 0 reads the zero top
// boundary).  Split layout: the low half takes lane l-1's high-half row, the
// high half takes this lane's own low-half row of the previous step.
template <bool SPLIT>
__device__ __forceinline__ uint32_t from_above(uint32_t own_bottom, uint32_t top_mask) {
    const uint32_t d = shr1_group(own_bottom, top_mask);
    if constexpr (SPLIT) return hi_to_lo_own_lo_to_hi(own_bottom, d);
    else return d;
}

// ---------------------------------------------------------------------------
// ACGT fast path.  When every window byte of a wave is one of A, C, G, T (and
// the scoring scheme fits, p.f16_ok), the DP runs on packed f16 values: a cell
// of score H holds H * 2^-11, exact for H < 2048, so
//   * the substitution score s = +match / -mismatch of a packed cell pair is one
//     v_perm_b32 lookup: both values are f16 numbers whose low byte is zero, so
//     only their high bytes live in the tables.  Each packed row keeps two
//     4-byte tables (lo half in bytes 0-3, hi half in bytes 4-7: byte k = hi(+m)
//     if the row's base has class k, else hi(-mm)), and each window column's
//     LDS word becomes a selector {12, class(lo), 12, 4 + class(hi)} (selector
//     12 reads 0x00; padding columns select 0x00 twice, s = +0);
//   * H_diag + s is one v_pk_add_f16 (negative results are harmless: the
//     three-way max always sees an E >= 0), and E = max(H - gap, 0) is one
//     v_pk_add_f16 with the clamp modifier -- two ops fewer per packed row than
//     the integer path (add match, saturating subtract).
// The class of A/C/G/T is ((b >> 1) ^ (b >> 2)) & 3 = 0/1/2/3.  Padding
// columns with s = 0 copy a diagonal value one row down, so a padding cell
// never beats the real cell it copies (equal score, larger i).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t base_class(uint32_t b) { return ((b >> 1) ^ (b >> 2)) & 3u; }

__device__ __forceinline__ bool is_acgt(uint32_t b) {
    const uint32_t o = b - 0x41u;  // A C G T = 0x41 + {0, 2, 6, 19}
    return o < 20u && ((0x80045u >> o) & 1u);
}

// u16 window code half (byte << shift or the sentinel) -> fast path possible
__device__ __forceinline__ bool code_ok(uint32_t v, uint32_t shift) {
    return (v & kWinSentinel) || is_acgt(v >> shift);
}

__device__ __forceinline__ uint32_t win_selector(uint32_t word, uint32_t shift) {
    const uint32_t lo = word & 0xFFFFu, hi = word >> 16;
    const uint32_t sl = (lo & kWinSentinel) ? 12u : base_class(lo >> shift);
    const uint32_t sh = (hi & kWinSentinel) ? 12u : 4u + base_class(hi >> shift);
    return 12u | (sl << 8) | (12u << 16) | (sh << 24);
}

// A read byte outside A/C/G/T (N, lower case, ...) can never equal a window
// byte of a fast-path wave, so its row (like a padding row) is all mismatch.
__device__ __forceinline__ uint32_t row_table(uint32_t v, uint32_t shift, uint32_t mis4, uint32_t match_hi) {
    const uint32_t b = v >> shift;
    if ((v & kReadSentinel) || !is_acgt(b)) return mis4;
    const uint32_t sh = 8u * base_class(b);
    return (mis4 & ~(0xFFu << sh)) | (match_hi << sh);
}

// Checks this lane's share of the group's staged window stream; returns true
// (wave-uniform) if every window byte of the wave is A/C/G/T, and then
// rewrites the stream in place as selectors.  Reads may hold any byte.
__device__ __forceinline__ bool to_fast_path(uint32_t* stream, int words, int lg, int G, bool active,
                                             uint32_t shift, bool allowed) {
    if (!allowed) return false;
    bool ok = true;
    for (int k = lg; active && k < words; k += G) {
        const uint32_t w = stream[k];
        ok = ok && code_ok(w & 0xFFFFu, shift) && code_ok(w >> 16, shift);
    }
    if (__builtin_amdgcn_ballot_w64(!ok) != 0) return false;
    for (int k = lg; active && k < words; k += G) stream[k] = win_selector(stream[k], shift);
    __syncthreads();
    return true;
}

// Fast-path staging straight from the window bytes (16-byte aligned batches):
// each dword of four columns is classified in SWAR form, checked against
// A/C/G/T (canonical bytes rebuilt by one v_perm from the classes) and turned
// into four selector words, written to LDS as 16-byte stores.  Columns past a
// window get selector 12 (s = 0).  Returns false if this lane saw any other
// window byte; the caller then stages integer codes instead.
__device__ __forceinline__ uint32_t class4(uint32_t x) { return ((x >> 1) ^ (x >> 2)) & 0x03030303u; }
__device__ __forceinline__ uint32_t canon4(uint32_t cl) { return __builtin_amdgcn_perm(0u, 0x54474341u, cl); }
// 0xFF in each byte e < rem (rem clamped to [0, 4])
__device__ __forceinline__ uint32_t byte_mask(int rem) {
    return rem >= 4 ? ~0u : (rem <= 0 ? 0u : ~0u >> (32 - 8 * rem));
}

// One round of up to kRound 16-column chunks per lane: chunk k = k0 + u * G + lg
// (two cover 32 G columns: every window up to 384 bp in one round).
constexpr int kRound = 2;
struct WinRound {
    uint4 a[kRound], b[kRound];
    uint32_t prev[kRound];  // split: the byte before each chunk
};

template <bool SPLIT, bool GEN>
__device__ __forceinline__ void load_round(const SwParams& p, const PairMeta& q, int k0, int lg, int G,
                                           WinRound& w) {
    const uint8_t* wa = win_row<GEN>(p, q.pa, q.sa);
    const uint8_t* wb = win_row<GEN>(p, q.pb, q.sb);
    // last chunk to load per pair: the end of ITS window (not the launch's
    // longest, which a length bucket's short windows would over-read by up to
    // a 128-byte line each), and never past the row or the stream -- lanes
    // past it re-load that chunk (the same line, coalesced)
    const int stream_top = (int)((p.lds_stride - kLead) >> 4);
    const int top = (GEN ? stream_top : min((int)(p.win_stride >> 4), stream_top)) - 1;
    const int top_a = max(min(top, ((q.na + 15) >> 4) - 1), 0);
    const int top_b = max(min(top, ((q.nb + 15) >> 4) - 1), 0);
    const int last = win_last<GEN>(p, q.na);
#pragma unroll
    for (int u = 0; u < kRound; ++u) {
        // clamped chunk index: always a legal load; columns past the window are masked
        const int k = k0 + u * G + lg;
#if MSW_PROBE_NO_WIN
        w.a[u] = w.b[u] = make_uint4(0x03020100u + min(k, top), 0x01000302u, 0x02010003u, 0x00030201u ^ q.pa);
        w.prev[u] = 0;
        (void)wa; (void)wb; (void)last; (void)top_a; (void)top_b;
#else
        w.a[u] = win_chunk<GEN>(wa, min(k, top_a));
        if constexpr (SPLIT) w.prev[u] = wa[min(max(16 * k - 1, 0), last)];
        else w.b[u] = win_chunk<GEN>(wb, min(k, top_b));
#endif
    }
}

template <bool SPLIT>
__device__ __forceinline__ uint32_t sel_round(const PairMeta& q, uint32_t* stream, int k0, int nch, int lg, int G,
                                              const WinRound& w) {
    uint32_t bad = 0u;
#pragma unroll
    for (int u = 0; u < kRound; ++u) {
        const int k = k0 + u * G + lg;
        if (k < nch) {
            const uint32_t xa[4] = {w.a[u].x, w.a[u].y, w.a[u].z, w.a[u].w};
            uint32_t xb[4] = {0u, 0u, 0u, 0u};
            if constexpr (!SPLIT) { xb[0] = w.b[u].x; xb[1] = w.b[u].y; xb[2] = w.b[u].z; xb[3] = w.b[u].w; }
            uint32_t carry = SPLIT ? (w.prev[u] & 0xFFu) : 0u;
            uint4* dst = reinterpret_cast<uint4*>(stream + kLead + 16 * k);
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const int c0 = 16 * k + 4 * d;
                const uint32_t x_a = xa[d];
                const uint32_t ma = byte_mask(q.na - c0);
                uint32_t x_b, mb;
                if constexpr (SPLIT) {  // high half: column c - 1, valid for 1 <= c <= n
                    x_b = (x_a << 8) | carry;
                    carry = x_a >> 24;
                    mb = byte_mask(q.na + 1 - c0) & (c0 == 0 ? ~0xFFu : ~0u);
                } else {
                    x_b = xb[d];
                    mb = byte_mask(q.nb - c0);
                }
                const uint32_t ca = class4(x_a), cb = class4(x_b);
                bad |= ((canon4(ca) ^ x_a) & ma) | ((canon4(cb) ^ x_b) & mb);
                const uint32_t sa = (ca & ma) | (0x0C0C0C0Cu & ~ma);
                const uint32_t sb = ((cb | 0x04040404u) & mb) | (0x0C0C0C0Cu & ~mb);
                uint32_t o[4];
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    // selector bytes {12, sa_e, 12, sb_e}: v_perm leaves 0x00 at bytes 0 and 2
                    o[e] = __builtin_amdgcn_perm(sb, sa, 0x000C000Cu | (uint32_t)e << 8 | (uint32_t)(4 + e) << 24) |
                           0x000C000Cu;
                dst[d] = make_uint4(o[0], o[1], o[2], o[3]);
            }
        }
    }
    return bad;
}

// ---------------------------------------------------------------------------
// The DP.  Per packed cell pair (same (i, j) in both halves):
//  integer path (any bytes, any scheme):
//   linear:  a  = min(rc ^ w, delta)            substitution penalty 0 / delta
//            t1 = sat(DG - a)                   DG = H_diag + match -> max(H_diag + s, 0)
//            h  = max3(t1, E_left, E_up)        E = sat(H - gap)
//   affine:  every H, E, F and t1 carries a bias K = 256 + ge (H* = H + K),
//            which keeps all their subtractions non-negative per u16 half, so
//            they run as full-rate v_sub_u32/v_add_u32 on the packed pair:
//            t1* = (H*_diag + match) - a          (may sit below K: negative)
//            E*  = max(E*_left - ge, GK_left)     GK = sat(H* - (go+ge+K)) + K
//            F*  = max(F*_up   - ge, GK_up)       = max(H - go - ge, 0) + K
//            h*  = max3(t1*, E*, F*)  >= K: the zero floor comes from GK.
//  f16 path (ACGT windows, see above), values H * 2^-11:
//   linear:  t1 = H_diag + s                    s = perm(table_hi, table_lo, selector)
//            h  = max3(t1, E_left, E_up)        E = clamp(H - gap) >= 0
//   affine:  G  = clamp(H - go - ge)
//            E  = max(E_left - ge, G_left),  F = max(F_up - ge, G_up)
//            h  = max3(t1, E, F)                (E, F >= 0: the zero floor)
//   Diagonal term of the next row and column, formed in the row chain (below).
// ---------------------------------------------------------------------------
// Row-group scheduling of the f16 loop (kPermLead in sw_body), per variant:
// 0 = hipcc's own schedule.  MI355X, 10k pairs (tools/ab_sweep.sh): linear
// 54.0 -> 49.8 us with 2 (1: 53.1, 3: 53.8); every other variant is as fast
// or faster with 0 (linear + coords 66.4 vs 67.6, affine + coords 97.0 vs 111).
// Prologue order (profiles/r02/ab/): window loads issued
// with the read loads, before the wave waits on the pair lengths.
// Explicitly scheduled f16 loops of the pairs layout (see sw_body), per
// scoring kind.  MI355X, tools/sched_ab.sh (10k pairs = one wave per SIMD /
// 65k-200k pairs), explicit vs hipcc's schedule: linear 46.0 vs 48.1 us /
// 227 vs 231 us, linear + coords 69.5 vs 77.2 / 347 vs 354, affine + coords
// 102.9 vs 103.4 / 1585 vs 1594 (200k); affine score-only is faster with
// hipcc's own schedule at 10k (81.1 vs 85.4, equal at 65k), so it keeps it.
constexpr bool explicit_sched(bool affine, bool coords) { return !affine || coords; }
// Wavefront steps per loop iteration, per variant (2 or 4; 4 halves the
// LDS-address adds and avoids rotating the prefetched window words), and
// whether an odd KR's last row is folded into the score two steps at a time
// (one max3 per two steps instead of one max per step).  MI355X, tools/ab_sweep.sh
// (10k / 65k pairs): 4 steps -- linear 9.00 -> 9.25 / 12.20 -> 12.61 TCUPS,
// affine 4.97 -> 5.48 / 7.08 -> 7.17; with best-cell keys it loses (linear +
// coords 6.77 -> 6.03, affine + coords 4.64 -> 3.97 at 10k), so those keep 2.
// An odd KR's last row is folded into the score two steps at a time.
constexpr int step_unroll(bool /*affine*/, bool coords) { return coords ? 2 : 4; }
constexpr int perm_lead(bool affine, bool coords) { return !affine && !coords ? 2 : 0; }

template <int KR, bool AFFINE, bool COORDS, bool SPLIT, bool GEN = false>
__device__ __forceinline__ bool sw_body(const SwParams& p, uint32_t block, uint32_t* lds, uint64_t& t_loop) {
    const int lane = threadIdx.x;
    const int G = (int)p.group_lanes;
    const int g_raw = lane / G;
    // Lanes past groups * G idle: they run the loop on group 0's stream with
    // empty pairs and write nothing.
    const bool active = g_raw < (int)p.groups;
    const int g = active ? g_raw : 0;
    const int lg = active ? lane - g_raw * G : 0;
    // An opaque all-ones / zero word (not a bool), so the AND after the DPP
    // move folds into one v_and_b32_dpp instead of becoming a v_cndmask.
    uint32_t top_mask = lg == 0 ? 0u : ~0u;
    asm volatile("" : "+v"(top_mask));
    const PairMeta q = load_meta<SPLIT, GEN>(p, g, block, active);
    // Staging.  The lengths, the read bytes and the first round of window
    // chunks are all in flight before anything waits on the lengths (one
    // memory round trip); 16-byte aligned batches under an f16 scheme stage
    // selectors directly and fall back to integer codes only if some window
    // byte of the wave is not A/C/G/T.
    uint32_t rb_a[KR], rb_b[KR];
    load_read_bytes<KR, SPLIT>(p, q.pa, q.pb, lg, rb_a, rb_b);
    const bool try_fast = p.f16_ok && p.win_vec;
    WinRound w0;
    if (try_fast) load_round<SPLIT, GEN>(p, q, 0, lg, G, w0);
    const int skew = SPLIT ? 2 * (G - 1) + 1 : G - 1;
    // wavefront steps, rounded up to a multiple of the steps per iteration
    // (the explicitly scheduled f16 loops of the pairs layout run four steps
    // per iteration; an integer-path wave of the same kernel then rounds to four too)
    constexpr int kUnroll = (!SPLIT && explicit_sched(AFFINE, COORDS)) ? 4 : step_unroll(AFFINE, COORDS);
    const int steps = (wave_max_nonneg(max(q.na, q.nb)) + skew + kUnroll - 1) & ~(kUnroll - 1);
    uint32_t* stream = lds + g * p.lds_stride;
    uint32_t rc[KR];
    read_codes<KR, SPLIT>(p, q, lg, rb_a, rb_b, rc);
    bool fast;
    if (try_fast) {
        const int nch = (int)((p.lds_stride - kLead) >> 4);  // chunks of the whole stream
        uint32_t bad = 0u;
        if (active) {
            for (int k = lg; k < kLead; k += G) stream[k] = 0x0C0C0C0Cu;
            bad = sel_round<SPLIT>(q, stream, 0, nch, lg, G, w0);
            for (int k0 = kRound * G; k0 < nch; k0 += kRound * G) {  // windows past 16 kRound G columns
                WinRound w;
                load_round<SPLIT, GEN>(p, q, k0, lg, G, w);
                bad |= sel_round<SPLIT>(q, stream, k0, nch, lg, G, w);
            }
        }
        fast = __builtin_amdgcn_ballot_w64(bad != 0u) == 0;
        if (!fast) stage_window<SPLIT, GEN>(p, q, stream, steps, lg, G, active);
    } else {
        stage_window<SPLIT, GEN>(p, q, stream, steps, lg, G, active);
        __syncthreads();
        fast = to_fast_path(stream, kLead + steps, lg, G, active, p.code_shift, p.f16_ok != 0);
    }
    __syncthreads();

    uint32_t E[KR], GK[AFFINE ? KR : 1];
    uint32_t key_a[COORDS ? KR : 1], key_b[COORDS ? KR : 1];
    uint32_t best = 0u;
    // lane reads column t - lg (pairs) / t - 2lg (split) at stream index kLead + that
    const uint32_t* wp = stream + (kLead - (SPLIT ? 2 * lg : lg));
    const uint32_t nj_lane = (uint32_t)(0xFFFF + (SPLIT ? 2 * lg : lg));
    const uint32_t lds_wp = (uint32_t)(uintptr_t)wp;  // LDS byte address of wp[0]

    // The whole DP for one arithmetic domain: F16 = ACGT table lookups on f16
    // values, else xor/min on the byte codes with u16 integer values.
    auto run = [&](auto f16_tag) __attribute__((always_inline)) {
        constexpr bool F16 = decltype(f16_tag)::value;
        // integer path constants
        const uint32_t match2 = p.match2, delta2 = p.delta2, ext2 = p.gap2, oe2 = p.open_ext2;
        const uint32_t bias2 = (AFFINE && !F16) ? p.bias2 : 0u;  // K in both halves (integer affine)
        const uint32_t kmatch2 = add_nc(bias2, match2);
        const uint32_t og2 = oe2 - bias2;                       // integer affine: go + ge
        // f16 path constants: -gap (linear) / -ge (affine), -(go + ge)
        const uint32_t nge = p.f16_ngap2, noe = p.f16_noe2;
        uint32_t tab_lo[F16 ? KR : 1], tab_hi[F16 ? KR : 1];
        if constexpr (F16) {
            const uint32_t mis4 = (p.f16_hi >> 8) * 0x01010101u, match_hi = p.f16_hi & 0xFFu;
#pragma unroll
            for (int r = 0; r < KR; ++r) {
                tab_lo[r] = row_table(rc[r] & 0xFFFFu, p.code_shift, mis4, match_hi);
                tab_hi[r] = row_table(rc[r] >> 16, p.code_shift, mis4, match_hi);
            }
        }
        // F16: the substitution score s; integer: the penalty a = match - s.
        auto sub = [&](int r, uint32_t w) __attribute__((always_inline)) -> uint32_t {
            if constexpr (F16) return __builtin_amdgcn_perm(tab_hi[r], tab_lo[r], w);
            else return pk_min(rc[r] ^ w, delta2);
        };
#pragma unroll
        for (int r = 0; r < KR; ++r) {
            E[r] = bias2;                                    // E = 0 (integer affine: E* = K)
            if constexpr (AFFINE) GK[r] = bias2;             // G = 0
            if constexpr (COORDS) { key_a[r] = 0u; key_b[r] = 0u; }
        }
        uint32_t f_bot = bias2, h_bot = bias2;               // F = 0, H = 0

        // Software pipeline: t1 (the diagonal term) of step t+1 is formed inside
        // step t's row chain, as soon as the H it needs is known, so each link of
        // the dependent max3 -> sub chain has independent work beside it
        // (waves issue in order; a lone wave otherwise stalls on every link).
        uint32_t t1a[KR], t1b[KR];
        using P0 = std::integral_constant<int, 0>;
        using P1 = std::integral_constant<int, 1>;
        if constexpr (F16 && !SPLIT && explicit_sched(AFFINE, COORDS)) {
            // The f16 loops of the pairs layout (every config's main kernel),
            // explicitly scheduled.  Every instruction is pinned by a
            // sched_barrier so that each link of the row chain -- linear:
            // max3 -> clamp -> max3; affine: F = max(F_up - ge, G_up) -> max3 ->
            // G = clamp(H - go - ge) -> next row's F -- has an independent
            // instruction beside it: the substitution perm of the next row, the
            // next step's diagonal add, the next row's E, a best-cell key or a
            // score fold.  That keeps a lone wave (one per SIMD, config 2)
            // issuing without dependency stalls AND without the wait states
            // hipcc otherwise inserts (an s_nop between a v_pk_maximum3_f16 and
            // its immediate consumer, 13 per four linear steps, and an s_nop 1
            // before the DPP hand-off), which cost a lone wave ~3.8 / ~7.8
            // cycles each (tools/ubench_valu.hip, profiles/r02/ubench_valu_gfx950.txt);
            // it also makes the loop immune to hipcc's register-pressure-driven
            // rescheduling (affine + coordinates ran 96 or 104 us at 10k pairs
            // depending on unrelated prologue code).  The next step's row-0
            // perm is issued in the last row's slot (it needs the word of step
            // t+2, w2); score folds (rows 2k, 2k+1) run two rows later, the
            // last pair at the next step's start; the hand-offs (DPP) for the
            // next step are issued at the end of this one, three or more
            // instructions after the rows they read.
#define MSW_SB __builtin_amdgcn_sched_barrier(0)
            {
                const uint32_t w0 = wp[0];
#pragma unroll
                for (int r = 0; r < KR; ++r) t1a[r] = sub(r, w0);   // H_diag = 0
            }
            uint32_t an0 = sub(0, wp[1]);  // row 0's substitution at step 1's column
            uint32_t hpend = 0u, hkm2 = 0u;
            uint32_t hu = shr1_group(h_bot, top_mask);                  // H of the row above
            uint32_t fu = AFFINE ? shr1_group(f_bot, top_mask) : 0u;   // F of the row above (affine)
            auto sstep = [&](int t, uint32_t w1, uint32_t w2, const uint32_t (&t1)[KR], uint32_t (&t1n)[KR],
                             auto parity) __attribute__((always_inline)) {
                constexpr int kParity = decltype(parity)::value;
                // linear: up = E of the row above; affine: fsub = F_up - ge (the
                // row's F needs G_up from the previous row's clamp), e_next = the
                // next row's E = max(E_left - ge, G_left), both formed a row ahead
                uint32_t up = 0u, g_up = 0u, e_next = 0u, fsub = 0u;
                if constexpr (AFFINE) {
                    fsub = hadd(fu, nge);
                    MSW_SB;
                    g_up = hadd_clamp(hu, noe);
                    MSW_SB;
                    const uint32_t el = hadd(E[0], nge);
                    MSW_SB;
                    t1n[0] = hadd(hu, an0);
                    MSW_SB;
                    e_next = hmax(el, GK[0]);
                    MSW_SB;
                } else {
                    up = hadd_clamp(hu, nge);
                    MSW_SB;
                    t1n[0] = hadd(hu, an0);
                    MSW_SB;
                }
                uint32_t nja = 0u;
                if constexpr (COORDS) {
                    nja = (nj_lane - (uint32_t)t) & 0xFFFFu;
                    MSW_SB;
                } else if constexpr (KR & 1) {
                    // score fold left over from the previous step: odd KR pairs
                    // the last rows of two steps, even KR the previous step's last pair
                    if constexpr (kParity == 0) {
                        best = track_max3(best, hpend, h_bot);
                        MSW_SB;
                    } else {
                        hpend = h_bot;
                    }
                } else {
                    best = track_max3(best, hkm2, h_bot);
                    MSW_SB;
                }
                uint32_t hh[KR];
                // Best-cell keys of row r - 1 are formed during row r (two
                // instructions) and folded into the running maxima a few slots
                // later, so neither waits on a fresh value; the last row's after
                // the loop.
                uint32_t ka = 0u, kb = 0u;
                auto key_form = [&](int r) __attribute__((always_inline)) {
                    ka = (hh[r] << 16) | nja;
                    MSW_SB;
                    kb = (hh[r] & 0xFFFF0000u) | nja;
                    MSW_SB;
                };
                auto key_fold = [&](int r) __attribute__((always_inline)) {
                    key_a[r] = max(key_a[r], ka);
                    MSW_SB;
                    key_b[r] = max(key_b[r], kb);
                    MSW_SB;
                };
#pragma unroll
                for (int r = 0; r < KR; ++r) {
                    const bool last = r + 1 == KR;
                    uint32_t h, a = 0u;
                    if constexpr (AFFINE) {
                        // F -> [el, perm] -> h -> [fsub, e_next, keys r-1] -> G -> [t1n, keys r-1] -> next F
                        const uint32_t e = e_next;
                        const uint32_t F = hmax(fsub, g_up);                // [chain]
                        MSW_SB;
                        uint32_t el = 0u;
                        if (!last) {
                            el = hadd(E[r + 1], nge);
                            MSW_SB;
                            a = sub(r + 1, w1);
                        } else {
                            an0 = sub(0, w2);
                        }
                        MSW_SB;
                        h = pk_max3(t1[r], e, F);                           // [chain]
                        MSW_SB;
                        hh[r] = h;
                        E[r] = e;
                        if (!last) fsub = hadd(F, nge);
                        else fu = shr1_group(F, top_mask);                  // next step's F hand-off
                        MSW_SB;
                        if (!last) {
                            e_next = hmax(el, GK[r + 1]);
                            MSW_SB;
                        }
                        if constexpr (COORDS) {
                            if (r > 0) key_form(r - 1);
                        }
                        g_up = GK[r] = hadd_clamp(h, noe);                  // [chain]
                        MSW_SB;
                    } else {
                        // h -> [perm, keys r-1] -> E -> [t1n, keys r-1] -> next h
                        h = pk_max3(t1[r], E[r], up);                       // [chain]
                        MSW_SB;
                        hh[r] = h;
                        if (!last) a = sub(r + 1, w1);
                        else an0 = sub(0, w2);
                        MSW_SB;
                        if constexpr (COORDS) {
                            if (r > 0) key_form(r - 1);
                        }
                        up = E[r] = hadd_clamp(h, nge);                     // [chain]
                        MSW_SB;
                    }
                    if (!last) {
                        t1n[r + 1] = hadd(h, a);
                        MSW_SB;
                    }
                    if constexpr (COORDS) {
                        if (r > 0) key_fold(r - 1);
                    } else if (r >= 2 && (r & 1) == 0) {
                        best = track_max3(best, hh[r - 2], hh[r - 1]);
                        MSW_SB;
                    }
                }
                if constexpr (COORDS) {
                    key_form(KR - 1);
                    key_fold(KR - 1);
                }
                h_bot = hh[KR - 1];
                if constexpr (!COORDS && (KR & 1) == 0) hkm2 = hh[KR - 2];
                hu = shr1_group(h_bot, top_mask);
                MSW_SB;
            };
            uint2 wa = make_uint2(wp[1], wp[2]);
            uint2 wb;
            asm volatile("ds_read2_b32 %0, %1 offset0:3 offset1:4" : "=v"(wb) : "v"(lds_wp));
            for (int t = 0; t < steps; t += 4) {
                const uint32_t base = lds_wp + 4u * (uint32_t)t;
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wb));
                sstep(t, wa.x, wa.y, t1a, t1b, P0{});
                sstep(t + 1, wa.y, wb.x, t1b, t1a, P1{});
                asm volatile("ds_read2_b32 %0, %1 offset0:5 offset1:6" : "=v"(wa) : "v"(base));
                sstep(t + 2, wb.x, wb.y, t1a, t1b, P0{});
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wa));
                sstep(t + 3, wb.y, wa.x, t1b, t1a, P1{});
                asm volatile("ds_read2_b32 %0, %1 offset0:7 offset1:8" : "=v"(wb) : "v"(base));
            }
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wb));
            // the score pair still pending after the last (odd) step
            if constexpr (!COORDS) best = track_max3(best, (KR & 1) ? hpend : hkm2, h_bot);
#undef MSW_SB
            return;
        }
        {
            const uint32_t w0 = wp[0];
#pragma unroll
            for (int r = 0; r < KR; ++r) {
                const uint32_t a = sub(r, w0);               // H_diag = 0
                t1a[r] = F16 ? a : (AFFINE ? kmatch2 - a : pk_satsub(match2, a));
            }
        }
        // One wavefront step: consumes t1 (this step's diagonal terms), produces
        // t1n (the next step's) from w, the window word of step t + 1.  Called
        // with alternating buffers so the hand-over needs no register copies.
        uint32_t hpend = 0u;  // last row's H of the even step, folded with the odd one's
        auto step = [&](int t, uint32_t w, const uint32_t (&t1)[KR], uint32_t (&t1n)[KR], auto parity)
                        __attribute__((always_inline)) {
            constexpr int kParity = decltype(parity)::value;
            // Unbiased values cross the lanes (the zero fill is the top boundary),
            // the bias is re-added on arrival: no u16 half ever goes negative.
            // Only H (and affine F) cross: E resp. G of the row above are
            // functions of its H, recomputed here instead of a second DPP move.
            const uint32_t h_up = from_above<SPLIT>(h_bot - bias2, top_mask);
            uint32_t up;    // linear: E of the row above; affine: F of the row above
            uint32_t g_up;  // affine: G of the row above
            if constexpr (F16) {
                if constexpr (AFFINE) {
                    up = from_above<SPLIT>(f_bot, top_mask);
                    g_up = hadd_clamp(h_up, noe);
                } else {
                    up = hadd_clamp(h_up, nge);
                    g_up = 0u;
                }
            } else if constexpr (AFFINE) {
                up = add_nc(from_above<SPLIT>(f_bot - bias2, top_mask), bias2);
                g_up = add_nc(pk_satsub(h_up, og2), bias2);
            } else {
                up = pk_satsub(h_up, ext2);
                g_up = 0u;
            }
            // Substitution terms of the next column.  With kPermLead > 0 the f16
            // loop issues them kPermLead rows ahead, one per row group, and fences
            // each row group (sched_barrier): a lone wave issues in order, and a
            // perm between the max3 -> clamp -> max3 links of the row chain fills
            // the wait for their results (hipcc otherwise bunches the perms up
            // front).  Measured per variant (perm_lead above).
            constexpr int kPermLead = F16 ? perm_lead(AFFINE, COORDS) : 0;
            uint32_t a_n[KR];
#pragma unroll
            for (int r = 0; r < KR; ++r)
                if (!kPermLead || r < kPermLead) a_n[r] = sub(r, w);
            // row 0's diagonal next step: the lane above's H now
            if constexpr (F16) t1n[0] = hadd(h_up, a_n[0]);
            else t1n[0] = AFFINE ? add_nc(h_up, kmatch2) - a_n[0] : pk_satsub(add_nc(h_up, kmatch2), a_n[0]);
            const uint32_t nj_a = (nj_lane - (uint32_t)t) & 0xFFFFu;
            const uint32_t nj_b = SPLIT ? ((nj_lane + 1u - (uint32_t)t) & 0xFFFFu) : nj_a;
            uint32_t hprev = 0u;
#pragma unroll
            for (int r = 0; r < KR; ++r) {
                uint32_t h;
                if constexpr (F16) {
                    if (kPermLead && r + kPermLead < KR) a_n[r + kPermLead] = sub(r + kPermLead, w);
                    if constexpr (AFFINE) {
                        const uint32_t e = hmax(hadd(E[r], nge), GK[r]);
                        up = hmax(hadd(up, nge), g_up);
                        h = pk_max3(t1[r], e, up);
                        E[r] = e;
                        g_up = GK[r] = hadd_clamp(h, noe);
                    } else {
                        h = pk_max3(t1[r], E[r], up);
                        up = E[r] = hadd_clamp(h, nge);
                    }
                    if (r + 1 < KR) t1n[r + 1] = hadd(h, a_n[r + 1]);
                } else if constexpr (AFFINE) {
                    const uint32_t e = pk_max(E[r] - ext2, GK[r]);     // full-rate sub, no borrow
                    up = pk_max(up - ext2, g_up);
                    h = pk_max3(t1[r], e, up);
                    E[r] = e;
                    g_up = GK[r] = add_nc(pk_satsub(h, oe2), bias2);   // oe2 = go + ge + K
                    if (r + 1 < KR) t1n[r + 1] = add_nc(h, match2) - a_n[r + 1];
                } else {
                    h = pk_max3(t1[r], E[r], up);
                    up = E[r] = pk_satsub(h, ext2);
                    if (r + 1 < KR) t1n[r + 1] = pk_satsub(add_nc(h, match2), a_n[r + 1]);
                }
                if (r + 1 == KR) h_bot = h;
                if constexpr (COORDS) {
                    key_a[r] = max(key_a[r], (h << 16) | nj_a);
                    key_b[r] = max(key_b[r], (h & 0xFFFF0000u) | nj_b);
                } else {
                    if (r & 1) {
                        best = track_max3(best, hprev, h);
                    } else if (r + 1 == KR) {  // an odd KR's last row: folded two steps at a time
                        if constexpr (kParity == 0) hpend = h;
                        else best = track_max3(best, hpend, h);
                    }
                    hprev = h;
                }
                if constexpr (kPermLead > 0) __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (AFFINE) f_bot = up;
        };
        // Step count rounded up to a multiple of the steps per iteration: the
        // extra steps score padding columns,
        // which never reach a real cell's score.
        // The window words are read from LDS two steps or more before use, so
        // a lone wave never waits on LDS latency.  The read is an asm
        // statement (hipcc would otherwise sink it to the consuming iteration); its
        // wait names the destination, so nothing reads it before the data lands.
        if constexpr (kUnroll == 4) {
            // Four steps per iteration: the words of steps t+1..t+2 (wa) and
            // t+3..t+4 (wb) are each re-read into the same registers right after
            // their last use, two steps before they are needed again, and one
            // address add serves four steps.
            uint2 wa = make_uint2(wp[1], wp[2]);
            uint2 wb;
            asm volatile("ds_read2_b32 %0, %1 offset0:3 offset1:4" : "=v"(wb) : "v"(lds_wp));
            for (int t = 0; t < steps; t += 4) {
                const uint32_t base = lds_wp + 4u * (uint32_t)t;
                step(t, wa.x, t1a, t1b, P0{});
                step(t + 1, wa.y, t1b, t1a, P1{});
                asm volatile("ds_read2_b32 %0, %1 offset0:5 offset1:6" : "=v"(wa) : "v"(base));
                asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(wb));
                step(t + 2, wb.x, t1a, t1b, P0{});
                step(t + 3, wb.y, t1b, t1a, P1{});
                asm volatile("ds_read2_b32 %0, %1 offset0:7 offset1:8" : "=v"(wb) : "v"(base));
                asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(wa));
            }
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wb));
        } else {
            uint32_t w1 = wp[1], w2 = wp[2];
            uint2 wn;
            asm volatile("ds_read2_b32 %0, %1 offset0:3 offset1:4" : "=v"(wn) : "v"(lds_wp));
            for (int t = 0; t < steps; t += 2) {
                step(t, w1, t1a, t1b, P0{});
                step(t + 1, w2, t1b, t1a, P1{});
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wn));
                w1 = wn.x;
                w2 = wn.y;
                asm volatile("ds_read2_b32 %0, %1 offset0:3 offset1:4"
                             : "=v"(wn) : "v"(lds_wp + 4u * (uint32_t)(t + 2)));
            }
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wn));
        }
    };
    if (p.trace) t_loop = __builtin_amdgcn_s_memrealtime();
    if (fast) run(std::true_type{});
    else run(std::false_type{});

    const uint32_t bias = fast ? 0u : (p.bias2 & 0xFFFFu) * (AFFINE ? 1u : 0u);
    if constexpr (COORDS) finish_coords<KR, SPLIT>(p, q, lg, G, key_a, key_b, bias, fast);
    else finish_score<SPLIT>(p, q, lg, G, best, bias, fast);
    return fast;
}

// Diagnostics (MSW_WAVE_TRACE, tools/wave_trace.py): per block, start and end
// on the 100 MHz constant clock, the shader-clock cycles between them, the
// ticks spent before the DP loop (staging), the wave's HW_ID / XCC_ID and
// what it ran.
struct WaveClock {
    uint64_t t0, c0;
};
__device__ __forceinline__ WaveClock trace_begin(const SwParams& p) {
    WaveClock w{0, 0};
    if (p.trace) {
        w.t0 = __builtin_amdgcn_s_memrealtime();
        w.c0 = __builtin_amdgcn_s_memtime();
    }
    return w;
}
__device__ __forceinline__ void trace_end(const SwParams& p, const WaveClock& w, bool fast, bool split,
                                          int kr, uint64_t t_loop) {
    if (!p.trace) return;
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        const uint32_t hw_id = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));    // HW_REG_XCC_ID
        uint64_t* o = p.trace + 4ull * blockIdx.x;
        o[0] = w.t0;
        o[1] = t1;
        o[2] = (uint64_t)hw_id | ((uint64_t)xcc << 32) | ((uint64_t)fast << 40) | ((uint64_t)split << 41) |
               ((uint64_t)kr << 48);
        // shader cycles (40 bits) | constant-clock ticks before the DP loop << 40
        o[3] = ((c1 - w.c0) & 0xFFFFFFFFFFull) | ((t_loop - w.t0) << 40);
    }
}

// Blocks are dealt round-robin over the 8 XCDs (blocks b and b + 8 share
// one; MI355X_MICROARCH.md, workgroup dispatch), each XCD with its own L2.
// Adjacent blocks score adjacent pairs, whose row ends and length / order
// entries share cache lines, so the identity map has up to 8 L2s fetch each
// such line.  This (bijective) map gives each run of G consecutive logical
// blocks to one XCD, within full windows of 8G blocks (a tail keeps the
// identity); dispatch order moves by < 8G blocks, so heaviest-first grids
// stay heaviest first.  Speed only (traffic), never correctness.
template <uint32_t G>
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
    constexpr uint32_t span = 8u * G;
    const uint32_t base = b - b % span;
    if (base + span > nb) return b;
    const uint32_t r = b - base;
    return base + (r % 8u) * G + r / 8u;
}

// One layout for the whole grid (GEN: windows read from the resident genome).
template <int KR, bool AFFINE, bool COORDS, bool SPLIT, bool GEN = false>
__global__ __launch_bounds__(64) void sw_kernel(SwParams p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const WaveClock wc = trace_begin(p);
    uint64_t t_loop = 0;
    // identity block order: the XCD-grouped map below cut config 2's fetched
    // bytes 5.36 -> 4.99 MB per launch but slowed it 46.2 -> 50.2 us
    // (profiles/r03/traffic/xcd_remap_ab.jsonl); kept for the bucketed grid
    const bool fast = sw_body<KR, AFFINE, COORDS, SPLIT, GEN>(p, blockIdx.x, lds, t_loop);
    trace_end(p, wc, fast, SPLIT, KR, t_loop);
}

// Mixed grid for small batches: blocks [0, p.pairs_blocks) run the pairs
// layout (8 pairs each, at most one per SIMD), the rest the split layout
// (4 pairs each) over the remaining slots; the block's layout is uniform.
// Waves are dispatched in block order, so the split waves fill in beside the
// pairs waves instead of stacking a second 8-pair wave on some SIMDs.
template <int KRP, bool AFFINE, bool COORDS>
__global__ __launch_bounds__(64) void sw_mixed_kernel(SwParams p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const WaveClock wc = trace_begin(p);
    uint64_t t_loop = 0;
    if (blockIdx.x < p.pairs_blocks) {
        const bool fast = sw_body<KRP, AFFINE, COORDS, false>(p, blockIdx.x, lds, t_loop);
        trace_end(p, wc, fast, false, KRP, t_loop);
    } else {
        SwParams q = p;
        const uint32_t done = p.pairs_blocks * pairs_per_wave(false, p.groups);
        q.n_slots = p.n_slots - done;
        q.order = p.order ? p.order + done : nullptr;
        if (!p.order) q.slot_base = done;
        q.out_slot_base = p.out_slot_base + done;
        const bool fast = sw_body<(KRP + 1) / 2, AFFINE, COORDS, true>(q, blockIdx.x - p.pairs_blocks, lds,
                                                                      t_loop);
        trace_end(p, wc, fast, true, (KRP + 1) / 2, t_loop);
    }
}

// Length-bucketed grid (MultiTable): each block finds its bucket (<= 16
// entries, wave-uniform scalar scan) and runs the pairs layout with that
// bucket's rows per lane, window stream stride and f16 eligibility.  One
// launch for a whole mixed-length batch: no per-bucket launch tails.
template <int KR, bool AFFINE, bool COORDS>
__device__ __forceinline__ void multi_body(const SwParams& q, uint32_t blk, uint32_t* lds) {
    const WaveClock wc = trace_begin(q);
    uint64_t t_loop = 0;
    const bool fast = sw_body<KR, AFFINE, COORDS, false>(q, blk, lds, t_loop);
    trace_end(q, wc, fast, false, KR, t_loop);
}

// WIDE: the table's buckets have 17..24 rows per lane (reads of 257..384
// bases) -- a separate instance, so their registers do not lower the
// occupancy of the common KR <= 16 instance.
template <bool AFFINE, bool COORDS, bool WIDE = false>
__global__ __launch_bounds__(64) void sw_multi_kernel(SwParams p, MultiTable t) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t lb = xcd_block<4>(blockIdx.x, gridDim.x);
    uint32_t b = 0;
    while (b + 1 < t.n_buckets && lb >= t.block_end[b]) ++b;
    const uint32_t blk = lb - (b ? t.block_end[b - 1] : 0u);
    SwParams q = p;
    q.order = p.order + t.slot_begin[b];
    q.out_slot_base = p.out_slot_base + t.slot_begin[b];
    q.n_slots = t.count[b];
    q.lds_stride = t.lds_stride[b];
    q.f16_ok = t.f16_ok[b];
    if constexpr (WIDE) {
        switch (t.kr[b]) {
            case 17: multi_body<17, AFFINE, COORDS>(q, blk, lds); break;
            case 18: multi_body<18, AFFINE, COORDS>(q, blk, lds); break;
            case 19: multi_body<19, AFFINE, COORDS>(q, blk, lds); break;
            case 20: multi_body<20, AFFINE, COORDS>(q, blk, lds); break;
            case 21: multi_body<21, AFFINE, COORDS>(q, blk, lds); break;
            case 22: multi_body<22, AFFINE, COORDS>(q, blk, lds); break;
            case 23: multi_body<23, AFFINE, COORDS>(q, blk, lds); break;
            default: multi_body<24, AFFINE, COORDS>(q, blk, lds); break;
        }
    } else {
        switch (t.kr[b]) {
            case 1: multi_body<1, AFFINE, COORDS>(q, blk, lds); break;
            case 2: multi_body<2, AFFINE, COORDS>(q, blk, lds); break;
            case 3: multi_body<3, AFFINE, COORDS>(q, blk, lds); break;
            case 4: multi_body<4, AFFINE, COORDS>(q, blk, lds); break;
            case 5: multi_body<5, AFFINE, COORDS>(q, blk, lds); break;
            case 6: multi_body<6, AFFINE, COORDS>(q, blk, lds); break;
            case 7: multi_body<7, AFFINE, COORDS>(q, blk, lds); break;
            case 8: multi_body<8, AFFINE, COORDS>(q, blk, lds); break;
            case 9: multi_body<9, AFFINE, COORDS>(q, blk, lds); break;
            case 10: multi_body<10, AFFINE, COORDS>(q, blk, lds); break;
            case 11: multi_body<11, AFFINE, COORDS>(q, blk, lds); break;
            case 12: multi_body<12, AFFINE, COORDS>(q, blk, lds); break;
            case 13: multi_body<13, AFFINE, COORDS>(q, blk, lds); break;
            case 14: multi_body<14, AFFINE, COORDS>(q, blk, lds); break;
            case 15: multi_body<15, AFFINE, COORDS>(q, blk, lds); break;
            default: multi_body<16, AFFINE, COORDS>(q, blk, lds); break;
        }
    }
}

}  // namespace msw
