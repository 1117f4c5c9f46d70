// msw_long.hip -- Smith-Waterman for pairs beyond the packed kernels' limits
// (read > 256 bases or window > 4096, each up to kMaxLongLen = 32767).
//
// The packed kernels (msw_device.h) keep a whole read in 16 lanes' VGPRs and
// a whole window in an LDS stream, with 16-bit cells; real data has reads
// longer than 256 bases (MiSeq 2x300, long-read fragments) and windows of any
// length, and the reference's recurrence (smith_waterman.cl:112-126, the
// intended SW) has no length limit.  This kernel scores those pairs exactly,
// with the same conventions as the oracle (oracle/sw_oracle.c): i32 cells,
// best cell = max score, then smallest i, then smallest j.
//
// Mapping (one wave64 per pair; blocks take the launch's slots from a work
// queue, heaviest first when the host sorted them -- msw_runtime.cpp
// bucket_chunk -- so mixed lengths balance over the SIMDs):
//  * the read is cut into strips of 64*R rows (R = 1..8 rows per lane); in a
//    strip, lane l owns rows [l*R, l*R+R) and sweeps the window with the
//    one-column-per-lane skew of the packed kernels: at step t it scores
//    column t-l, its top row taking H (and Gotoh's F) of lane l-1's bottom row
//    from the previous step through one DPP wave_shr:1;
//  * lane 0's top input is the previous strip's bottom row, kept in a
//    per-block scratch row in global memory (L2-resident): loaded 64 columns
//    at a time into one VGPR that one DPP wave_shl:1 per step moves down to
//    lane 0, while lane 63's bottom row is collected by another wave_shl:1
//    (lane 63 taking the new value) and stored 64 columns at a time -- the
//    next strip reads column c before this strip overwrites it, so one row
//    serves both;
//  * the window sits in LDS ([64 pad | n bytes | 64 pad]); lane l reads byte
//    t-l each step (64 consecutive bytes: conflict-free);
//  * columns outside [0, n) (the wavefront's fill and drain) are masked to
//    H = 0 only in the 64-step blocks that contain them;
//  * score-only: one v_max per cell; best cell: per row (score, j) with a
//    strict '>' in column order, merged per strip in row order, then one
//    64-bit key reduce over the wave: (score, -i, -j).
// VALU-bound like the packed kernels (~7 i32 ops per cell linear, ~10 affine);
// a fallback for the rare long pair, bit-exact with the same tests.
#include "msw_kernels.h"

#include <type_traits>

namespace msw {
namespace {

constexpr int32_t kNeg = -(1 << 29);  // -inf for E/F: stays far from overflow over 32767 steps
constexpr int32_t kNoMatch = 0x100;   // read code past the read: equals no window byte

// lane l <- src of lane l-1; lane 0 <- lane0 (DPP wave_shr:1, bound_ctrl off:
// the invalid source leaves the old value, which is lane0)
__device__ __forceinline__ int32_t shr1_or(int32_t src, int32_t lane0) {
    return __builtin_amdgcn_update_dpp(lane0, src, 0x138, 0xF, 0xF, false);
}

// lane l <- src of lane l+1; lane 63 <- lane 63 of in63 (DPP wave_shl:1,
// bound_ctrl off): collects lane 63's values of successive steps in a
// register, oldest in lane 0, or (in63 = 0) rotates the next value into lane 0
__device__ __forceinline__ int32_t shl1_or(int32_t src, int32_t in63) {
    return __builtin_amdgcn_update_dpp(in63, src, 0x130, 0xF, 0xF, false);
}

__device__ __forceinline__ int32_t coherent_load(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int R, bool AFFINE, bool COORDS>
__global__ __launch_bounds__(64) void sw_long_kernel(SwParams p) {
    extern __shared__ uint8_t lds_win[];  // [64 pad | window | 64 pad]
    const int lane = (int)threadIdx.x;
    const int32_t match = (int32_t)(p.match2 & 0xFFFFu);
    const int32_t mismatch = match - (int32_t)(p.delta2 & 0xFFFFu);
    const int32_t gap = (int32_t)(p.gap2 & 0xFFFFu);  // linear gap / affine gap_extend
    const int32_t goe = (int32_t)(p.open_ext2 & 0xFFFFu) - (int32_t)(p.bias2 & 0xFFFFu);
    // the substitution values live in VGPRs (v_cndmask operands), loaded once
    int32_t vmatch, vmismatch;
    asm volatile("v_mov_b32 %0, %1" : "=v"(vmatch) : "s"(match));
    asm volatile("v_mov_b32 %0, %1" : "=v"(vmismatch) : "s"(mismatch));
    const uint32_t cols = p.long_cols;
    int32_t* const bnd_h = p.long_scratch ? p.long_scratch + (size_t)blockIdx.x * cols * (AFFINE ? 2u : 1u) : nullptr;
    int32_t* const bnd_f = bnd_h ? bnd_h + cols : nullptr;

    // next slot: one atomic per slot from lane 0 when the queue is on
    auto next_slot = [&](uint32_t slot) {
        if (!p.long_next) return slot + gridDim.x;
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(p.long_next, 1u);
        return gridDim.x + (uint32_t)__builtin_amdgcn_readfirstlane((int)k);
    };
    for (uint32_t slot = blockIdx.x; slot < p.n_slots; slot = next_slot(slot)) {
        const uint32_t pair = p.order ? p.order[slot] : p.slot_base + slot;
        const uint32_t outi = p.out_by_slot ? p.out_slot_base + slot : pair;
        const int m = p.read_len[pair], n = p.win_len[pair];
        const uint8_t* rd = p.reads + (size_t)pair * p.read_stride;
        const uint8_t* wn = p.wins + (size_t)pair * p.win_stride;
        __syncthreads();  // the previous slot's window reads are done
        for (int k = lane; k < n; k += 64) lds_win[64 + k] = wn[k];
        __syncthreads();

        // running best of this lane's rows over all strips
        int32_t lbest = 0, li = -1, lj = -1;
        const int strips = (m > 0 && n > 0) ? (m + 64 * R - 1) / (64 * R) : 0;
        for (int s = 0; s < strips; ++s) {
            const bool bin = s > 0, bout = s + 1 < strips;  // wave-uniform
            const int row0 = s * 64 * R + lane * R;
            int32_t rb[R], hl[R], h2[R], ee[R], bs[R], bj[R];
#pragma unroll
            for (int k = 0; k < R; ++k) {
                rb[k] = row0 + k < m ? (int32_t)rd[row0 + k] : kNoMatch;
                hl[k] = 0;
                ee[k] = kNeg;
                bs[k] = 0;
                bj[k] = -1;
            }
            int32_t best = 0;
            int32_t hb = 0, fb = kNeg, dg = 0;  // bottom row H / F of the last step; row 0's diagonal
            int32_t bo_h = 0, bo_f = kNeg;      // lane 63's bottom row of the last 64 steps (oldest in lane 0)
            const int steps = n + 63;
            for (int tb = 0; tb < steps; tb += 64) {
                // previous strip's bottom row, columns [tb, tb + 64); lane 0
                // holds column t (shifted down one lane per step)
                int32_t bi_h = 0, bi_f = kNeg;
                if (bin) {
                    bi_h = coherent_load(bnd_h + tb + lane);
                    if (AFFINE) bi_f = coherent_load(bnd_f + tb + lane);
                }
                // one step: H of the lane's rows at column t - lane; `in` holds
                // them at the previous column (left; row k-1's is row k's
                // diagonal), `out` receives them -- two steps per iteration
                // swap the arrays instead of copying registers
                auto step = [&](auto mask_tag, int u, const int32_t(&in)[R], int32_t(&out)[R])
                                __attribute__((always_inline)) {
                    constexpr bool MASK = decltype(mask_tag)::value;
                    const int t = tb + u;
                    const int32_t up0 = shr1_or(hb, bi_h);
                    int32_t fu = kNeg;
                    if (AFFINE) fu = shr1_or(fb, bi_f);
                    if (bin) {
                        bi_h = shl1_or(bi_h, 0);
                        if (AFFINE) bi_f = shl1_or(bi_f, kNeg);
                    }
                    const int j = t - lane;
                    const int32_t w = lds_win[64 + j];
                    const bool ok = !MASK || (uint32_t)j < (uint32_t)n;
#pragma unroll
                    for (int k = 0; k < R; ++k) {
                        const int32_t diag = k ? in[k - 1] : dg;
                        const int32_t up = k ? out[k - 1] : up0;
                        const int32_t sc = rb[k] == w ? vmatch : vmismatch;
                        int32_t h;
                        if (AFFINE) {
                            ee[k] = max(ee[k] - gap, in[k] - goe);
                            fu = max(fu - gap, up - goe);
                            h = max(max(diag + sc, ee[k]), max(fu, 0));
                        } else {
                            h = max(max(diag + sc, max(up, in[k]) - gap), 0);
                        }
                        if (MASK) h = ok ? h : 0;
                        if (COORDS) {
                            if (h > bs[k]) {
                                bs[k] = h;
                                bj[k] = j;
                            }
                        } else {
                            best = max(best, h);
                        }
                        out[k] = h;
                    }
                    dg = up0;
                    hb = out[R - 1];
                    if (AFFINE) fb = fu;
                    if (bout) {
                        // lane 63 scored column c = t - 63 of the strip's bottom row
                        const int c = t - 63;
                        bo_h = shl1_or(bo_h, hb);
                        if (AFFINE) bo_f = shl1_or(bo_f, fb);
                        if ((c & 63) == 63 && c >= 63) {  // lanes hold columns [c - 63, c]
                            bnd_h[c - 63 + lane] = bo_h;
                            if (AFFINE) bnd_f[c - 63 + lane] = bo_f;
                        }
                    }
                };
                auto block = [&](auto mask_tag) __attribute__((always_inline)) {
                    const int ue = min(64, steps - tb);
                    int u = 0;
                    for (; u + 1 < ue; u += 2) {
                        step(mask_tag, u, hl, h2);
                        step(mask_tag, u + 1, h2, hl);
                    }
                    if (u < ue) {
                        step(mask_tag, u, hl, h2);
#pragma unroll
                        for (int k = 0; k < R; ++k) hl[k] = h2[k];
                    }
                };
                if (tb >= 63 && tb + 64 <= n) block(std::false_type{});
                else block(std::true_type{});
            }
            if (bout && (n & 63) != 0 && n - 64 + lane >= 0) {  // lanes hold columns [n - 64, n - 1]
                bnd_h[n - 64 + lane] = bo_h;
                if (AFFINE) bnd_f[n - 64 + lane] = bo_f;
            }
            if (COORDS) {
#pragma unroll
                for (int k = 0; k < R; ++k)
                    if (bs[k] > lbest) {  // rows in increasing i: strict '>' keeps the smallest i
                        lbest = bs[k];
                        li = row0 + k;
                        lj = bj[k];
                    }
            } else {
                lbest = max(lbest, best);
            }
            __syncthreads();  // this strip's bottom row is stored before the next strip loads it
        }
        if (COORDS) {
            uint64_t key = lbest > 0 ? ((uint64_t)lbest << 32) | ((uint64_t)(32767 - li) << 15) | (uint64_t)(32767 - lj)
                                     : 0ull;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const uint64_t o = __shfl_xor(key, off, 64);
                key = o > key ? o : key;
            }
            if (lane == 0) {
                const int32_t sc = (int32_t)(key >> 32);
                p.score[outi] = sc;
                p.end_i[outi] = (int16_t)(sc > 0 ? 32767 - (int32_t)((key >> 15) & 0x7FFF) : -1);
                p.end_j[outi] = (int16_t)(sc > 0 ? 32767 - (int32_t)(key & 0x7FFF) : -1);
            }
        } else {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) lbest = max(lbest, __shfl_xor(lbest, off, 64));
            if (lane == 0) {
                p.score[outi] = lbest;
                if (p.end_i) {
                    p.end_i[outi] = -1;
                    p.end_j[outi] = -1;
                }
            }
        }
    }
}

template <int R>
hipError_t go(const SwParams& p, bool affine, bool coords, uint32_t blocks, size_t shm, hipStream_t stream) {
    const dim3 grid(blocks), block(64);
    if (affine) {
        if (coords) hipLaunchKernelGGL((sw_long_kernel<R, true, true>), grid, block, shm, stream, p);
        else hipLaunchKernelGGL((sw_long_kernel<R, true, false>), grid, block, shm, stream, p);
    } else {
        if (coords) hipLaunchKernelGGL((sw_long_kernel<R, false, true>), grid, block, shm, stream, p);
        else hipLaunchKernelGGL((sw_long_kernel<R, false, false>), grid, block, shm, stream, p);
    }
    return hipGetLastError();
}

template <int R>
int resident(bool affine, bool coords, size_t shm) {
    int nb = 0;
    hipError_t e;
    if (affine)
        e = coords ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sw_long_kernel<R, true, true>, 64, shm)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sw_long_kernel<R, true, false>, 64, shm);
    else
        e = coords ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sw_long_kernel<R, false, true>, 64, shm)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sw_long_kernel<R, false, false>, 64, shm);
    return e == hipSuccess && nb > 0 ? nb : 1;
}

}  // namespace

int long_blocks_per_cu(bool affine, bool coords, uint32_t max_read_len, uint32_t max_win_len) {
    const size_t shm = long_lds_bytes(max_win_len);
    switch (long_rows_per_lane(max_read_len)) {
        case 1: return resident<1>(affine, coords, shm);
        case 2: return resident<2>(affine, coords, shm);
        case 3: return resident<3>(affine, coords, shm);
        case 4: return resident<4>(affine, coords, shm);
        case 5: return resident<5>(affine, coords, shm);
        case 6: return resident<6>(affine, coords, shm);
        case 7: return resident<7>(affine, coords, shm);
        default: return resident<8>(affine, coords, shm);
    }
}

int long_rows_per_lane(uint32_t max_read_len) {
    // as few strips of <= 64 * kLongMaxR rows as the longest read needs, its
    // rows spread evenly over them: 600 rows -> two strips of 320 (R = 5),
    // not 512 + 88, which also fits a 300-row read into one strip at 94 %.
    // (Bucketing long pairs by their own R measured slower: one launch per
    // R leaves each launch too few waves, tools/long_bench.py mixed case.)
    const uint32_t m = max_read_len ? max_read_len : 1u;
    const uint32_t strips = (m + 64u * kLongMaxR - 1) / (64u * kLongMaxR);
    const uint32_t r = (m + 64u * strips - 1) / (64u * strips);
    return r < 1 ? 1 : (r > (uint32_t)kLongMaxR ? kLongMaxR : (int)r);
}

// lane 0 loads columns up to n + 125 (the drain's 64-column blocks)
uint32_t long_scratch_cols(uint32_t max_win_len) { return ((max_win_len + 63u) & ~63u) + 128u; }

size_t long_lds_bytes(uint32_t max_win_len) { return (size_t)((max_win_len + 128u + 15u) & ~15u); }

hipError_t launch_sw_long(const SwParams& p, bool affine, bool coords, uint32_t max_read_len, uint32_t max_win_len,
                          uint32_t blocks, hipStream_t stream) {
    if (p.n_slots == 0 || blocks == 0) return hipSuccess;
    if (max_read_len > (uint32_t)kMaxLongLen || max_win_len > (uint32_t)kMaxLongLen) return hipErrorInvalidValue;
    const int r = long_rows_per_lane(max_read_len);
    // more than one strip needs the boundary rows
    if (max_read_len > 64u * (uint32_t)r && (!p.long_scratch || p.long_cols < long_scratch_cols(max_win_len)))
        return hipErrorInvalidValue;
    const size_t shm = long_lds_bytes(max_win_len);
    switch (r) {
        case 1: return go<1>(p, affine, coords, blocks, shm, stream);
        case 2: return go<2>(p, affine, coords, blocks, shm, stream);
        case 3: return go<3>(p, affine, coords, blocks, shm, stream);
        case 4: return go<4>(p, affine, coords, blocks, shm, stream);
        case 5: return go<5>(p, affine, coords, blocks, shm, stream);
        case 6: return go<6>(p, affine, coords, blocks, shm, stream);
        case 7: return go<7>(p, affine, coords, blocks, shm, stream);
        default: return go<8>(p, affine, coords, blocks, shm, stream);
    }
}

}  // namespace msw
