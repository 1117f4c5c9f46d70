// msw_kernels.hip -- hand-written gfx950 kernels for batched Smith-Waterman.
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
//  - One wave64 = 4 lane groups of 16 (one DPP row each).  A group scores TWO
//    pairs at once: pair "a" in the low 16 bits and pair "b" in the high 16
//    bits of every register, so each packed-u16 VALU op updates two cells.
//  - Lane l of a group owns read rows [l*KR, l*KR+KR) in VGPRs and sweeps the
//    window with a one-column skew per lane (anti-diagonal wavefront): at step
//    t lane l scores column t-l, reading that column's packed window code from
//    an LDS stream.  Lane l-1's bottom-row values enter through DPP row_shr:1
//    with bound_ctrl zero fill, which is the zero top boundary for lane 0.
//  - Cell values are small non-negative integers kept as u16; the three-way max
//    runs as v_pk_maximum3_f16 on their (denormal, ordered) f16 bit patterns,
//    and the zero floor comes from u16 saturating subtracts.
//  - Padding (rows past a read, columns past a window, the wavefront's
//    fill/drain columns) uses sentinel codes that mismatch everything, so no
//    per-cell masking is needed: such cells never reach the pair's score.
#include "msw_kernels.h"

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
// DPP row_shr:1 inside each 16-lane row; lane 0 of the row reads 0 (bound_ctrl),
// which is exactly the matrix's zero top boundary for E, F, G and H.
__device__ __forceinline__ uint32_t shr1_zero(uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)src, 0x111, 0xF, 0xF, true);
}

struct PairMeta {
    uint32_t pa, pb;  // pair indices (meaningful only when va / vb)
    bool va, vb;
    int ma, mb, na, nb;
};

__device__ __forceinline__ PairMeta load_meta(const SwParams& p, uint32_t slot_a) {
    PairMeta q;
    const uint32_t slot_b = slot_a + 1;
    q.va = slot_a < p.n_slots;
    q.vb = slot_b < p.n_slots;
    q.pa = q.va ? (p.order ? p.order[slot_a] : slot_a) : 0u;
    q.pb = q.vb ? (p.order ? p.order[slot_b] : slot_b) : 0u;
    q.ma = q.va ? (int)p.read_len[q.pa] : 0;
    q.mb = q.vb ? (int)p.read_len[q.pb] : 0;
    q.na = q.va ? (int)p.win_len[q.pa] : 0;
    q.nb = q.vb ? (int)p.win_len[q.pb] : 0;
    return q;
}

__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
    return v;
}

// Packed window stream of this lane group in LDS:
// stream[kLead + c] = code(win_a[c]) | code(win_b[c]) << 16 for column c,
// sentinels in front (the wavefront's fill columns) and past each window.
__device__ __forceinline__ void stage_window(const SwParams& p, const PairMeta& q, uint32_t* stream,
                                             int steps, int lg) {
    const uint8_t* wa = p.wins + (uint64_t)q.pa * p.win_stride;
    const uint8_t* wb = p.wins + (uint64_t)q.pb * p.win_stride;
    stream[lg] = kWinSentinel2;
    for (int c = lg; c < steps; c += kGroupLanes) {
        const uint32_t ca = c < q.na ? ((uint32_t)wa[c] << p.code_shift) : kWinSentinel;
        const uint32_t cb = c < q.nb ? ((uint32_t)wb[c] << p.code_shift) : kWinSentinel;
        stream[kLead + c] = ca | (cb << 16);
    }
}

template <int KR>
__device__ __forceinline__ void load_read_codes(const SwParams& p, const PairMeta& q, int lg,
                                                uint32_t (&rc)[KR]) {
    const uint8_t* ra = p.reads + (uint64_t)q.pa * p.read_stride;
    const uint8_t* rb = p.reads + (uint64_t)q.pb * p.read_stride;
#pragma unroll
    for (int r = 0; r < KR; ++r) {
        const int i = lg * KR + r;
        const uint32_t ca = i < q.ma ? ((uint32_t)ra[i] << p.code_shift) : kReadSentinel;
        const uint32_t cb = i < q.mb ? ((uint32_t)rb[i] << p.code_shift) : kReadSentinel;
        rc[r] = ca | (cb << 16);
    }
}

__device__ __forceinline__ uint32_t group_pk_max(uint32_t v) {
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) v = pk_max(v, (uint32_t)__shfl_xor((int)v, off, kGroupLanes));
    return v;
}

// Best-cell key: score in the high word, (0xFFFF - i, 0xFFFF - j) in the low
// word, so the max key is max score, then smallest i, then smallest j -- the
// oracle's row-major scan with strict '>'.
__device__ __forceinline__ uint64_t group_max_u64(uint64_t v) {
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(v, off, kGroupLanes);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ void store_score(const SwParams& p, bool valid, uint32_t pair, uint32_t s) {
    if (valid) p.score[pair] = (int32_t)s;
}

__device__ __forceinline__ void store_hit(const SwParams& p, bool valid, uint32_t pair, uint64_t key) {
    if (!valid) return;
    const uint32_t s = (uint32_t)(key >> 32);
    p.score[pair] = (int32_t)s;
    if (p.end_i) {
        const uint32_t lo = (uint32_t)key;
        p.end_i[pair] = s ? (int16_t)(0xFFFFu - (lo >> 16)) : (int16_t)-1;
        p.end_j[pair] = s ? (int16_t)(0xFFFFu - (lo & 0xFFFFu)) : (int16_t)-1;
    }
}

// Per-row keys (h << 16 | 0xFFFF - j, one per packed half) -> group best hits.
template <int KR>
__device__ __forceinline__ void finish_coords(const SwParams& p, const PairMeta& q, int lg,
                                              const uint32_t (&key_a)[KR], const uint32_t (&key_b)[KR]) {
    uint64_t ga = 0, gb = 0;
#pragma unroll
    for (int r = 0; r < KR; ++r) {
        const uint64_t ni = 0xFFFFu - (uint32_t)(lg * KR + r);
        const uint64_t ka = ((uint64_t)(key_a[r] >> 16) << 32) | (ni << 16) | (key_a[r] & 0xFFFFu);
        const uint64_t kb = ((uint64_t)(key_b[r] >> 16) << 32) | (ni << 16) | (key_b[r] & 0xFFFFu);
        ga = ka > ga ? ka : ga;
        gb = kb > gb ? kb : gb;
    }
    ga = group_max_u64(ga);
    gb = group_max_u64(gb);
    if (lg == 0) {
        store_hit(p, q.va, q.pa, ga);
        store_hit(p, q.vb, q.pb, gb);
    }
}

// ---------------------------------------------------------------------------
// Linear gap.  Per packed cell pair (two pairs, same (i, j)):
//   a  = min(rc ^ w, delta)        substitution penalty, 0 or match-mismatch
//   t1 = sat(DG - a)               DG = H_diag + match, so t1 = max(H_diag + s, 0)
//   h  = max3(t1, E_left, E_up)    E = sat(H - gap)
//   E  = sat(h - gap); DG(next row, next column) = h + match
// All t1 of a step are formed first (they only read last step's values), so
// the H+match of row r can land in the register row r+1 just consumed.
// ---------------------------------------------------------------------------
template <int KR, bool COORDS>
__global__ __launch_bounds__(64) void sw_linear_kernel(SwParams p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int lane = threadIdx.x;
    const int g = lane >> 4, lg = lane & 15;
    const PairMeta q = load_meta(p, blockIdx.x * (uint32_t)kPairsPerWave + 2u * g);
    const int steps = __builtin_amdgcn_readfirstlane(wave_max_i32(max(q.na, q.nb))) + kGroupLanes - 1;
    uint32_t* stream = lds + g * p.lds_stride;
    stage_window(p, q, stream, steps, lg);
    uint32_t rc[KR];
    load_read_codes<KR>(p, q, lg, rc);
    __syncthreads();

    const uint32_t match2 = p.match2, delta2 = p.delta2, gap2 = p.gap2;
    uint32_t E[KR], DG[KR];
    uint32_t key_a[KR], key_b[KR];
#pragma unroll
    for (int r = 0; r < KR; ++r) { E[r] = 0u; DG[r] = match2; key_a[r] = 0u; key_b[r] = 0u; }
    uint32_t e_bot = 0u, h_bot = 0u, d_up_prev = match2;
    uint32_t best = 0u;
    // lane lg reads column t - lg: stream index kLead + t - lg (kLead sentinels in front)
    const uint32_t* wp = stream + (kLead - lg);

    uint32_t w_next = wp[0];  // one step of LDS lookahead
    for (int t = 0; t < steps; ++t) {
        const uint32_t w = w_next;
        w_next = wp[t + 1];
        const uint32_t e_up = shr1_zero(e_bot);
        const uint32_t d_up = shr1_zero(h_bot) + match2;   // v_add_u32_dpp; lane 0 -> 0 + match
        DG[0] = d_up_prev;
        uint32_t t1[KR];
#pragma unroll
        for (int r = 0; r < KR; ++r) t1[r] = pk_satsub(DG[r], pk_min(rc[r] ^ w, delta2));
        const uint32_t nj = COORDS ? ((uint32_t)(0xFFFF + lg - t) & 0xFFFFu) : 0u;
        uint32_t up = e_up, hprev = 0u;
#pragma unroll
        for (int r = 0; r < KR; ++r) {
            const uint32_t h = pk_max3(t1[r], E[r], up);
            up = E[r] = pk_satsub(h, gap2);
            if (r + 1 < KR) DG[r + 1] = pk_add(h, match2);
            else h_bot = h;
            if constexpr (COORDS) {
                key_a[r] = max(key_a[r], (h << 16) | nj);
                key_b[r] = max(key_b[r], (h & 0xFFFF0000u) | nj);
            } else {
                if (r & 1) best = pk_max3(best, hprev, h);
                else if (r + 1 == KR) best = pk_max(best, h);
                hprev = h;
            }
        }
        e_bot = E[KR - 1];
        d_up_prev = d_up;
    }

    if constexpr (COORDS) {
        finish_coords<KR>(p, q, lg, key_a, key_b);
    } else {
        best = group_pk_max(best);
        if (lg == 0) {
            store_score(p, q.va, q.pa, best & 0xFFFFu);
            store_score(p, q.vb, q.pb, best >> 16);
        }
    }
}

// ---------------------------------------------------------------------------
// Affine gap (Gotoh), values floored at 0 (identical H: DESIGN.md proof).
//   E  = max(sat(E_left - ge), G_left)      G = sat(H - go - ge)
//   F  = max(sat(F_up - ge),   G_up)
//   h  = max3(sat(DG - a), E, F)
//   G  = sat(h - go - ge); DG(next row, next column) = h + match
// ---------------------------------------------------------------------------
template <int KR, bool COORDS>
__global__ __launch_bounds__(64) void sw_affine_kernel(SwParams p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int lane = threadIdx.x;
    const int g = lane >> 4, lg = lane & 15;
    const PairMeta q = load_meta(p, blockIdx.x * (uint32_t)kPairsPerWave + 2u * g);
    const int steps = __builtin_amdgcn_readfirstlane(wave_max_i32(max(q.na, q.nb))) + kGroupLanes - 1;
    uint32_t* stream = lds + g * p.lds_stride;
    stage_window(p, q, stream, steps, lg);
    uint32_t rc[KR];
    load_read_codes<KR>(p, q, lg, rc);
    __syncthreads();

    const uint32_t match2 = p.match2, delta2 = p.delta2, ext2 = p.gap2, oe2 = p.open_ext2;
    uint32_t E[KR], G[KR], DG[KR];
    uint32_t key_a[KR], key_b[KR];
#pragma unroll
    for (int r = 0; r < KR; ++r) { E[r] = 0u; G[r] = 0u; DG[r] = match2; key_a[r] = 0u; key_b[r] = 0u; }
    uint32_t f_bot = 0u, g_bot = 0u, h_bot = 0u, d_up_prev = match2;
    uint32_t best = 0u;
    const uint32_t* wp = stream + (kLead - lg);

    uint32_t w_next = wp[0];  // one step of LDS lookahead
    for (int t = 0; t < steps; ++t) {
        const uint32_t w = w_next;
        w_next = wp[t + 1];
        uint32_t f = shr1_zero(f_bot);
        uint32_t g_up = shr1_zero(g_bot);
        const uint32_t d_up = shr1_zero(h_bot) + match2;
        DG[0] = d_up_prev;
        uint32_t t1[KR];
#pragma unroll
        for (int r = 0; r < KR; ++r) t1[r] = pk_satsub(DG[r], pk_min(rc[r] ^ w, delta2));
        const uint32_t nj = COORDS ? ((uint32_t)(0xFFFF + lg - t) & 0xFFFFu) : 0u;
        uint32_t hprev = 0u;
#pragma unroll
        for (int r = 0; r < KR; ++r) {
            const uint32_t e = pk_max(pk_satsub(E[r], ext2), G[r]);
            f = pk_max(pk_satsub(f, ext2), g_up);
            const uint32_t h = pk_max3(t1[r], e, f);
            E[r] = e;
            g_up = G[r] = pk_satsub(h, oe2);
            if (r + 1 < KR) DG[r + 1] = pk_add(h, match2);
            else h_bot = h;
            if constexpr (COORDS) {
                key_a[r] = max(key_a[r], (h << 16) | nj);
                key_b[r] = max(key_b[r], (h & 0xFFFF0000u) | nj);
            } else {
                if (r & 1) best = pk_max3(best, hprev, h);
                else if (r + 1 == KR) best = pk_max(best, h);
                hprev = h;
            }
        }
        f_bot = f;
        g_bot = G[KR - 1];
        d_up_prev = d_up;
    }

    if constexpr (COORDS) {
        finish_coords<KR>(p, q, lg, key_a, key_b);
    } else {
        best = group_pk_max(best);
        if (lg == 0) {
            store_score(p, q.va, q.pa, best & 0xFFFFu);
            store_score(p, q.vb, q.pb, best >> 16);
        }
    }
}

// ---------------------------------------------------------------------------
// smith_waterman_align (smith_waterman.cl:11-71) restated.  Work item (g, t)
// of the reference NDRange runs a Kadane scan (cur = max(cur + s, 0)) over
// positions g*C + t + k*W < min((g+1)*C, L), s = +2 / -1 (:39-53); the result
// is the max over all work items (work-group reduce + atomic_max, :55-70).
// Items are grid-strided; reduction is wave-level + one atomicMax per wave.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sw_compat_kernel(const uint8_t* __restrict__ s1,
                                                        const uint8_t* __restrict__ s2,
                                                        int32_t* result, uint64_t L, uint32_t W,
                                                        uint64_t G) {
    const uint64_t C = (L + G - 1) / G;
    const uint64_t items = G * (uint64_t)W;
    int best = 0;
    for (uint64_t it = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; it < items;
         it += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t g = it / W, t = it - g * W;
        const uint64_t start = g * C;
        if (start >= L) continue;
        const uint64_t end = min(start + C, L);
        int cur = 0;
        for (uint64_t pos = start + t; pos < end; pos += W) {
            cur = max(cur + (s1[pos] == s2[pos] ? 2 : -1), 0);
            best = max(best, cur);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) best = max(best, __shfl_xor(best, off, 64));
    if ((threadIdx.x & 63) == 0 && best > 0) atomicMax(result, best);
}

// ---------------------------------------------------------------------------
// Launchers.
// ---------------------------------------------------------------------------
template <int KR>
static hipError_t launch_kr(const SwParams& p, bool affine, bool coords, hipStream_t stream) {
    const dim3 grid((p.n_slots + kPairsPerWave - 1) / kPairsPerWave), block(64);
    const size_t shm = lds_bytes(p.lds_stride);
    if (affine) {
        if (coords) hipLaunchKernelGGL((sw_affine_kernel<KR, true>), grid, block, shm, stream, p);
        else hipLaunchKernelGGL((sw_affine_kernel<KR, false>), grid, block, shm, stream, p);
    } else {
        if (coords) hipLaunchKernelGGL((sw_linear_kernel<KR, true>), grid, block, shm, stream, p);
        else hipLaunchKernelGGL((sw_linear_kernel<KR, false>), grid, block, shm, stream, p);
    }
    return hipGetLastError();
}

hipError_t launch_sw(const SwParams& p, bool affine, bool coords, uint32_t max_read_len,
                     hipStream_t stream) {
    if (p.n_slots == 0) return hipSuccess;
    switch (rows_per_lane(max_read_len)) {
        case 1: return launch_kr<1>(p, affine, coords, stream);
        case 2: return launch_kr<2>(p, affine, coords, stream);
        case 3: return launch_kr<3>(p, affine, coords, stream);
        case 4: return launch_kr<4>(p, affine, coords, stream);
        case 5: return launch_kr<5>(p, affine, coords, stream);
        case 6: return launch_kr<6>(p, affine, coords, stream);
        case 7: return launch_kr<7>(p, affine, coords, stream);
        case 8: return launch_kr<8>(p, affine, coords, stream);
        case 9: return launch_kr<9>(p, affine, coords, stream);
        case 10: return launch_kr<10>(p, affine, coords, stream);
        case 11: return launch_kr<11>(p, affine, coords, stream);
        case 12: return launch_kr<12>(p, affine, coords, stream);
        case 13: return launch_kr<13>(p, affine, coords, stream);
        case 14: return launch_kr<14>(p, affine, coords, stream);
        case 15: return launch_kr<15>(p, affine, coords, stream);
        case 16: return launch_kr<16>(p, affine, coords, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_compat(const uint8_t* s1, const uint8_t* s2, int32_t* result, uint64_t L,
                         uint32_t W, uint64_t G, hipStream_t stream) {
    const uint64_t items = G * (uint64_t)W;
    uint64_t blocks = (items + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(sw_compat_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, s1, s2, result,
                       L, W, G);
    return hipGetLastError();
}

}  // namespace msw
