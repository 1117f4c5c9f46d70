// msw_kernels.hip -- launch dispatch of the gfx950 Smith-Waterman kernels,
// plus the two small kernels (compat restatement, window cut).
//
// The SW kernel templates live in msw_device.h; their instance set is split
// over the msw_launch_*.hip translation units (pairs linear / pairs affine /
// split / mixed / multi linear / multi affine) so hipcc builds them in
// parallel.  launch_sw / launch_sw_multi below pick the unit and instance.
#include <algorithm>
#include "msw_device.h"
#include "msw_launch.h"

namespace msw {

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
// Window cut for genome-resident batches (msw_align_reads,
// msw_genome_cut_device): pair p's window genome[pos[p], pos[p] + len) with
// len = want[p] clipped at the genome end (0 outside it) and at ws -> out[p * ws ..],
// zero-padded to ws; out_len[p] = len when out_len is given.  One thread per
// 16-byte output chunk: five aligned dword loads, v_alignbyte to the window's
// byte offset, one 16-byte store (consecutive threads write consecutive
// chunks of a row).  The genome allocation is padded by >= 20 bytes, so the
// fifth dword never leaves it.  HBM-bound: ~2 bytes moved per window byte.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cut_windows_kernel(const uint8_t* __restrict__ g, uint64_t glen,
                                                          const int64_t* __restrict__ pos,
                                                          const uint16_t* __restrict__ want,
                                                          const uint16_t* __restrict__ rlen, uint32_t window,
                                                          uint8_t* __restrict__ out, uint16_t* __restrict__ out_len,
                                                          uint32_t chunks, uint64_t ws, uint64_t n) {
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t p = t / chunks;
    if (p >= n) return;
    const uint32_t c = (uint32_t)(t - p * chunks);
    const uint64_t start = (uint64_t)pos[p];  // negative positions wrap past glen
    const uint64_t room = start < glen ? glen - start : 0;
    // requested length: want[p], or (device-resident reads) --window / 2 x read length (capped)
    const uint64_t wl = want ? want[p] : (window ? window : min(2u * rlen[p], (uint32_t)kMaxWinLen));
    const int len = (int)min(min(wl, room), ws);
    if (out_len && c == 0) out_len[p] = (uint16_t)len;
    const int rem = len - 16 * (int)c;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (rem > 0) {
        const uint64_t a = start + 16u * c;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(g + (a & ~3ull));
        uint32_t x[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) x[k] = src[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t v = __builtin_amdgcn_alignbyte(x[k + 1], x[k], (uint32_t)(a & 3u));
            const int nb = rem - 4 * k;
            w[k] = nb >= 4 ? v : (nb > 0 ? v & ((1u << (8 * nb)) - 1u) : 0u);
        }
    }
    *reinterpret_cast<uint4*>(out + p * ws + 16ull * c) = make_uint4(w[0], w[1], w[2], w[3]);
}


// ---------------------------------------------------------------------------
// Pair order from slot order (planned length-bucketed launches).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gather_results_kernel(const uint32_t* __restrict__ inv,
                                                             const int32_t* __restrict__ src_score,
                                                             const int16_t* __restrict__ src_i,
                                                             const int16_t* __restrict__ src_j,
                                                             int32_t* __restrict__ score, int16_t* __restrict__ end_i,
                                                             int16_t* __restrict__ end_j, uint64_t n) {
    const uint64_t k = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (k >= n) return;
    const uint32_t s = inv[k];
    score[k] = src_score[s];
    if (end_i) {
        end_i[k] = src_i[s];
        end_j[k] = src_j[s];
    }
}

// ---------------------------------------------------------------------------
// Device -> pinned host copy on the caller's stream (msw_memcpy_d2h_async):
// 16-byte vector loads and stores over the body when source and destination
// share their alignment mod 16, bytes for the head and tail (or everything
// when they do not).  Plain vector stores over PCIe.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void d2h_copy_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                       uint64_t bytes, uint64_t head, uint64_t body16) {
    const uint64_t tid = (uint64_t)blockIdx.x * 256u + threadIdx.x, nth = (uint64_t)gridDim.x * 256u;
    uint4* d4 = reinterpret_cast<uint4*>(dst + head);
    const uint4* s4 = reinterpret_cast<const uint4*>(src + head);
    for (uint64_t k = tid; k < body16; k += nth) d4[k] = s4[k];
    const uint64_t tail0 = head + 16u * body16, rest = head + (bytes - tail0);
    for (uint64_t i = tid; i < rest; i += nth) {
        const uint64_t b = i < head ? i : tail0 + (i - head);
        dst[b] = src[b];
    }
}

// The ranges of a one-chunk host call, host memory -> HBM (launch_pull_copy):
// 16-byte loads over PCIe, grid-stride per range.
__global__ __launch_bounds__(256) void pull_copy_kernel(PullRanges r) {
    const uint64_t tid = (uint64_t)blockIdx.x * 256u + threadIdx.x, nth = (uint64_t)gridDim.x * 256u;
#pragma unroll
    for (int k = 0; k < kPullRanges; ++k) {
        uint8_t* d = r.dst[k];
        const uint8_t* s = r.src[k];
        const uint64_t bytes = r.bytes[k];
        const uint64_t head = std::min<uint64_t>(bytes, (16u - ((uintptr_t)d & 15u)) & 15u);
        const uint64_t body = (bytes - head) >> 4;
        uint4* d4 = reinterpret_cast<uint4*>(d + head);
        const uint4* s4 = reinterpret_cast<const uint4*>(s + head);
        for (uint64_t i = tid; i < body; i += nth) d4[i] = s4[i];
        const uint64_t tail0 = head + 16u * body, rest = head + (bytes - tail0);
        for (uint64_t i = tid; i < rest; i += nth) {
            const uint64_t b = i < head ? i : tail0 + (i - head);
            d[b] = s[b];
        }
    }
}

// ---------------------------------------------------------------------------
// Dispatch.
// ---------------------------------------------------------------------------
thread_local int* t_occupancy = nullptr;

int sw_blocks_per_cu(const SwParams& p, bool affine, bool coords, uint32_t max_read_len, Layout layout) {
    int nb = 0;
    t_occupancy = &nb;
    const hipError_t e = launch_sw(p, affine, coords, max_read_len, layout, nullptr);
    t_occupancy = nullptr;
    return e == hipSuccess ? nb : 0;
}

int sw_multi_blocks_per_cu(const SwParams& p, const MultiTable& t, bool affine, bool coords) {
    int nb = 0;
    t_occupancy = &nb;
    const hipError_t e = launch_sw_multi(p, t, affine, coords, nullptr);
    t_occupancy = nullptr;
    return e == hipSuccess ? nb : 0;
}

int cut_blocks_per_cu() {
    int nb = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, cut_windows_kernel, 256, 0) == hipSuccess ? nb : 0;
}

hipError_t launch_sw(const SwParams& p, bool affine, bool coords, uint32_t max_read_len, Layout layout,
                     hipStream_t stream) {
    if (p.n_slots == 0) return hipSuccess;
    if (p.win_src) {  // genome windows: pairs layout, KR <= 16 only (the runtime checks with genome_layout_ok)
        const int kr = rows_per_lane(max_read_len, false, p.group_lanes);
        if (layout != Layout::kPairs || kr < 1 || kr > 16) return hipErrorInvalidValue;
        return affine ? launch_genome_aff(p, coords, kr, stream) : launch_genome_lin(p, coords, kr, stream);
    }
    if (layout == Layout::kMixed) {
        const uint32_t rest = p.n_slots - min(p.n_slots, p.pairs_blocks * pairs_per_wave(false, p.groups));
        const uint32_t blocks = p.pairs_blocks + (rest + p.groups - 1) / p.groups;
        const int krp = rows_per_lane(max_read_len, false, p.group_lanes);
        if (krp % 2 != 0 || krp > 16) return hipErrorInvalidValue;  // odd KR: caller picks pairs/split
        return launch_mixed(p, affine, coords, krp, blocks, stream);
    }
    if (layout == Layout::kSplit) {
        const int kr = rows_per_lane(max_read_len, true, p.group_lanes);
        if (kr < 1 || kr > 8) return hipErrorInvalidValue;
        return launch_split(p, affine, coords, kr, stream);
    }
    const int kr = rows_per_lane(max_read_len, false, p.group_lanes);
    if (kr < 1 || kr > kMaxRowsPerLane) return hipErrorInvalidValue;
    if (kr > 16) return launch_pairs_wide(p, affine, coords, kr, stream);
    return affine ? launch_pairs_aff(p, coords, kr, stream) : launch_pairs_lin(p, coords, kr, stream);
}

hipError_t launch_sw_multi(const SwParams& p, const MultiTable& t, bool affine, bool coords,
                           hipStream_t stream) {
    if (t.n_buckets == 0) return hipSuccess;
    if (!p.order || t.n_buckets > (uint32_t)kMaxBuckets || p.group_lanes != 16 || p.groups != 4)
        return hipErrorInvalidValue;
    // one table is all KR <= 16 buckets or all KR 17..24 (the wide instance)
    const bool wide = t.kr[0] > (uint32_t)kMaxMultiKR;
    uint32_t stride = 0;
    for (uint32_t b = 0; b < t.n_buckets; ++b) {
        const bool ok = wide ? t.kr[b] > (uint32_t)kMaxMultiKR && t.kr[b] <= (uint32_t)kMaxRowsPerLane
                             : t.kr[b] >= 1 && t.kr[b] <= (uint32_t)kMaxMultiKR;
        if (!ok) return hipErrorInvalidValue;
        stride = max(stride, t.lds_stride[b]);
    }
    const uint32_t grid = t.block_end[t.n_buckets - 1];
    const size_t shm = lds_bytes(stride, p.groups);
    if (wide) return launch_multi_wide(p, t, affine, coords, grid, shm, stream);
    return affine ? launch_multi_aff(p, t, coords, grid, shm, stream) : launch_multi_lin(p, t, coords, grid, shm, stream);
}

hipError_t launch_cut_windows(const uint8_t* genome, uint64_t glen, const int64_t* pos, const uint16_t* want,
                              uint8_t* out, uint16_t* out_len, uint32_t ws, uint64_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (ws == 0 || ws % 16 != 0 || ((uintptr_t)out & 15) != 0) return hipErrorInvalidValue;
    const uint32_t chunks = ws / 16;
    const uint64_t blocks = (n * chunks + 255) / 256;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(cut_windows_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, genome, glen, pos, want,
                       (const uint16_t*)nullptr, 0u, out, out_len, chunks, (uint64_t)ws, n);
    return hipGetLastError();
}

hipError_t launch_cut_windows_for_reads(const uint8_t* genome, uint64_t glen, const int64_t* pos,
                                        const uint16_t* rlen, uint32_t window, uint8_t* out, uint16_t* out_len,
                                        uint32_t ws, uint64_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (ws == 0 || ws % 16 != 0 || ((uintptr_t)out & 15) != 0) return hipErrorInvalidValue;
    const uint32_t chunks = ws / 16;
    const uint64_t blocks = (n * chunks + 255) / 256;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(cut_windows_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, genome, glen, pos,
                       (const uint16_t*)nullptr, rlen, window, out, out_len, chunks, (uint64_t)ws, n);
    return hipGetLastError();
}

hipError_t launch_gather_results(const uint32_t* inv, const int32_t* src_score, const int16_t* src_i,
                                 const int16_t* src_j, int32_t* score, int16_t* end_i, int16_t* end_j, uint64_t n,
                                 hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n + 255) / 256;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gather_results_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, inv, src_score, src_i,
                       src_j, score, end_i, end_j, n);
    return hipGetLastError();
}

hipError_t launch_d2h_copy(void* dst, const void* src, uint64_t bytes, hipStream_t stream) {
    if (bytes == 0) return hipSuccess;
    const uintptr_t ad = (uintptr_t)dst, as = (uintptr_t)src;
    uint64_t head = bytes, body16 = 0;
    if ((ad & 15) == (as & 15)) {
        head = std::min<uint64_t>(bytes, (16 - (ad & 15)) & 15);
        body16 = (bytes - head) / 16;
    }
    const uint64_t work = std::max<uint64_t>(body16, head + (bytes - head - 16 * body16));
    const uint64_t blocks = std::min<uint64_t>(1024, std::max<uint64_t>(1, (work + 255) / 256));
    hipLaunchKernelGGL(d2h_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (uint8_t*)dst, (const uint8_t*)src,
                       bytes, head, body16);
    return hipGetLastError();
}

hipError_t launch_pull_copy(const PullRanges& r, hipStream_t stream) {
    uint64_t most = 0;
    for (int k = 0; k < kPullRanges; ++k) most = std::max(most, r.bytes[k] >> 4);
    // ~4 loads in flight per thread of the largest range, at most 512 blocks
    // (the PCIe link, not the CUs, bounds it; the call's scoring kernel and
    // the other stream's share the CUs)
    const uint64_t blocks = std::min<uint64_t>(512, std::max<uint64_t>(1, (most + 1023) / 1024));
    hipLaunchKernelGGL(pull_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, r);
    return hipGetLastError();
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
