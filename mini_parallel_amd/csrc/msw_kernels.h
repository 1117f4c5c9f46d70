// msw_kernels.h -- device-side parameter block and launchers (internal).
#pragma once
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
constexpr int kMaxReadLen = 256;       // KR <= 16
constexpr int kMaxWinLen = 4096;
constexpr int kLead = 16;              // sentinel words in front of each window stream

// u32 words per lane-group stream: kLead + (max_win + 15) steps, rounded so that
// the four groups of a wave start 16 banks apart (stride == 16 mod 32).
inline uint32_t stream_stride(uint32_t max_win_len) {
    uint32_t words = kLead + max_win_len + kGroupLanes - 1;
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
    uint32_t match2;          // match, duplicated into both u16 halves
    uint32_t delta2;          // match - mismatch
    uint32_t gap2;            // linear: gap penalty; affine: gap_extend
    uint32_t open_ext2;       // affine: gap_open + gap_extend
};

// Rows per lane for a read-length bound (ceil(m / 16), at least 1).
inline int rows_per_lane(uint32_t max_read_len) {
    int kr = (int)((max_read_len + kGroupLanes - 1) / kGroupLanes);
    return kr < 1 ? 1 : kr;
}

// Dynamic LDS bytes for one 64-lane block.
inline size_t lds_bytes(uint32_t lds_stride) { return 4u * (size_t)lds_stride * sizeof(uint32_t); }

hipError_t launch_sw(const SwParams& p, bool affine, bool coords, uint32_t max_read_len,
                     hipStream_t stream);

// smith_waterman_align restated: result must be zeroed before the launch.
hipError_t launch_compat(const uint8_t* s1, const uint8_t* s2, int32_t* result, uint64_t L,
                         uint32_t W, uint64_t G, hipStream_t stream);

}  // namespace msw
